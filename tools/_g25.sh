#!/bin/bash
# round 4: C3 / C4 reset, lane-per-env kernel against the wave-per-env default
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python tools/reset_rate.py --configs c3,c4 --variants wave,lane > gpurun_out/g25_reset.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g25_reset.log | tail -20
