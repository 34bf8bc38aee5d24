#!/bin/bash
# round 4 final A: the whole GPU suite, smoke, the driver's bench line
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=_r4 T_TESTS=900 bash tools/gpu.sh tests smoke bench
