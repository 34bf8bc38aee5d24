#!/bin/bash
# round 4: the last build at its defaults -- the whole GPU suite and smoke
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=_r4d T_TESTS=900 bash tools/gpu.sh tests smoke
