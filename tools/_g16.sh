#!/bin/bash
# round 4 final B: rocprofv3 trace + PMC of the C3 and C5 step loops, kernel trace of the code act (C3, C5)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
CFG=c3 TAG=_c3 bash tools/gpu.sh profile || exit 1
CFG=c5 TAG=_c5 bash tools/gpu.sh profile || exit 1
mkdir -p gpurun_out/prof_act
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_act/c3 -o run --output-format csv -- python3 tools/time_act.py --precision f32 --input code > gpurun_out/prof_act/c3.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_act/c5 -o run --output-format csv -- python3 tools/time_act.py --precision f32 --input code --envs 131072 > gpurun_out/prof_act/c5.log 2>&1 || exit 1
grep -h "us/launch" gpurun_out/prof_act/*.log
