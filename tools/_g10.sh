#!/bin/bash
# round 4: staging rate (fixed probe), act stamps at C5 (first vs later passes)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 120 tools/stage_probe.bin > gpurun_out/g10_stage.log 2>&1; rc=$?
cat gpurun_out/g10_stage.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps --envs 131072 > gpurun_out/g10_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g10_stamps.log
