#!/bin/bash
# round 4: code act v4 -- per-slice layer-0 stamps, no-decode diagnostic
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in prod nodec; do
  case $v in
    prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
    *) timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --precision f32 --input code ;;
  esac >> gpurun_out/g11_act.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/g11_act.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps --slices 10 > gpurun_out/g11_stamps.log 2>&1 || exit 1
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps --slices 10 --envs 131072 >> gpurun_out/g11_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g11_stamps.log
