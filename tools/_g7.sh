#!/bin/bash
# round 4: where the code act's time goes -- LDS staging rate of a 160 KB image on every CU
# (tools/stage_probe), the product act against no-staging / no-MFMA builds, per-phase stamps
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 120 tools/stage_probe.bin > gpurun_out/g7_stage.log 2>&1 || exit 1
cat gpurun_out/g7_stage.log
for r in 1 2; do
  for v in prod nostage nomfma; do
    case $v in
      prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      *) timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --precision f32 --input code ;;
    esac >> gpurun_out/g7_act.log 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/g7_act.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst3.so --precision f32 --input code --stamps > gpurun_out/g7_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g7_stamps.log
