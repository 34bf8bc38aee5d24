#!/bin/bash
# round 4: code act diagnostics (LDS-light, MFMA-free, read depth) and step stamps at C3 / C5 (packed ground)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2; do
  for v in prod code2 pd12 pd4 half nomfma; do
    case $v in
      prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      code2) DRL_QN_CODE3=0 timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      *) timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --precision f32 --input code ;;
    esac >> gpurun_out/g5_act.log 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/g5_act.log
timeout -k 10 300 python tools/stamps.py --prebuilt --config c5 --steps 8 > gpurun_out/g5_stamps_c5.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g5_stamps_c5.log
timeout -k 10 300 python tools/stamps.py --prebuilt --config c3 --steps 8 > gpurun_out/g5_stamps_c3.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g5_stamps_c3.log
