#!/bin/bash
# round 4: code act v4 knobs (decode pins, early first code vector, MFMA/VALU interleave), interleaved timing
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "qnet_act_code" > gpurun_out/g12_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g12_tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in prod pin early iglp piniglp nodec; do
    case $v in
      prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      *) timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --precision f32 --input code ;;
    esac >> gpurun_out/g12_act.log 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/g12_act.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps --slices 10 > gpurun_out/g12_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g12_stamps.log
