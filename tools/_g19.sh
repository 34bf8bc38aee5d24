#!/bin/bash
# round 4: code act v4 knobs -- layer 1's first split in layer 0's last slice (es), layer-1 MFMA/VALU interleave
# (iglp1), ring depth 8 (pd8): parity of es / esig, interleaved timing
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in es esig; do
  DRL_LIB=tools/var_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "qnet_act_code" > gpurun_out/g19_tests_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/g19_tests_$v.log
done
for r in 1 2 3; do
  for v in prod es iglp1 pd8 esig; do
    case $v in
      prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      *) timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --precision f32 --input code ;;
    esac >> gpurun_out/g19_act.log 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/g19_act.log
