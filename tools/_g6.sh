#!/bin/bash
# round 4: code act -- the 4-tiles-per-wave form (var_act4: one wave per SIMD) parity + timing against the
# product (2 tiles, two waves per SIMD) and round 3's kernel; diagnostics; step stamps at C3 / C5
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
DRL_LIB=tools/var_act4.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "code or qnet" > gpurun_out/g6_act4_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g6_act4_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for r in 1 2; do
  for v in act4 act4pd12 prod code2 pd12 half nomfma; do
    case $v in
      prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      code2) DRL_QN_CODE3=0 timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      *) timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --precision f32 --input code ;;
    esac >> gpurun_out/g6_act.log 2>&1 || exit 1
  done
done
for v in act4 prod code2; do
  case $v in
    prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 ;;
    code2) DRL_QN_CODE3=0 timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 ;;
    *) timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --precision f32 --input code --envs 131072 ;;
  esac >> gpurun_out/g6_act.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/g6_act.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_act4s.so --precision f32 --input code --stamps > gpurun_out/g6_stamps_act4.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g6_stamps_act4.log
timeout -k 10 300 python tools/stamps.py --prebuilt --config c5 --steps 8 > gpurun_out/g6_stamps_c5.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g6_stamps_c5.log
