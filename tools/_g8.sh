#!/bin/bash
# round 4: code act v4 (one wave per SIMD, four tiles per wave): parity of the code/qnet tests, timing against
# v3 / v2 and read-depth variants, per-phase stamps
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "code or qnet or dqn" > gpurun_out/g8_tests.log 2>&1; rc=$?
tail -15 gpurun_out/g8_tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in prod v3; do
    case $v in
      prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      v3) DRL_QN_CODE=3 timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      v2) DRL_QN_CODE=2 timeout -k 10 120 python tools/time_act.py --precision f32 --input code ;;
      *) timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --precision f32 --input code ;;
    esac >> gpurun_out/g8_act.log 2>&1 || exit 1
  done
done
for v in prod v3; do
  case $v in
    prod) timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 ;;
    v3) DRL_QN_CODE=3 timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 ;;
  esac >> gpurun_out/g8_act.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/g8_act.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps > gpurun_out/g8_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g8_stamps.log
