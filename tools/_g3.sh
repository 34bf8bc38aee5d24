#!/bin/bash
# round 4: code act v3 -- parity first, then timing against the round-3 kernel, then phase stamps
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "code or qnet or dqn or train_loop" > gpurun_out/g3_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g3_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for r in 1 2; do
  timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g3_time.log 2>&1 || exit 1
  DRL_QN_CODE3=0 timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g3_time.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 >> gpurun_out/g3_time.log 2>&1 || exit 1
DRL_QN_CODE3=0 timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 >> gpurun_out/g3_time.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g3_time.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst3.so --precision f32 --input code --stamps > gpurun_out/g3_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g3_stamps.log
