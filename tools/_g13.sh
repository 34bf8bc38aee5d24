#!/bin/bash
# round 4: code act v4 -- parity (code / qnet / dqn / fullsize loop), timing at C3 / C5, per-slice stamps
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "code or qnet or dqn or train_loop" > gpurun_out/g13_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g13_tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g13_act.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 >> gpurun_out/g13_act.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g13_act.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps --slices 10 > gpurun_out/g13_stamps.log 2>&1 || exit 1
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps --slices 10 --envs 131072 >> gpurun_out/g13_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g13_stamps.log
