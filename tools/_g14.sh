#!/bin/bash
# round 4: code act v4 with slices >= 2 staged inside layer 0 -- parity, A/B timing, stamps
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "code or qnet or dqn or train_loop" > gpurun_out/g14_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g14_tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g14_act.log 2>&1 || exit 1
  timeout -k 10 120 python tools/time_act.py --lib tools/var_nodma.so --precision f32 --input code >> gpurun_out/g14_act.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 >> gpurun_out/g14_act.log 2>&1 || exit 1
timeout -k 10 120 python tools/time_act.py --lib tools/var_nodma.so --precision f32 --input code --envs 131072 >> gpurun_out/g14_act.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g14_act.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps --slices 10 > gpurun_out/g14_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g14_stamps.log
