#!/bin/bash
# round 4: code act with the second pass's codes loaded in the prologue -- parity, act alone, train loops (C3, C5)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "code or qnet or dqn or train_loop" > gpurun_out/g24_tests.log 2>&1; rc=$?
tail -2 gpurun_out/g24_tests.log
[ $rc -ne 0 ] && exit $rc
for e in 65536 131072; do
  timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs $e >> gpurun_out/g24_act.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/g24_act.log
for c in c3 c5; do
  timeout -k 10 300 python3 tools/loop_only.py --config $c --segments 3 > gpurun_out/g24_loop_$c.log 2>&1 || exit 1
  grep us_per_step gpurun_out/g24_loop_$c.log
done
mkdir -p gpurun_out/prof_loop3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_loop3/c5 -o run --output-format csv -- python3 tools/loop_only.py --config c5 --segments 3 > gpurun_out/prof_loop3/c5.log 2>&1 || exit 1
grep -h "code4" gpurun_out/prof_loop3/c5/run_kernel_stats.csv
