#!/bin/bash
# round 4: 16-B replay add -- parity (replay / code / dqn / train loop tests), loop timing and kernel trace at C3
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/prof_loop2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "replay or code or dqn or train_loop" > gpurun_out/g21_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g21_tests.log
[ $rc -ne 0 ] && exit $rc
for c in c3 c5; do
  timeout -k 10 300 python3 tools/loop_only.py --config $c --segments 3 > gpurun_out/g21_loop_$c.log 2>&1 || exit 1
  grep us_per_step gpurun_out/g21_loop_$c.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_loop2/c3 -o run --output-format csv -- python3 tools/loop_only.py --config c3 --segments 3 > gpurun_out/prof_loop2/c3.log 2>&1 || exit 1
grep -h "replay" gpurun_out/prof_loop2/c3/run_kernel_stats.csv
