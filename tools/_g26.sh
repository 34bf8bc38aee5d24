#!/bin/bash
# round 4: reset with 2 / 4 waves (envs) per workgroup -- parity of the reset tests on each, then rates
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for w in 2 4; do
  DRL_RESET_WPB=$w timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "reset" > gpurun_out/g26_tests_$w.log 2>&1 || exit 1
  echo "wpb $w: $(tail -1 gpurun_out/g26_tests_$w.log)"
done
for w in 1 2 4 1 2 4; do
  DRL_RESET_WPB=$w timeout -k 10 300 python tools/reset_rate.py --configs c3,c4,c5 --variants wave > gpurun_out/g26_rate_$w.log 2>&1 || exit 1
  grep -v amdgpu gpurun_out/g26_rate_$w.log | sed "s/^/wpb $w /" | tail -3
done
