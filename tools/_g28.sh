#!/bin/bash
# round 4: reset with 8 waves per workgroup at C5 -- parity, then rates against 4
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
DRL_RESET_WPB=8 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "reset" > gpurun_out/g28_tests_8.log 2>&1 || exit 1
echo "wpb 8: $(tail -1 gpurun_out/g28_tests_8.log)"
for w in 4 8 4 8; do
  DRL_RESET_WPB=$w timeout -k 10 300 python tools/reset_rate.py --configs c4,c5 --variants wave > gpurun_out/g28_rate_$w.log 2>&1 || exit 1
  grep -v amdgpu gpurun_out/g28_rate_$w.log | sed "s/^/wpb $w /" | tail -2
done
