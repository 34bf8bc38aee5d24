#!/bin/bash
# DQN tests (both precisions), then act timing per precision.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dqn.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_dqn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_dqn.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for p in bf16 f32 bf16 f32; do
  timeout -k 10 120 python tools/time_act.py --precision $p >> gpurun_out/time_act.log 2>&1 || exit $?
done
cat gpurun_out/time_act.log
