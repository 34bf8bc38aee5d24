#!/bin/bash
# GPU: DQN tests on the product library, then act timing A/B: the product
# build against each of VARLIB (tools/variants.py builds, space-separated),
# per precision, two rounds.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dqn.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_dqn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_dqn.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for p in ${PRECISIONS:-f32}; do
    echo "== round $r precision $p product" >> gpurun_out/time_act.log
    timeout -k 10 120 python tools/time_act.py --precision $p >> gpurun_out/time_act.log 2>&1 || exit $?
    for v in $VARLIB; do
      echo "== round $r precision $p $v" >> gpurun_out/time_act.log
      timeout -k 10 120 python tools/time_act.py --precision $p --lib $v >> gpurun_out/time_act.log 2>&1 || exit $?
    done
  done
done
cat gpurun_out/time_act.log
