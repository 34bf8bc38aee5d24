#!/bin/bash
# GPU: DQN/replay tests on the default build, then the C3 train loop per
# variant build (VARS -> tools/var_<v>.so), alternating, two rounds.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_dqn.py -m gpu -q --maxfail=3 > gpurun_out/pytest_dqn.log 2>&1
rc=$?; echo "dqn tests rc=$rc: $(tail -1 gpurun_out/pytest_dqn.log)"; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for v in $VARS; do
    DRL_LIB=tools/var_$v.so timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-reset-bench --rollout-chunk 0 > gpurun_out/loop_$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/loop_$v.json').read().strip().splitlines()[-1]); print('$v', 'train_loop', round(d['train_loop']['us_per_step'], 2), 'us/step')"
  done
done
