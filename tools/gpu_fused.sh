#!/bin/bash
# GPU: DQN + train-segment tests, then the C3 train loop with the synthetic
# actions fused into the act launch and as their own launch, two rounds.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_dqn.py tests/test_gpu_parity.py -m gpu -q --maxfail=3 -k "dqn or qnet or train_segment or replay" > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_fused.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for f in "" "--unfused-act"; do
    timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps 200 --warmup 20 --no-cpu-baseline --no-reset-bench $f > gpurun_out/fused.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/fused.json').read().strip().splitlines()[-1]); print('${f:-fused}', 'train_loop', round(d['train_loop']['us_per_step'], 2), 'us/step; act alone', round(d['dqn_consumer']['act_us'], 2))"
  done
done
