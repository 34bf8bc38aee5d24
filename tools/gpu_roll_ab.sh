#!/bin/bash
# GPU: drl_rollout A/B across variant builds (VARS -> tools/var_<v>.so), C3
# rollout value (bench.py's rollout leg only), two rounds; the rollout parity
# tests on VARLIB first.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${VARLIB:-}" ]; then
  DRL_LIB=$VARLIB timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q --maxfail=3 -k "rollout" > gpurun_out/pytest_var.log 2>&1
  rc=$?; echo "variant rollout tests ($VARLIB) rc=$rc"; tail -1 gpurun_out/pytest_var.log
  [ $rc -le 1 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARS; do
    DRL_LIB=tools/var_$v.so timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 500 --warmup 100 --no-cpu-baseline \
      --no-reset-bench --no-dqn --loop-segments 0 > gpurun_out/roll_$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/roll_$v.json').read().strip().splitlines()[-1]); r=d['rollout']; print('$v', 'rollout', round(r['ms_per_step']*1e3, 2), 'us/step', 'no_obs', round(r['no_obs']['ms_per_step']*1e3, 2), 'step', round(d['roofline']['avg_launch_us'], 2))"
  done
done
