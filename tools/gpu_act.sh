#!/bin/bash
# GPU: parity suite (default build), the DQN tests on act-kernel variant
# builds (VARS="q0 t2r2 ..." -> tools/var_<v>.so), act timing per variant,
# then one default bench line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for v in ${VARS:-}; do
  DRL_LIB=tools/var_$v.so timeout -k 10 300 python -m pytest tests/test_dqn.py -m gpu -q --maxfail=3 > gpurun_out/pytest_dqn_$v.log 2>&1
  rc=$?; echo "dqn tests $v rc=$rc: $(tail -1 gpurun_out/pytest_dqn_$v.log)"
  [ $rc -le 1 ] || exit $rc
done
for r in 1 2; do
  for v in ${VARS:-}; do
    timeout -k 10 120 python tools/time_act.py --lib tools/var_$v.so --envs 65536 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 400 python bench.py --steps 500 --warmup 50 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'us', d['roofline']['avg_launch_us'], 'train_loop', d['train_loop']['us_per_step'], 'act', d['dqn_consumer']['act_us'], 'rollout', d['rollout']['value'])"
