#!/bin/bash
# GPU: the bench's step line (cached stores, refills included) for each
# tools/var_<v>.so in VARS, ROUNDS rounds, one config (CFG).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARS; do
    DRL_LIB=tools/var_$v.so timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 400 --warmup 40 --no-cpu-baseline \
      --no-reset-bench --no-dqn --loop-segments 0 --rollout-chunk 0 --no-pmc-traffic > gpurun_out/varstep_$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/varstep_$v.json').read().strip().splitlines()[-1]); f=d['refill']; print('${CFG:-c3} $v value %.4g' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'step %.2f' % d['roofline']['avg_launch_us'], 'refill/step %.2f' % f['per_step_us'])"
  done
done
