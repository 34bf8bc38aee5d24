#!/bin/bash
# GPU: refill cadence A/B (DRL_REFILL_EVERY) on the bench's step line, two
# rounds.  CADENCES="c5:11,16,22 c3:25,32" (config:cadence list).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for spec in ${CADENCES:-c5:11,16,22 c3:25,32}; do
    cfg=${spec%%:*}
    for ev in $(echo ${spec#*:} | tr , ' '); do
      DRL_REFILL_EVERY=$ev timeout -k 10 200 python bench.py --config $cfg --steps 400 --warmup 40 --no-cpu-baseline \
        --no-reset-bench --no-dqn --loop-segments 0 --rollout-chunk 0 --no-pmc-traffic > gpurun_out/refill_${cfg}_${ev}.json 2>/dev/null || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/refill_${cfg}_${ev}.json').read().strip().splitlines()[-1]); f=d['refill']; print('$cfg every', f['every'], 'value %.4g' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'step %.2f' % d['roofline']['avg_launch_us'], 'refill/step %.2f' % f['per_step_us'])"
    done
  done
done
