#!/bin/bash
# GPU: the bench's train loop with cached vs streaming observation stores in
# the step (DRL_LOOP_OBS_STREAM), per config in CFGS, two rounds.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for c in ${CFGS:-c3 c4 c5}; do
    for m in 0 1; do
      DRL_LOOP_OBS_STREAM=$m timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline \
        --no-reset-bench --rollout-chunk 0 --no-pmc-traffic > gpurun_out/loop_${c}_$m.json 2>/dev/null || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/loop_${c}_$m.json').read().strip().splitlines()[-1]); t=d['train_loop']; print('$c stream=$m loop %.2f us/step' % t['us_per_step'])"
    done
  done
done
