#!/bin/bash
# tools/loop_ab.sh — the bench's train loop (with the learner) serial vs parallel graph branches, C3 and C5
# (GPU box; run through gpurun).  -> gpurun_out/loop_ab_<cfg>_<mode>.json
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
A="--steps 20 --warmup 5 --no-cpu-baseline --no-reset-bench --rollout-chunk 0 --no-pmc-traffic --cached-steps 0 --c5-envs 0"
for c in ${LCFGS:-c3 c5}; do
  for m in serial parallel; do
    P=""; [ $m = parallel ] && P="--parallel-loop"
    timeout -k 10 300 python bench.py --config $c $A $P > gpurun_out/loop_ab_${c}_$m.json 2> gpurun_out/loop_ab_${c}_$m.log || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/loop_ab_${c}_$m.json')); t=d['train_loop']; print('$c $m', round(t['us_per_step'],2))"
  done
done
