#!/bin/bash
# round 4: refill cadence at C3 / C5 with the round-3 block-conversion refill (DRL_REFILL_EVERY), 1000-step lines,
# interleaved; the ring tests at the default
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
A="--no-cpu-baseline --no-reset-bench --no-dqn --rollout-chunk 0 --loop-segments 0 --no-pmc-traffic --cached-steps 0 --c5-envs 0"
for r in 1 2; do
  for e in 32 48 64; do
    DRL_REFILL_EVERY=$e timeout -k 10 300 python bench.py --config c3 --steps 1000 --warmup 50 $A > gpurun_out/g22_c3_$e.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/g22_c3_$e.json'));print('c3 every $e', round(d['value']/1e9,4), 'e9', round(d['ms_per_step']*1e3,3), 'us/step refill', round(d['refill']['per_step_us'],3), 'launch', round(d['refill']['avg_launch_us'],1))"
  done
  for e in 22 32 44; do
    DRL_REFILL_EVERY=$e timeout -k 10 300 python bench.py --config c5 --steps 300 --warmup 20 $A > gpurun_out/g22_c5_$e.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/g22_c5_$e.json'));print('c5 every $e', round(d['value']/1e9,4), 'e9', round(d['ms_per_step']*1e3,2), 'us/step refill', round(d['refill']['per_step_us'],3), 'launch', round(d['refill']['avg_launch_us'],1))"
  done
done
