#!/bin/bash
# round 4: C3 step ring window (DRL_CQ_NARROW 1 / 3 entries per lane vs 2) on the packed ground, 1000-step bench lines
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
A="--no-cpu-baseline --no-reset-bench --no-dqn --rollout-chunk 0 --loop-segments 0 --no-pmc-traffic --cached-steps 0 --c5-envs 0"
for r in 1 2; do
  for v in prod cq1 cq3; do
    if [ $v = prod ]; then unset DRL_LIB; else export DRL_LIB=tools/var_$v.so; fi
    timeout -k 10 300 python bench.py --config c3 --steps 1000 --warmup 50 $A > gpurun_out/g30_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/g30_$v.json'));print('$v', round(d['value']/1e9,4), 'e9 launch', round(d['roofline']['avg_launch_us'],3), 'us/step', round(d['ms_per_step']*1e3,3))"
  done
done
