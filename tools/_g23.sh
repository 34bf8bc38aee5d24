#!/bin/bash
# round 4: the new refill cadence (C3 48, C4 38, C5 28) against the old (32, 31, 22), 1000/300-step lines; ring and
# refill GPU tests
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ring or refill or cadence or fullsize or rollout" > gpurun_out/g23_tests.log 2>&1; rc=$?
tail -2 gpurun_out/g23_tests.log
[ $rc -ne 0 ] && exit $rc
A="--no-cpu-baseline --no-reset-bench --no-dqn --rollout-chunk 0 --loop-segments 0 --no-pmc-traffic --cached-steps 0 --c5-envs 0"
for r in 1 2; do
  for ce in c3: c3:32 c4: c4:31 c5: c5:22; do
    c=${ce%%:*}; e=${ce##*:}; st=1000; [ $c = c5 ] && st=300
    if [ -n "$e" ]; then export DRL_REFILL_EVERY=$e; else unset DRL_REFILL_EVERY; fi
    timeout -k 10 300 python bench.py --config $c --steps $st --warmup 50 $A > gpurun_out/g23_${c}_${e:-new}.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/g23_${c}_${e:-new}.json'));print('$c every', d['refill']['every'], round(d['value']/1e9,4), 'e9', round(d['ms_per_step']*1e3,3), 'us/step refill', round(d['refill']['per_step_us'],3))"
  done
done
unset DRL_REFILL_EVERY
