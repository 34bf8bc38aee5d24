#!/bin/bash
# train-loop A/B: one stream vs the replay add and the refill on parallel graph branches
# (bench.py's train loop; the other measurements trimmed).
mkdir -p gpurun_out
export TMPDIR=/tmp
L="--steps 20 --warmup 2 --no-cpu-baseline --no-reset-bench --rollout-chunk 0 --no-pmc-traffic --c5-envs 0 --cached-steps 0 --loop-segments 5"
for r in 1 2; do
  for mode in "one" "par"; do
    case $mode in
      one) A="" ;;
      par) A="--parallel-loop" ;;
    esac
    timeout -k 10 300 python bench.py $L $A > gpurun_out/loop_ab.json 2> gpurun_out/loop_ab.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -3 gpurun_out/loop_ab.err; exit $rc; fi
    MODE=$mode python - <<'PY' || exit 1
import json, os
t = open("gpurun_out/loop_ab.json").read()
d = json.loads(t[t.find('{"metric"'):].splitlines()[0])
print(os.environ["MODE"], round(d["train_loop"]["us_per_step"], 2), "us/step")
PY
  done
done
