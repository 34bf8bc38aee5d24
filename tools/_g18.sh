#!/bin/bash
# round 4 final check on the final build: the whole GPU suite, smoke, and the driver's own bench command
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=_r4b T_TESTS=900 bash tools/gpu.sh tests smoke || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r4_driver.json 2> gpurun_out/bench_r4_driver.err || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_r4_driver.json"))
r = d["roofline"]; c5 = d["c5"]; q = d["dqn_consumer"]
print("C3 value %.3e ms/step %.2f launch %.2f read B/env %.1f | C5 value %.3e launch %.1f frac %.3f | act_code %.2f us frac %.3f | loop %.1f / c5 loop %.1f" % (
    d["value"], d["ms_per_step"] * 1e3, r["avg_launch_us"], r["traffic_detail"]["read_bytes_per_env"],
    c5["value"], c5["roofline"]["avg_launch_us"], c5["roofline"]["frac"], q["act_code_f32_us"], q["act_code_roofline"]["frac"],
    d["train_loop"]["us_per_step"], c5["train_loop"]["us_per_step"]))
PY
