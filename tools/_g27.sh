#!/bin/bash
# round 4: the final build (reset 4 waves per workgroup at >= 4096 cells): whole GPU suite, smoke, reset rates,
# driver bench
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=_r4c T_TESTS=900 bash tools/gpu.sh tests smoke || exit 1
timeout -k 10 300 python tools/reset_rate.py --configs c3,c4,c5 --variants wave > gpurun_out/g27_rate.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g27_rate.log | tail -3
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r4_driver3.json 2> gpurun_out/bench_r4_driver3.err || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_r4_driver3.json"))
r = d["roofline"]; c5 = d["c5"]; q = d["dqn_consumer"]
print("C3 value %.3e ms/step %.2f launch %.2f | C5 value %.3e launch %.1f frac %.3f | act_code %.2f us | loop %.1f / c5 loop %.1f | resets/s %.3e" % (
    d["value"], d["ms_per_step"] * 1e3, r["avg_launch_us"], c5["value"], c5["roofline"]["avg_launch_us"], c5["roofline"]["frac"],
    q["act_code_f32_us"], d["train_loop"]["us_per_step"], c5["train_loop"]["us_per_step"], d["resets_per_s"]))
PY
