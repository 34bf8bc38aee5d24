#!/bin/bash
# round 4: probe test, act stamps, ring-window (CQ=1) A/B + parity + PMC bytes
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "hbm_probe" > gpurun_out/g2_probe.log 2>&1 || exit 1
tail -2 gpurun_out/g2_probe.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst2.so --precision f32 --input code --stamps > gpurun_out/g2_stamps.log 2>&1 || exit 1
timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g2_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g2_stamps.log
DRL_LIB=tools/var_cq1.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ring or rollout or full_size or trajectory" > gpurun_out/g2_cq1_tests.log 2>&1 || exit 1
tail -2 gpurun_out/g2_cq1_tests.log
for r in 1 2; do
for v in "" tools/var_cq1.so; do
  timeout -k 10 200 python tools/ab.py ${v:+--lib $v} --config c3 --rounds 5 --steps 200 --variants spec1 > gpurun_out/g2_ab_${r}_$(basename ${v:-prod}).log 2>&1 || exit 1
  echo "$r ${v:-prod}: $(grep -v amdgpu gpurun_out/g2_ab_${r}_$(basename ${v:-prod}).log | tail -1)"
done
done
A="--steps 200 --warmup 20 --no-cpu-baseline --no-reset-bench --no-dqn --rollout-chunk 0 --loop-segments 0 --cached-steps 0 --c5-envs 0"
timeout -k 10 300 python bench.py $A > gpurun_out/g2_bench_prod.json 2>gpurun_out/g2_bench_prod.err || exit 1
DRL_LIB=tools/var_cq1.so timeout -k 10 300 python bench.py $A > gpurun_out/g2_bench_cq1.json 2>gpurun_out/g2_bench_cq1.err || exit 1
python - <<'PY'
import json
for n in ("prod", "cq1"):
    d = json.load(open(f"gpurun_out/g2_bench_{n}.json"))
    r = d["roofline"]
    print(n, "ms/step", round(d["ms_per_step"] * 1e3, 2), "launch", round(r["avg_launch_us"], 2),
          "read B/env", round(r["traffic_detail"]["read_bytes_per_env"], 1), "write", round(r["traffic_detail"]["write_bytes_per_env"], 1),
          "copy peak", round(r.get("peak_measured", 0)), "read peak", round(r.get("peak_measured_detail", {}).get("read_GBs", 0)))
PY
