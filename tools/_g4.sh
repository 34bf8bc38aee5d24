#!/bin/bash
# round 4: (1) code act v3 in the main tree: parity, timing vs the round-3 kernel, stamps;
# (2) the nibble-ground branch (worktree _wt/nib): the whole GPU suite, then the driver's bench line
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
export ROOT=$PWD
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "code or qnet or dqn" > gpurun_out/g4_code3_tests.log 2>&1; rc=$?
tail -3 gpurun_out/g4_code3_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for r in 1 2; do
  timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g4_time.log 2>&1 || exit 1
  DRL_QN_CODE3=0 timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g4_time.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 >> gpurun_out/g4_time.log 2>&1 || exit 1
DRL_QN_CODE3=0 timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 >> gpurun_out/g4_time.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g4_time.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst3.so --precision f32 --input code --stamps > gpurun_out/g4_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g4_stamps.log
cd _wt/nib || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $ROOT/gpurun_out/g4_nib_tests.log 2>&1; rc=$?
tail -15 $ROOT/gpurun_out/g4_nib_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $ROOT/gpurun_out/g4_nib_bench.json 2> $ROOT/gpurun_out/g4_nib_bench.err || exit 1
python - <<'PY'
import json
d = json.load(open("/dev/stdin" if False else __import__("os").environ["ROOT"] + "/gpurun_out/g4_nib_bench.json"))
r = d["roofline"]; c5 = d["c5"]
print("C3 value %.3e ms/step %.2f launch %.2f read B/env %.1f write %.1f | C5 value %.3e launch %.1f read %.1f frac %.3f" % (
    d["value"], d["ms_per_step"] * 1e3, r["avg_launch_us"], r["traffic_detail"]["read_bytes_per_env"],
    r["traffic_detail"]["write_bytes_per_env"], c5["value"], c5["roofline"]["avg_launch_us"],
    c5["roofline"]["traffic_detail"]["read_bytes_per_env"], c5["roofline"]["frac"]))
print("resets/s", d["resets_per_s"], "act_code_us", d["dqn_consumer"]["act_code_f32_us"], "loop", d["train_loop"]["us_per_step"],
      "c5 loop", c5["train_loop"]["us_per_step"])
PY
