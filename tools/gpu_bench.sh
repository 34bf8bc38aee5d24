# Bench lines on one GPU: C3 (the driver's default run) and C4/C5 (no CPU baseline).
set -u
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python bench.py ${C3_ARGS:-} > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
for c in ${MORE_CFGS:-c4 c5}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/bench_c*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, f"value={d['value']:.4g} us/launch={r['avg_launch_us']:.2f} frac={r['frac']:.3f} frac_rw={r['frac_read_plus_write']:.3f}",
          "resets/s=%.3g" % d["resets_per_s"], "loop=", json.dumps(d.get("train_loop")), "dqn act_us=", (d.get("dqn_consumer") or {}).get("act_us"),
          "cpu=", (d.get("cpu_baseline") or {}).get("value"))
PY
