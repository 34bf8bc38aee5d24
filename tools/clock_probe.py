#!/usr/bin/env python3
"""Diagnostic: the GPU's shader clock and power while a workload runs.

A thread polls `rocm-smi --showclocks --showpower --json` (read-only) while
the main thread replays, for --seconds each:
  loop  the C5 (or --config) train loop as bench.py times it (HIP graph of 100 steps),
  act   drl_qnet_act_code alone on the same env's codes, back to back,
  flush the same act with a 256 MB overwrite before every launch,
  step  the env step alone,
and prints the median sclk / power per phase (question: is the in-loop act
slower than the standalone one because the clock drops under the loop's load?).

python tools/clock_probe.py [--config c5] [--seconds 4]
"""
import argparse
import json
import os
import re
import statistics
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def smi_sample():
    out = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--json"], capture_output=True, text=True,
                         timeout=20).stdout
    d = json.loads(out[out.index("{"):])
    card = d[sorted(k for k in d if k.startswith("card"))[0]]
    sclk = pw = None
    for k, v in card.items():
        kl = k.lower()
        if "sclk" in kl and sclk is None:
            m = re.search(r"(\d+)\s*mhz", str(v).lower())
            sclk = int(m.group(1)) if m else None
        if "power" in kl and "socket" in kl or ("average graphics package power" in kl):
            try:
                pw = float(re.findall(r"[\d.]+", str(v))[0])
            except (IndexError, ValueError):
                pass
    return sclk, pw


class Poller(threading.Thread):
    def __init__(self):
        super().__init__(daemon=True)
        self.phase = None
        self.samples = {}
        self.stop = False

    def run(self):
        while not self.stop:
            ph = self.phase
            try:
                s = smi_sample()
            except Exception as e:  # noqa: BLE001 (diagnostic: report and go on)
                print("rocm-smi:", e, file=sys.stderr)
                s = (None, None)
            if ph is not None and ph == self.phase:
                self.samples.setdefault(ph, []).append(s)
            time.sleep(0.05)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--seconds", type=float, default=4.0)
    args = ap.parse_args()
    import torch
    import bench
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    G, N, E = bench.CONFIGS[args.config][:3]
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    raw = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--json"], capture_output=True, text=True,
                         timeout=20).stdout
    print("raw rocm-smi (idle):", raw[:3000], flush=True)
    print("parsed (idle):", smi_sample(), flush=True)
    poll = Poller()
    poll.start()
    timing = {}

    def run_phase(name, fn, per_call_steps=1):
        torch.cuda.synchronize()
        poll.phase = name
        t0 = time.time()
        n = 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        while time.time() - t0 < args.seconds:
            for _ in range(20):
                fn()
            n += 20
            torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        poll.phase = None
        timing[name] = e0.elapsed_time(e1) * 1e3 / (n * per_call_steps)
        print(f"{name}: {timing[name]:.1f} us per call", flush=True)

    # the train loop (graph), as bench.train_loop_bench captures it
    loop = bench.TrainSegment(env, 100, input="code")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        loop.run()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loop.run()
    run_phase("loop", g.replay, per_call_steps=100)
    net = loop.net
    code = env.new_code()
    env.get_code(out=code)
    acts = torch.zeros((E, N), dtype=torch.int32, device="cuda")
    run_phase("act", lambda: net.act(code, 0.1, actions=acts))
    junk = torch.empty(64 << 20, dtype=torch.float32, device="cuda")

    def flush_act():
        junk.fill_(1.0)
        net.act(code, 0.1, actions=acts)
    run_phase("act+flush (fill included)", flush_act)
    st_acts = env.synth_actions(seed=1, step=0)
    run_phase("step", lambda: env.step(st_acts))
    poll.stop = True
    out = {"config": args.config, "us_per_call": timing}
    for ph, ss in poll.samples.items():
        cl = [s[0] for s in ss if s[0]]
        pw = [s[1] for s in ss if s[1]]
        out[ph] = {"samples": len(ss), "sclk_mhz_median": statistics.median(cl) if cl else None,
                   "sclk_mhz_min": min(cl) if cl else None, "power_w_median": statistics.median(pw) if pw else None}
    print(json.dumps(out, indent=1))
    env.check_errors()


if __name__ == "__main__":
    main()
