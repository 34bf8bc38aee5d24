"""Time drl_refill at C3 for different amounts of ring work (tools/, GPU).

The ring's count field is lowered by k before each timed refill, so the refill
re-draws the k forgotten entries (the same values: the stream is fixed).
python tools/refill_time.py [--config c3] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402

CFG = {"c3": (16, 8, 65536), "c3h": (16, 8, 32768), "c3q": (16, 8, 16384), "c4": (32, 16, 65536), "c5": (64, 32, 131072), "c2": (16, 8, 4096)}


def timed_refill(env, s):
    """Kernel time of one refill: the GPU is kept busy (torch.cuda._sleep) while
    the events and the launch are queued, so no host gap is timed."""
    torch.cuda._sleep(200000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    env.refill()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-step", action="store_true", help="skip the step timing (timing-only refill builds)")
    args = ap.parse_args()
    G, N, E = CFG[args.config]
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    for t in range(40):
        env.step(env.synth_actions(seed=1, step=t), obs_k=1)
    torch.cuda.synchronize()
    mi = env.state.mt_index
    out = {"config": args.config, "refill_every": env.refill_every}
    s = torch.cuda.current_stream()
    for k in [0, 4, 8, 16, 24, 32, 48, 64]:
        ts = []
        for _ in range(args.reps):
            env.refill()
            env._since_refill = 0
            cnt = (mi >> 20) & 1023
            newc = torch.clamp(cnt - k, min=0)
            mi.copy_((mi & 0x00FFFFFF) | (newc << 24))
            ts.append(timed_refill(env, s))
        ts.sort()
        out[f"k{k}_us"] = round(ts[len(ts) // 2], 2)
    # steady state: refill_every steps of consumption, then the timed refill
    ts = []
    every, env.refill_every = env.refill_every, 0
    for r in range(args.reps):
        for t in range(every):
            env.step(env.synth_actions(seed=5, step=1000 + r * 64 + t), obs_k=1)
        ts.append(timed_refill(env, s))
    env.refill_every = every
    ts.sort()
    out["steady_us"] = round(ts[len(ts) // 2], 2)
    if args.no_step:
        print(json.dumps(out))
        return
    # the step alone, cadence off
    env.refill_every = 0
    acts = [env.synth_actions(seed=2, step=t) for t in range(20)]
    obs = torch.empty((E, 1, 7, 7, 6), device="cuda")
    env.refill()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for a in acts[:10]:
        env.step(a, obs_k=1, obs=obs, obs_stream=True)
    e1.record(s)
    torch.cuda.synchronize()
    out["step_us"] = round(e0.elapsed_time(e1) * 1e3 / 10, 2)
    env.check_errors()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
