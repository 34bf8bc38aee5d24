#!/usr/bin/env python3
"""Launch time of drl_step vs number of envs (latency/tail vs throughput).

python tools/scan_envs.py --config c3 --envs 8192,24576,49152,65536,98304,131072,262144
"""
import argparse
import ctypes
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402
from dronerl_amd._native import lib  # noqa: E402


def time_env(G, N, E, K, steps, rounds):
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    acts = torch.empty((steps, E, N), dtype=torch.int32, device="cuda")
    for t in range(steps):
        env.synth_actions(seed=5, step=t, out=acts[t])
    W = env.layout.obs_window
    rew = torch.empty((E, N), device="cuda")
    dn = torch.empty((E, N), dtype=torch.uint8, device="cuda")
    obs = torch.empty((E, max(K, 1), W, W, 6), device="cuda")
    L = lib()
    cp, st = ctypes.byref(env._cp), env.state.c()
    sp = ctypes.byref(st)
    ap_ = [ctypes.c_void_p(acts[t].data_ptr()) for t in range(steps)]
    rp, dp, op = (ctypes.c_void_p(x.data_ptr()) for x in (rew, dn, obs))
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = []
    for r in range(rounds + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for t in range(steps):
            L.drl_step(cp, sp, ap_[t], rp, dp, op if K else None, K, None, s)
        e1.record()
        torch.cuda.synchronize()
        if r:
            res.append(e0.elapsed_time(e1) * 1e3 / steps)
    return statistics.median(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--envs", default="8192,24576,49152,65536,98304,131072,262144")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--obs", type=int, default=1)
    args = ap.parse_args()
    G, N, _, K = CONFIGS[args.config]
    K = args.obs
    for E in [int(v) for v in args.envs.split(",")]:
        us = time_env(G, N, E, K, args.steps, args.rounds)
        print(f"{args.config} K={K} E={E:8d}  {us:9.2f} us/launch  {E / us * 1e6:.3e} env-steps/s  "
              f"{us * 1e3 / E:.3f} ns/env", flush=True)


if __name__ == "__main__":
    main()
