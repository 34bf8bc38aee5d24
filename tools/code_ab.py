#!/usr/bin/env python3
"""A/B: drl_step with and without the policy code output, interleaved blocks
(diagnostic).  python tools/code_ab.py [--config c3] [--rounds 5] [--steps 100]"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--only", default="", choices=("", "plain", "code", "codeonly", "noobs"))
    args = ap.parse_args()
    G, N, E = bench.CONFIGS[args.config][:3]
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    env.refill_every = 0
    W = env.layout.obs_window
    obs = torch.empty((E, 1, W, W, 6), device="cuda")
    code = env.new_code()
    acts = [env.synth_actions(seed=1, step=t) for t in range(args.steps)]
    res = {"plain": [], "code": [], "codeonly": [], "noobs": []}
    for r in range(args.rounds):
        for name in ((args.only,) if args.only else ("plain", "code", "codeonly", "noobs")):
            env.reset(seed=r)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for t in range(args.steps):
                if name in ("plain", "code"):
                    env.step(acts[t], obs_k=1, obs=obs, code=code if name == "code" else None)
                else:
                    env.step(acts[t], code=code if name == "codeonly" else None)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / args.steps)
    for k, v in res.items():
        if not v:
            continue
        print(f"{args.config} {k}: median {statistics.median(v):.2f} us/step, min {min(v):.2f}", flush=True)


if __name__ == "__main__":
    main()
