#!/usr/bin/env python3
"""Interleaved in-process A/B timing of drl_step variants (methodology rule 24).

python tools/ab.py --config c3 --rounds 5 --steps 100
Variants (env knobs read per call): specN = DRL_SPECIALIZE (compile-time
geometry instance on/off), noobs = step without observation, wideN =
observation store mode (0: 8-B stores, 1: 16-B via LDS transpose, the
default).  Prints median/min µs per launch.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--lib", default="", help="alternative library (tools/variants.py build)")
    ap.add_argument("--variants", default="spec1,spec0,spec1_noobs,spec0_noobs",
                    help="comma list; each: specN[_noobs][_wide0|_wide1][_nt1]")
    args = ap.parse_args()
    if args.lib:
        import dronerl_amd._native as nat
        nat.LIB_PATH = os.environ["DRL_LIB"] = os.path.abspath(args.lib)
    G, N, E, K = CONFIGS[args.config]
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    T = args.steps
    acts = torch.empty((T, E, N), dtype=torch.int32, device="cuda")
    for t in range(T):
        env.synth_actions(seed=5, step=t, out=acts[t])
    W = env.layout.obs_window
    rew = torch.empty((E, N), device="cuda")
    dn = torch.empty((E, N), dtype=torch.uint8, device="cuda")
    obs = torch.empty((E, K, W, W, 6), device="cuda")
    L = lib()
    cp, st = ctypes.byref(env._cp), env.state.c()
    sp = ctypes.byref(st)
    ap_ = [ctypes.c_void_p(acts[t].data_ptr()) for t in range(T)]
    rp, dp, op = (ctypes.c_void_p(x.data_ptr()) for x in (rew, dn, obs))
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    variants = args.variants.split(",")
    res = {v: [] for v in variants}
    for r in range(args.rounds + 1):
        for v in variants:
            parts = v.split("_")
            os.environ["DRL_SPECIALIZE"] = parts[0][4:] if parts[0].startswith("spec") else "1"
            os.environ["DRL_OBS_WIDE"] = next((x[4:] for x in parts if x.startswith("wide")), "1")
            k = 0 if "noobs" in parts else K
            o = op if k else None
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            flags = 1 if "nt1" in parts else 0  # DRL_STEP_OBS_STREAM
            for t in range(T):
                L.drl_step_ex(cp, sp, ap_[t], rp, dp, o, k, None, flags, s)
            e1.record()
            torch.cuda.synchronize()
            if r:
                res[v].append(e0.elapsed_time(e1) * 1e3 / T)
    for v in variants:
        x = res[v]
        print(f"{os.path.basename(args.lib) or 'libdronerl.so'} {args.config} {v:12s} median {statistics.median(x):8.2f} us  min {min(x):8.2f} us  "
              f"-> {E / statistics.median(x) * 1e6:.3e} env-steps/s")


if __name__ == "__main__":
    main()
