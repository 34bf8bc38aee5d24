#!/usr/bin/env python3
"""Diagnostic: per-phase wave timing of drl_step from s_memtime stamps.

Builds a separate libdronerl_stamps.so (-DDRL_STAMPS; never the product
library), runs the bench workload and prints mean/median phase durations
(shader clocks) over waves:
  0->1 loads + MT prefetch   1->2 claims/collision scan + DMA wait
  2->3 effects + ordering    3->4 respawn rounds   4->5 write-back
  5->6 observation
"""
import argparse
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def build_stamps_lib(flags=(), tag=""):
    from dronerl_amd import build as b
    out = os.path.join(REPO, "tools", f"libdronerl_stamps{tag}.so")  # never beside the product library
    cmd = [b.hipcc(), f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DDRL_STAMPS",
           "-I", os.path.join(REPO, "include"), "-o", out] + list(flags) + b.SOURCES
    subprocess.run(cmd, check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--envs", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--obs", type=int, default=1)
    ap.add_argument("--flags", default="", help="extra compile flags, comma separated")
    ap.add_argument("--tag", default="", help="library name suffix")
    ap.add_argument("--build-only", action="store_true", help="build the stamps library here and exit")
    ap.add_argument("--prebuilt", action="store_true", help="use the library --build-only made")
    args = ap.parse_args()
    flags = [f for f in args.flags.split(",") if f]
    if args.prebuilt:
        path = os.path.join(REPO, "tools", f"libdronerl_stamps{args.tag}.so")
    else:
        path = build_stamps_lib(flags, args.tag)
    if args.build_only:
        print(path)
        return
    import dronerl_amd._native as nat
    nat.LIB_PATH = os.environ["DRL_LIB"] = path
    L = nat.lib()
    L.drl_debug_set_stamps.argtypes = [ctypes.c_void_p]
    from bench import CONFIGS
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    G, N, E, K = CONFIGS[args.config]
    E = args.envs or E
    K = args.obs
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    P = env.layout.step_group_lanes
    nwaves = (E + 64 // P - 1) // (64 // P)
    # rows for every kernel of the stamps build: step waves, refill waves (E/4), resets (E)
    stamps = torch.zeros((max(nwaves, E) + 64, 16), dtype=torch.int64, device="cuda")
    assert L.drl_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
    acc = []
    rounds = []
    subs = []
    for t in range(args.steps):
        a = env.synth_actions(seed=1, step=t)
        env.step(a, obs_k=K)
        torch.cuda.synchronize()
        st = stamps[:nwaves].cpu().numpy().astype(np.int64)
        if t >= 2:
            acc.append(np.diff(st[:, :7], axis=1))
            rounds.append(st[:, 7].copy())
            subs.append(st[:, 10:14].copy())
        if t == args.steps - 1:
            # s_memrealtime (100 MHz, chip-wide) at wave start / end
            rs, re_ = st[:, 8], st[:, 9]
            t0 = rs.min()
            starts, ends = (rs - t0) / 100.0, (re_ - t0) / 100.0  # us
            span = ends.max()
            life = ends - starts
            print(f"launch span {span:.1f} us; wave start p10/50/90/max {np.percentile(starts, 10):.1f}/"
                  f"{np.percentile(starts, 50):.1f}/{np.percentile(starts, 90):.1f}/{starts.max():.1f} us; "
                  f"wave lifetime p10/50/90 {np.percentile(life, 10):.1f}/{np.percentile(life, 50):.1f}/"
                  f"{np.percentile(life, 90):.1f} us")
            conc = [int(((starts <= x) & (ends > x)).sum()) for x in np.linspace(0, span, 12)]
            print(f"  resident waves over the span (12 samples): {conc}")
            print(f"  wave end p10/50/90/99/max {np.percentile(ends, 10):.1f}/{np.percentile(ends, 50):.1f}/"
                  f"{np.percentile(ends, 90):.1f}/{np.percentile(ends, 99):.1f}/{ends.max():.1f} us; "
                  f"lifetime max {life.max():.1f} us")
            rl = st[:, 7]
            late = ends >= np.percentile(ends, 99)
            print("  wave end by respawn trips (trips: n / mean end us / max end us): " + ", ".join(
                f"{k}: {int((rl == k).sum())}/{ends[rl == k].mean():.1f}/{ends[rl == k].max():.1f}"
                for k in range(int(rl.max()) + 1) if (rl == k).any()))
            print(f"  latest 1% of waves: trips mean {rl[late].mean():.2f} (all waves {rl.mean():.2f}), "
                  f"start mean {starts[late].mean():.1f} us (all {starts.mean():.1f})")
            xcd = np.arange(len(starts)) % 8
            print("  per-XCD (block % 8) mean start / mean end / max end us: " + ", ".join(
                f"{starts[xcd == i].mean():.1f}/{ends[xcd == i].mean():.1f}/{ends[xcd == i].max():.1f}"
                for i in range(8)))
    d = np.concatenate(acc)
    names = ["loads+MT prefetch", "claims+DMA wait", "effects+ordering", "respawn rounds", "write-back",
             "observation"]
    tot = d.sum(1)
    print(f"{args.config} E={E} K={K}: wave lifetime (clk) mean {tot.mean():.0f} median {np.median(tot):.0f} "
          f"p90 {np.percentile(tot, 90):.0f}")
    sub = np.concatenate(subs)
    print("  respawn sub-phases, clk per wave (mean over waves): " + ", ".join(
        f"{n} {sub[:, i].mean():.0f}" for i, n in enumerate(["twists", "candidates", "placement", "round tail"])))
    rr = np.concatenate(rounds)
    print(f"  respawn loop trips per wave: mean {rr.mean():.2f}  median {np.median(rr):.0f}  p90 "
          f"{np.percentile(rr, 90):.0f}  max {rr.max()}  hist {np.bincount(rr, minlength=8)[:10].tolist()}")
    for i, n in enumerate(names):
        print(f"  {n:20s} mean {d[:, i].mean():8.0f}  median {np.median(d[:, i]):8.0f}  p90 "
              f"{np.percentile(d[:, i], 90):8.0f}  share {d[:, i].mean() / tot.mean() * 100:5.1f}%")


if __name__ == "__main__":
    main()
