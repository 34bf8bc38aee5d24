#!/usr/bin/env python3
"""Diagnostic: where drl_reset_wave_kernel's clocks go, per wave (one env).

Builds libdronerl_stamps.so (-DDRL_STAMPS; never the product library), runs
continuing resets at a config and prints the mean shader clocks per category:
  batched FY chunks (fy_chunk with swaps), count-only chunks, chunk moves and
  twists, one-draw-at-a-time FY tails, the drone sample, settle (placing
  objects), and the wave total; plus chunk and twist counts.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--envs", type=int, default=0)
    ap.add_argument("--resets", type=int, default=3)
    ap.add_argument("--prebuilt", action="store_true")
    args = ap.parse_args()
    from stamps import build_stamps_lib
    path = os.path.join(REPO, "tools", "libdronerl_stamps.so") if args.prebuilt else build_stamps_lib()
    import dronerl_amd._native as nat
    nat.LIB_PATH = os.environ["DRL_LIB"] = path
    L = nat.lib()
    L.drl_debug_set_stamps.argtypes = [ctypes.c_void_p]
    from bench import CONFIGS
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    G, N, E, _ = CONFIGS[args.config]
    E = args.envs or E
    # the buffer goes in before any kernel of this build runs
    stamps = torch.zeros((E, 16), dtype=torch.int64, device="cuda")
    assert L.drl_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    names = ["FY chunks (swaps)", "chunk moves + twists", "count-only chunks", "1-draw FY tails",
             "drone sample", "settle / place"]
    for r in range(args.resets):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        env.reset()
        ev1.record()
        torch.cuda.synchronize()
        # rows below E/4 also take the refill's per-wave stamps (the reset ends with one)
        st = stamps[E // 4 + 1:].cpu().numpy().astype("float64")
        tot = st[:, 9].mean()
        print(f"reset {r}: {ev0.elapsed_time(ev1):.2f} ms for {E} envs; wave clocks mean {tot:.0f}")
        for k, n in enumerate(names):
            print(f"  {n:22s} {st[:, k].mean():10.0f}  {st[:, k].mean() / tot * 100:5.1f}%")
        print(f"  chunks with swaps {st[:, 6].mean():.1f}, count-only {st[:, 8].mean():.1f}, "
              f"twists {st[:, 7].mean():.1f}; clk per swap chunk {st[:, 0].mean() / max(st[:, 6].mean(), 1):.0f}, "
              f"per count-only chunk {st[:, 2].mean() / max(st[:, 8].mean(), 1):.0f}, "
              f"per twist+move {st[:, 1].mean() / max(st[:, 7].mean(), 1):.0f}")


if __name__ == "__main__":
    main()
