#!/usr/bin/env python3
"""Diagnostic: per-wave clocks of drl_refill (-DDRL_STAMPS build, never the product).

python tools/refill_stamps.py --build-only   (here), then on the GPU:
python tools/refill_stamps.py --prebuilt [--k 20]
Per wave: first round trip, twist batches, passes (shader clocks), twists, passes.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=20, help="ring entries forgotten before the timed refill")
    ap.add_argument("--flags", default="")
    ap.add_argument("--tag", default="_refill")
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--prebuilt", action="store_true")
    args = ap.parse_args()
    from stamps import build_stamps_lib
    if args.prebuilt:
        path = os.path.join(REPO, "tools", f"libdronerl_stamps{args.tag}.so")
    else:
        path = build_stamps_lib([f for f in args.flags.split(",") if f], args.tag)
    if args.build_only:
        print(path)
        return
    import dronerl_amd._native as nat
    nat.LIB_PATH = os.environ["DRL_LIB"] = path
    L = nat.lib()
    L.drl_debug_set_stamps.argtypes = [ctypes.c_void_p]
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    E = 65536
    env = BatchedDeliveryDrones(EnvParams(n_drones=8, grid_size=16), E)
    buf = torch.zeros((E, 16), dtype=torch.int64, device="cuda")
    assert L.drl_debug_set_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    env.reset(seed=0)
    for t in range(40):
        env.step(env.synth_actions(seed=1, step=t), obs_k=1)
    env.refill()
    mi = env.state.mt_index
    cnt = (mi >> 24) & 127
    mi.copy_((mi & 0x00FFFFFF) | (torch.clamp(cnt - args.k, min=0) << 24))
    torch.cuda.synchronize()
    buf.zero_()
    env.refill()
    torch.cuda.synchronize()
    nw = (E + 15) // 16
    r = buf[:nw].cpu().numpy().astype(np.int64)
    names = ["rt1", "twists", "passes", "life"]
    for i, n in zip([1, 2, 3, 4], names):
        v = r[:, i]
        print(f"{n:8s} mean {v.mean():9.0f} p50 {np.percentile(v, 50):9.0f} p90 {np.percentile(v, 90):9.0f} "
              f"max {v.max():9.0f}")
    ntw, np_ = r[:, 5], r[:, 6]
    print("twists/wave mean %.2f max %d; passes/wave mean %.2f max %d" % (ntw.mean(), ntw.max(), np_.mean(), np_.max()))
    for k in range(0, int(ntw.max()) + 1):
        m = ntw == k
        if m.any():
            print(f"  {k} twists: {m.sum():5d} waves, life mean {r[m, 4].mean():8.0f}, twist clk {r[m, 2].mean():8.0f}")
    st = r[:, 0] - r[:, 0].min()
    rt = r[:, 7] - r[:, 7].min()
    print("wave start (clk) p50 %.0f p90 %.0f max %.0f; realtime span (100MHz ticks) %d" %
          (np.percentile(st, 50), np.percentile(st, 90), st.max(), rt.max()))


if __name__ == "__main__":
    main()
