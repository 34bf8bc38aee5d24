#!/usr/bin/env python3
"""Diagnostic: per-phase timing of drl_dqn_train_kernel from wall_clock64
stamps (100 MHz) of a -DDRL_DQN_STAMPS build (tools/var_dqnstamps.so, never
the product library).  Every figure is the latest workgroup's, in us from the
earliest workgroup start (median over steps).

python tools/learn_stamps.py [--config c3] [--steps 20] [--build]   (DQN_FLAGS="-D..." adds build macros)
Per workgroup: setup (segment table + sample), stage (the prefetch round),
compute (layer-0 tile + its write-through stores), drain (vmcnt + barrier),
ticket; the last workgroup: target forward, online forward, TD, backward +
biases, counters.  Times in us relative to the earliest workgroup start.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "tools", "var_dqnstamps.so")


def build():
    from dronerl_amd import build as b
    cmd = [b.hipcc(), f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DDRL_DQN_STAMPS",
           "-I", os.path.join(REPO, "include"), "-o", LIB] + os.environ.get("DQN_FLAGS", "").split() + b.SOURCES
    subprocess.run(cmd, check=True)


# the tails' stamp slots (workgroup 0 online, 1 target)
TAIL = [(0, "start"), (1, "setup"), (7, "staged"), (2, "prefetched"), (3, "tickets_in"), (8, "z0_in"), (9, "layer1"),
        (10, "layer2"), (4, "forward_done"), (5, "target_max_in"), (12, "bw_out"), (13, "bw_1"),
        (15, "bw_done"), (6, "deltas_handed"), (14, "biases_done")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--lib", default="", help="another stamps build (default tools/var_dqnstamps.so)")
    args = ap.parse_args()
    if args.build:
        build()
        return
    os.environ["DRL_LIB"] = os.path.abspath(args.lib) if args.lib else LIB
    import numpy as np
    import torch
    import bench
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    G, N, E = bench.CONFIGS[args.config][:3]
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    loop = bench.TrainSegment(env, 2, input="code")
    lr = loop.learner
    for t in range(3):  # fill the ring
        loop._act_step(t)
        loop._replay(t)
        loop._learn()
    torch.cuda.synchronize()
    nblk = lr.layout.grad_workgroups - 2  # workgroup 0: online tail, 1: target tail, 2..: layer 0
    st = lr.block[lr.layout.bytes - 8192:].view(torch.int64)
    rows = []
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for k in range(args.steps):
        st.zero_()
        ev[k][0].record()
        lr.train(loop.rb)
        ev[k][1].record()
        torch.cuda.synchronize()
        s = st.cpu().numpy().astype(np.int64).reshape(-1, 16)
        on, tg, blk = s[0, :16], s[1, :16], s[2:2 + nblk, :8]
        t0 = min(blk[:, 0].min(), on[0], tg[0])
        f = lambda x: (x - t0) / 100.0  # noqa: E731
        flat = st.cpu().numpy().astype(np.int64)
        mhz = (flat[1002] - flat[1000]) / max(1, flat[1003] - flat[1001]) * 100.0  # shader clock over the online tail
        rows.append({"blocks": f(blk), "on": f(on), "tg": f(tg), "event_us": ev[k][0].elapsed_time(ev[k][1]) * 1e3,
                     "mhz": mhz})
    med = lambda xs: float(np.median(xs))  # noqa: E731
    bl = np.stack([r["blocks"] for r in rows])
    on = np.stack([r["on"] for r in rows])
    tg = np.stack([r["tg"] for r in rows])
    out = {"config": args.config, "layer0_workgroups": nblk,
           "kernel_event_us": med([r["event_us"] for r in rows]),
           "shader_clock_mhz": med([r["mhz"] for r in rows]),
           "layer0_us": {name: med(bl[:, :, i].max(1)) for i, name in
                         [(0, "start"), (1, "setup"), (2, "staged"), (3, "z0_handed"), (4, "deltas_in"),
                          (6, "deltas_staged"), (7, "registers_written"), (5, "weights_done")]},
           # the same, split: online-side workgroups (layer-0 weights) and target-side ones (the later layers)
           "layer0_online_side_us": {name: med(bl[:, :nblk // 2, i].max(1)) for i, name in
                                     [(4, "deltas_in"), (6, "deltas_staged"), (7, "registers_written"),
                                      (5, "weights_done")]},
           "layer0_target_side_us": {name: med(bl[:, nblk // 2:, i].max(1)) for i, name in
                                     [(4, "deltas_in"), (6, "deltas_staged"), (7, "registers_written"),
                                      (5, "weights_done")]},
           "target_tail_us": {name: med(tg[:, i]) for i, name in TAIL if i < 5 or 7 <= i < 11},
           "online_tail_us": {name: med(on[:, i]) for i, name in TAIL}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
