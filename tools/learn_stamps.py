#!/usr/bin/env python3
"""Diagnostic: per-phase timing of drl_dqn_grad_kernel from wall_clock64
stamps (100 MHz) of a -DDRL_DQN_STAMPS build (tools/var_dqnstamps.so, never
the product library).

python tools/learn_stamps.py [--config c3] [--steps 20] [--build]
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
           "-I", os.path.join(REPO, "include"), "-o", LIB] + b.SOURCES
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--build", action="store_true")
    args = ap.parse_args()
    if args.build:
        build()
        return
    os.environ["DRL_LIB"] = LIB
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
    nblk = lr.layout.grad_workgroups - 2  # (+ the target and online tail workgroups)
    st = lr.block[lr.layout.bytes - 8192:].view(torch.int64)
    rows = []
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for k in range(args.steps):
        st.zero_()
        ev[k][0].record()
        lr.train(loop.rb)
        ev[k][1].record()
        torch.cuda.synchronize()
        s = st.cpu().numpy().astype(np.int64)
        blk = s[:8 * nblk].reshape(nblk, 8)[:, :5]
        tt = s[8 * nblk:8 * nblk + 3]          # target tail: start, setup, prefetch done
        to = s[8 * nblk + 8:8 * nblk + 11]     # online tail
        on = s[512:518]                        # online: wait done, fwd, mx, td, backward, end
        tg = s[520:522]                        # target: wait done, fwd
        t0 = min(blk[:, 0].min(), tt[0], to[0])
        f = lambda x: (x - t0) / 100.0  # noqa: E731
        rows.append({"blocks": f(blk), "tt": f(tt), "to": f(to), "on": f(on), "tg": f(tg),
                     "event_us": ev[k][0].elapsed_time(ev[k][1]) * 1e3})
    med = lambda xs: float(np.median(xs))  # noqa: E731
    bl = np.stack([r["blocks"] for r in rows])
    R = {k: np.stack([r[k] for r in rows]) for k in ("tt", "to", "on", "tg")}
    out = {"config": args.config, "layer0_workgroups": nblk,
           "grad_plus_update_event_us": med([r["event_us"] for r in rows]),
           "layer0_phase_us_median": {name: med(bl[:, :, i + 1] - bl[:, :, i])
                                      for i, name in enumerate(["setup", "stage", "compute", "drain_ticket"])},
           "layer0_start_spread_us": med(bl[:, :, 0].max(1) - bl[:, :, 0].min(1)),
           "last_ticket_us": med(bl[:, :, 4].max(1)),
           "target_tail": {"prefetch_done": med(R["tt"][:, 2]), "wait_done": med(R["tg"][:, 0]),
                           "forward_done": med(R["tg"][:, 1])},
           "online_tail": {"prefetch_done": med(R["to"][:, 2]), "wait_done": med(R["on"][:, 0]),
                           "forward_done": med(R["on"][:, 1]), "target_max_in": med(R["on"][:, 2]),
                           "td_done": med(R["on"][:, 3]), "backward_done": med(R["on"][:, 4]),
                           "end": med(R["on"][:, 5])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
