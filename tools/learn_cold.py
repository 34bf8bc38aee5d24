#!/usr/bin/env python3
"""Diagnostic: the learner launch (drl_dqn_train) with warm caches, after a
256 MB overwrite (code and data cold, as after the loop's step), and after the
overwrite followed by a read of the learner's data (agent block, packed net,
ring rows: data warm, the kernel's code still cold).  Per-launch HIP events,
median over --iters launches.

python tools/learn_cold.py [--config c3] [--iters 40]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=40)
    args = ap.parse_args()
    import torch
    import bench
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    G, N, E = bench.CONFIGS[args.config][:3]
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    loop = bench.TrainSegment(env, 2, input="code")
    for t in range(3):
        loop._act_step(t)
        loop._replay(t)
        loop._learn()
    torch.cuda.synchronize()
    lr, rb, net = loop.learner, loop.rb, loop.net
    junk = torch.empty(64 << 20, dtype=torch.float32, device="cuda")
    sink = torch.empty(4, dtype=torch.float32, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(prep):
        ts = []
        for i in range(args.iters):
            prep(i)
            e0.record()
            lr.train(rb)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        lr.check_errors()
        return statistics.median(ts)

    def warm_data():
        sink[0] = lr.block.view(torch.float32).sum()
        sink[1] = net.packed.view(torch.float32)[: net.packed.numel() // 4].sum()
        sink[2] = rb.obs.view(torch.float32).sum() + rb.next_obs.view(torch.float32).sum()

    out = {"config": args.config,
           "warm_us": run(lambda i: None),
           "flushed_us": run(lambda i: junk.fill_(float(i))),
           "flushed_then_data_read_us": run(lambda i: (junk.fill_(float(i)), warm_data())),
           "data_read_only_us": run(lambda i: warm_data())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
