#!/usr/bin/env python3
"""Run only bench.train_loop_bench (for kernel traces of the train loop)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
import dronerl_amd._native as nat  # noqa: E402
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--segments", type=int, default=2)
ap.add_argument("--lib", default="", help="alternative library (tools/variants.py)")
args = ap.parse_args()
if args.lib:
    nat.LIB_PATH = os.path.abspath(args.lib)
G, N, E, K = bench.CONFIGS[args.config]
env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
env.reset(seed=0)
r = bench.train_loop_bench(env, args.segments)
print(os.path.basename(nat.LIB_PATH), args.config, f"train loop {r['us_per_step']:.2f} us/step")
