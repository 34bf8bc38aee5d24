#!/usr/bin/env python3
"""drl_rollout at C3 with per-step output buffers vs one reused buffer (MALL-resident)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import dronerl_amd._native as nat  # noqa: E402
from bench import CONFIGS  # noqa: E402
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
if len(sys.argv) > 2:  # alternative library (tools/variants.py)
    nat.LIB_PATH = os.path.abspath(sys.argv[2])
G, N, E, K = CONFIGS[cfg]
env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
env.reset(seed=0)
T = 100
acts = torch.stack([env.synth_actions(seed=3, step=t) for t in range(T)])
for every in (True, False, True, False):
    env.rollout(acts, obs_k=K, every_step=every)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        env.rollout(acts, obs_k=K, every_step=every)
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.path.basename(nat.LIB_PATH)} {cfg} every_step={every}: {e0.elapsed_time(e1) * 1e3 / (3 * T):.2f} us/step")
