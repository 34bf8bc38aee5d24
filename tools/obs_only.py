"""Diagnostic: time / profile drl_obs (the standalone observation kernel) at C3."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402

env = BatchedDeliveryDrones(EnvParams(n_drones=8, grid_size=16), 65536)
env.reset(seed=0)
for t in range(20):
    env.step(env.synth_actions(seed=1, step=t))
out = torch.empty((65536, 1, 7, 7, 6), device="cuda")
for _ in range(30):
    env.get_obs(1, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(200000)
e0.record()
for _ in range(50):
    env.get_obs(1, out=out)
e1.record()
torch.cuda.synchronize()
print("drl_obs us", e0.elapsed_time(e1) * 1e3 / 50)
