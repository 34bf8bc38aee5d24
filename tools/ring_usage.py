"""Respawn-candidate ring consumption per env over k steps (GPU diagnostic).

After a full refill, steps run without refills; the ring count field of the
mt_index words gives each env's consumption.  Prints mean / p99 / max and the
fraction of envs whose ring ran dry (count 0).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402

CFG = {"c3": (16, 8, 65536), "c4": (32, 16, 65536), "c5": (64, 32, 131072)}
for name, (G, N, E) in CFG.items():
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    for t in range(30):
        env.step(env.synth_actions(seed=1, step=t))
    env.refill_every = 0
    env.refill()
    c0 = ((env.state.mt_index >> 20) & 1023).clone()
    out = {"config": name, "cadence": env.layout.refill_every, "start_mean": float(c0.float().mean())}
    t = 0
    for k in [1, 4, 8, 16, 24, 32, 48]:
        while t < k:
            env.step(env.synth_actions(seed=2, step=t))
            t += 1
        c = (env.state.mt_index >> 20) & 1023
        used = (c0 - c).float()
        out[f"k{k}"] = {"mean": round(float(used.mean()), 2), "p99": float(used.quantile(0.99)),
                        "max": float(used.max()), "dry": float((c == 0).float().mean())}
    print(json.dumps(out), flush=True)
