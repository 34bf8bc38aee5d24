"""ORACLE TOOLING ONLY — times the reference's own torch_impl env in this container.

VERDICT r5 item 8: bench.py's cpu_baseline times the build's C port of the
algorithm on the GPU box's host cores; the reference itself cannot run there
(/root/reference is absent on the box).  This script runs the reference's
torch_impl `DeliveryDrones.step()` (torch_impl/env/env.py:112-215) wrapped in
`WindowedGridView` (wrappers.py:46-73) -- the path north_star names -- with
uniform random actions on one core of this (build) container, for the
benchmark shapes, and writes profiles/r06_reference_torch_impl.json.
bench.py quotes that file as `cpu_baseline.reference_torch_impl`, labelled as
measured on different hardware.

Usage:  python oracle/time_reference_torch_impl.py [--seconds 10]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "gymshim"))
sys.path.insert(0, "/root/reference")

from torch_impl.env.env import DeliveryDrones  # noqa: E402
from torch_impl.env.wrappers import WindowedGridView  # noqa: E402

OUT = os.path.join(REPO, "profiles", "r06_reference_torch_impl.json")
CONFIGS = {"c1": (8, 4), "c3": (16, 8), "c4": (32, 16), "c5": (64, 32)}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def time_config(side: int, n: int, seconds: float, obs: bool) -> dict:
    # drone_density so that env.py:75's side = ceil(sqrt(n / density)) is `side`
    env = DeliveryDrones({"n_drones": n, "drone_density": n / (side * side)})
    if obs:
        env = WindowedGridView(env, radius=3)
    random.seed(0)
    env.reset()
    inner = env.env if obs else env
    assert inner.side_size == side, (inner.side_size, side)
    steps, t0 = 0, time.perf_counter()
    while True:
        for _ in range(100):
            env.step({i: random.randrange(5) for i in range(n)})
        steps += 100
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return {"env_steps_per_s": steps / dt, "steps": steps, "seconds": dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    args = ap.parse_args()
    out = {"what": "reference torch_impl DeliveryDrones.step (+ WindowedGridView radius 3), uniform random actions, "
                   "one env, one core, pure Python (torch_impl/env/env.py:112-215, wrappers.py:46-73)",
           "script": "oracle/time_reference_torch_impl.py",
           "hardware": f"build container, 1 core of {cpu_model()} (NOT the GPU box)",
           "python": platform.python_version(), "cores": 1, "configs": {}}
    for name, (side, n) in CONFIGS.items():
        with_obs = time_config(side, n, args.seconds, True)
        step_only = time_config(side, n, args.seconds / 2, False)
        out["configs"][name] = {"side": side, "n_drones": n, "step_obs_env_steps_per_s": with_obs["env_steps_per_s"],
                                "step_only_env_steps_per_s": step_only["env_steps_per_s"],
                                "timed_steps": with_obs["steps"]}
        print(name, out["configs"][name], flush=True)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
