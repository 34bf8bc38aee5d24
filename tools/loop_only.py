#!/usr/bin/env python3
"""Run bench.train_loop_bench alone (diagnostic, e.g. under rocprofv3 --kernel-trace).

python tools/loop_only.py [--config c3] [--segments 3] [--input code|obs] [--precision f32] [--lib var.so]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--segments", type=int, default=3)
    ap.add_argument("--input", default="code", choices=("code", "obs"))
    ap.add_argument("--precision", default="f32", choices=("f32", "bf16"))
    ap.add_argument("--lib", default="", help="alternative library (tools/variants.py)")
    ap.add_argument("--refill-branch", action="store_true", help="A/B: the refill on its own graph branch")
    ap.add_argument("--synth-in-act", action="store_true",
                    help="A/B: the act writes drones 1..N-1's synthetic columns (drl_qnet_act_synth) instead of the "
                    "step drawing them (drl_step_code_replay_synth, the default)")
    ap.add_argument("--synth-branch", action="store_true",
                    help="A/B: synthetic actions unfused, on their own graph branch beside the learner")
    args = ap.parse_args()
    if args.lib:
        import dronerl_amd._native as nat
        nat.LIB_PATH = os.environ["DRL_LIB"] = os.path.abspath(args.lib)
    G, N, E = bench.CONFIGS[args.config][:3]
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    r = bench.train_loop_bench(env, args.segments, precision=args.precision, input=args.input,
                               refill_branch=args.refill_branch, synth_branch=args.synth_branch,
                               fused=not args.synth_branch, synth_in_step=False if args.synth_in_act else None)
    print(json.dumps({k: r[k] for k in ("us_per_step", "precision", "input")}), flush=True)


if __name__ == "__main__":
    main()
