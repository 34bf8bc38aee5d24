"""Time drl_refill in steady state (tools/, GPU diagnostic).

Per config: reset, two refill cycles of steps, then `reps` times: the
layout's refill_every steps with the cadence off, then one refill timed with
HIP events while the GPU is kept busy (no host gap in the timed span).  The
library is dronerl_amd's, or DRL_LIB's (tools/variants.py builds).
python tools/refill_time.py [--configs c3,c5] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402

CFG = {"c3": (16, 8, 65536), "c4": (32, 16, 65536), "c5": (64, 32, 131072), "c2": (16, 8, 4096)}


def timed_refill(env, s):
    torch.cuda._sleep(200000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    env.refill()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c5")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="wave", help="list (drl_refill_list_kernel, the default), wave (DRL_REFILL_LIST=0: "
                    "drl_refill_kernel); "
                    "each timed on the same state per rep")
    args = ap.parse_args()
    variants = args.variants.split(",")
    s = torch.cuda.current_stream()
    for name in args.configs.split(","):
        G, N, E = CFG[name]
        env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
        env.reset(seed=0)
        every = env.refill_every
        obs = torch.empty((E, 1, 7, 7, 6), device="cuda")
        for t in range(2 * every):
            env.step(env.synth_actions(seed=1, step=t), obs_k=1, obs=obs)
        env.refill_every = 0
        tsv, dry, convs = {v: [] for v in variants}, [], {}
        for r in range(args.reps):
            for t in range(every):
                env.step(env.synth_actions(seed=5, step=1000 + r * every + t), obs_k=1, obs=obs)
            dry.append(float((((env.state.mt_index >> 20) & 1023) == 0).float().mean()))
            # every variant refills the same state (paired: same conversions)
            snap = env.state.clone()
            for v in variants[r % len(variants):] + variants[:r % len(variants)]:
                env.state = snap.clone()
                os.environ["DRL_REFILL_LIST"] = "1" if v == "list" else "0"
                cnt0 = (env.state.mt_index >> 20) & 1023
                tsv[v].append(timed_refill(env, s))
                conv = int((((env.state.mt_index >> 20) & 1023) > cnt0).sum())  # envs whose ring grew
                convs.setdefault(v, []).append(conv)
        os.environ.pop("DRL_REFILL_LIST", None)
        env.check_errors()
        for v, ts in tsv.items():
            print(json.dumps({"config": name, "variant": v, "us_and_converted": [[round(t, 1), c] for t, c in
                                                                                zip(ts, convs[v])]}), flush=True)
            ts.sort()
            med = ts[len(ts) // 2]
            cv = convs[v]
            print(json.dumps({"config": name, "variant": v, "envs": E, "refill_every": every,
                              "refill_us_median": round(med, 2), "refill_us_min": round(ts[0], 2),
                              "refill_us_mean": round(sum(ts) / len(ts), 2),
                              "per_step_us_mean": round(sum(ts) / len(ts) / every, 3),
                              "converted_envs_mean": sum(cv) / len(cv), "converted_envs_min": min(cv),
                              "converted_envs_max": max(cv),
                              "per_step_us": round(med / every, 3), "dry_fraction_mean": sum(dry) / len(dry),
                              "lib": os.environ.get("DRL_LIB", "in-tree")}), flush=True)
        del env, obs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
