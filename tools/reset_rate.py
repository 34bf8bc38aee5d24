#!/usr/bin/env python3
"""Reset-kernel A/B: resets/s per variant and agreement of the resulting state.

python tools/reset_rate.py --configs c3,c4,c5 --variants lane,wave,wave_fy64,wave_fy99999
lane = drl_reset_kernel (lane per env); wave = drl_reset_wave_kernel with the
batched shuffle (default: down to si = 1; wave_fyN: only while si >= N;
wave_fy99999 = one draw at a time; wave_serN: at most N i-range writers per
chunk by readlanes, more by the slot table; wave_padN: N more LDS bytes per
wave, a diagnostic of how the rate scales with waves per CU).  Knobs are env variables read per
drl_reset call.  The streams are seeded once with the lane kernel (so a
profiler filtered on drl_reset_wave sees only continuing resets); variants are
timed in interleaved rounds after warm-up resets, and every variant's ground /
drones / MT state after its resets must equal the first variant's.
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from dronerl_amd import BatchedDeliveryDrones, EnvParams  # noqa: E402

KNOBS = ("DRL_RESET_WAVE", "DRL_FY_BATCH_MIN", "DRL_FY_SERIAL", "DRL_RESET_LDS_PAD")


def set_knobs(v):
    for k in KNOBS:
        os.environ.pop(k, None)
    if v == "lane":
        os.environ["DRL_RESET_WAVE"] = "0"
    elif v is not None:
        os.environ["DRL_RESET_WAVE"] = "1"
        if "_fy" in v:
            os.environ["DRL_FY_BATCH_MIN"] = v.split("_fy")[1].split("_")[0]
        if "_ser" in v:
            os.environ["DRL_FY_SERIAL"] = v.split("_ser")[1].split("_")[0]
        if "_pad" in v:
            os.environ["DRL_RESET_LDS_PAD"] = v.split("_pad")[1].split("_")[0]


def snap(env):
    s = env.state
    return [t.clone() for t in (s.ground, s.drones, s.mt, s.mt_index)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c4,c5")
    ap.add_argument("--variants", default="wave,lane")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--envs", type=int, default=0, help="override num_envs")
    ap.add_argument("--reseed", action="store_true", help="also time reset(seed=...) (random.seed per env)")
    args = ap.parse_args()
    variants = args.variants.split(",")
    for cfg in args.configs.split(","):
        G, N, E, _ = CONFIGS[cfg]
        E = args.envs or E
        env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E)
        set_knobs("lane")
        env.reset(seed=0)
        seeded = env.state.clone()
        rates = {v: [] for v in variants}
        reseed = {v: [] for v in variants}
        states = {}
        for _ in range(args.rounds):
            for v in variants:
                env.state = seeded.clone()
                set_knobs(v)
                env.reset(seed=None)  # warm-up (also the state check)
                torch.cuda.synchronize()
                states.setdefault(v, snap(env))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    env.reset(seed=None)
                e1.record()
                torch.cuda.synchronize()
                rates[v].append(E * args.reps / (e0.elapsed_time(e1) / 1e3))
                if args.reseed:
                    e0.record()
                    env.reset(seed=12345)
                    e1.record()
                    torch.cuda.synchronize()
                    reseed[v].append(E / (e0.elapsed_time(e1) / 1e3))
                    states.setdefault(v + "/reseed", snap(env))
        set_knobs(None)
        ref = states[variants[0]]
        for v in variants:
            same = all(torch.equal(a, b) for a, b in zip(ref, states[v]))
            print(f"{cfg} G={G} N={N} E={E} {v:>14}: median {statistics.median(rates[v]):14,.0f}  "
                  f"max {max(rates[v]):14,.0f} resets/s  state==first:{same}", flush=True)
            if args.reseed:
                same = all(torch.equal(a, b) for a, b in zip(states[variants[0] + "/reseed"], states[v + "/reseed"]))
                print(f"{cfg} G={G} N={N} E={E} {v:>14}: reseeding reset {statistics.median(reseed[v]):14,.0f} "
                      f"resets/s  state==first:{same}", flush=True)


if __name__ == "__main__":
    main()
