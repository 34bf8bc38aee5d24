"""ORACLE TOOLING ONLY -- generates tests/golden/reset_states.npz and
tests/golden/mt_kat.npz.

Runs in the build container only (it imports /root/reference, which does not
exist on the GPU box), like oracle/gen_golden.py.

reset_states.npz: for every config below and seeds 0..15, ``random.seed(s);
env.reset()`` of the reference torch_impl env (env.py:68-101) -- ground codes,
drone positions / carry by index (dict order is 0..N-1 after a reset), the
CPython MT index after the reset and a sha256 of the 624 state words.

mt_kat.npz: MT19937 known answers from CPython's own `random` (the stream the
reference draws from): the first 16 getrandbits(32) for seeds 0..3,
getrandbits(k) for k = 1..8, randint(0, G-1) for G in {5,7,8,11,13,16,32,64},
a shuffle and a sample (both branches) per seed.

Usage:  python oracle/gen_reset_mt_golden.py
"""
from __future__ import annotations

import hashlib
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import OUT, full_params, snapshot  # noqa: E402  (imports the reference with the gym shim)

from torch_impl.env.env import DeliveryDrones  # noqa: E402

# name: (n_drones, drone_density) -> side = ceil(sqrt(n / density)) (env.py:75)
CONFIGS = {
    "c1_g8_n4": (4, 4 / 64), "c3_g16_n8": (8, 8 / 256), "c4_g32_n16": (16, 16 / 1024),
    "c5_g64_n32": (32, 32 / 4096), "t_g5_n1": (1, 0.05), "t_g7_n2": (2, 0.05), "t_g11_n6": (6, 0.05),
    "t_g13_n8": (8, 0.05),
}
SEEDS = list(range(16))


def mt_digest(words) -> bytes:
    return hashlib.sha256(np.asarray(words[:624], dtype="<u4").tobytes()).digest()


def gen_resets():
    out = {}
    for name, (n, dens) in CONFIGS.items():
        env = DeliveryDrones(full_params(n_drones=n, drone_density=dens))
        G = env.side_size
        ground = np.zeros((len(SEEDS), G, G), np.uint8)
        y = np.zeros((len(SEEDS), n), np.uint8)
        x = np.zeros((len(SEEDS), n), np.uint8)
        pk = np.zeros((len(SEEDS), n), bool)
        mtidx = np.zeros(len(SEEDS), np.int32)
        dig = np.zeros((len(SEEDS), 32), np.uint8)
        for k, s in enumerate(SEEDS):
            random.seed(s)
            env.reset()
            g, order, yy, xx, _, p = snapshot(env)
            assert list(order) == list(range(n))
            ground[k], y[k], x[k], pk[k] = g, yy, xx, p
            st = random.getstate()[1]
            mtidx[k] = st[624]
            dig[k] = np.frombuffer(mt_digest(st), np.uint8)
        out[f"{name}__side"] = np.int32(G)
        out[f"{name}__n"] = np.int32(n)
        out[f"{name}__ground"], out[f"{name}__y"], out[f"{name}__x"] = ground, y, x
        out[f"{name}__packet"], out[f"{name}__mtidx"], out[f"{name}__mtsha"] = pk, mtidx, dig
    out["seeds"] = np.array(SEEDS, np.int64)
    np.savez_compressed(os.path.join(OUT, "reset_states.npz"), **out)


def gen_mt_kat():
    seeds = [0, 1, 2, 3]
    sides = [5, 7, 8, 11, 13, 16, 32, 64]
    first16 = np.zeros((4, 16), np.uint32)
    bits = np.zeros((4, 8), np.uint32)
    rint = np.zeros((4, len(sides), 16), np.int32)
    shuf = np.zeros((4, 100), np.int32)
    samp_set = np.zeros((4, 8), np.int32)   # sample(range(300), 8): set branch (n > setsize 85)
    samp_pool = np.zeros((4, 4), np.int32)  # sample(range(13), 4): pool branch (n <= setsize 21)
    for i, s in enumerate(seeds):
        r = random.Random(s)
        first16[i] = [r.getrandbits(32) for _ in range(16)]
        r = random.Random(s)
        bits[i] = [r.getrandbits(k) for k in range(1, 9)]
        for gi, G in enumerate(sides):
            r = random.Random(s)
            rint[i, gi] = [r.randint(0, G - 1) for _ in range(16)]
        r = random.Random(s)
        lst = list(range(100))
        r.shuffle(lst)
        shuf[i] = lst
        r = random.Random(s)
        samp_set[i] = r.sample(range(300), 8)
        r = random.Random(s)
        samp_pool[i] = r.sample(range(13), 4)
    np.savez_compressed(os.path.join(OUT, "mt_kat.npz"), seeds=np.array(seeds), first16=first16, bits1_8=bits,
                        sides=np.array(sides), randint=rint, shuffle100=shuf, sample_set_300_8=samp_set,
                        sample_pool_13_4=samp_pool)


if __name__ == "__main__":
    gen_resets()
    gen_mt_kat()
    print("wrote", os.path.join(OUT, "reset_states.npz"), "and mt_kat.npz")
