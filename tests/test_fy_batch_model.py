"""Model check of the batched Fisher-Yates step used by drl_reset_wave_kernel
(`fy_chunk`, dronerl_kernels.hip): a plain-Python restatement of its
algorithm -- one-ballot acceptance when the draw width is uniform over the
chunk (fixed-point iteration otherwise), a bitmap OR with return to detect
repeated j's (in arbitrary lane order, as LDS atomics of one instruction),
ascending readlane passes over the lanes whose j lies in the chunk's own i
range (p chains) and over the repeated-j groups (q), j writes then i writes
-- must leave the list, si and the consumed draw count exactly as
Random.shuffle's one-draw-at-a-time loop (random.py:380-395) does.  (The
kernel itself is checked against the oracle in test_gpu_parity.py; this pins
the algorithm on CPU.)"""
import random

import pytest


def sequential(lst, us, si):
    lst = list(lst)
    for k, u in enumerate(us):
        if si < 1:
            return lst, si, k
        r = u >> (32 - (si + 1).bit_length())
        if r <= si:
            lst[si], lst[r] = lst[r], lst[si]
            si -= 1
    return lst, si, len(us)


def batched(lst, us, si0, order_rng=None, stats=None):
    """fy_chunk over one chunk: lane k holds draw us[k] (l0 = 0, l1 = len(us))."""
    lst, L = list(lst), len(us)
    kb = (si0 + 1).bit_length()
    slo = si0 - (L - 1)
    fast = slo >= 1 and (slo + 1).bit_length() == kb
    if fast:  # uniform draw width: r fixed per lane; bounds t_k in [0, k]
        r = [u >> (32 - kb) for u in us]
        hi = [r[k] <= si0 for k in range(L)]
        lo = [r[k] + k <= si0 for k in range(L)]
        S = hi
        if hi != lo:  # ambiguous lanes: fixed point from the upper bound
            while True:
                t = [sum(S[:k]) for k in range(L)]
                S2 = [r[k] + t[k] <= si0 for k in range(L)]
                if S2 == S:
                    break
                S = S2
            if stats is not None:
                stats["amb"] += 1
        elif stats is not None:
            stats["fast"] += 1
    else:
        S = [True] * L
        while True:
            t = [sum(S[:k]) for k in range(L)]
            s = [si0 - t[k] for k in range(L)]
            rk = [us[k] >> (32 - (max(s[k], 1) + 1).bit_length()) for k in range(L)]
            S2 = [s[k] >= 1 and rk[k] <= s[k] for k in range(L)]
            if S2 == S:
                break
            S = S2
        if stats is not None:
            stats["slow"] += 1
    acc = S
    m = sum(acc)
    si = si0 - m
    consumed = max(k for k in range(L) if acc[k]) + 1 if si == 0 else L
    if m == 0:
        return lst, si, consumed
    t = [sum(acc[:k]) for k in range(L)]
    if not fast:
        r = [us[k] >> (32 - (max(si0 - t[k], 1) + 1).bit_length()) for k in range(L)]
    j, ii = r, [si0 - t[k] for k in range(L)]
    slot = [si0 - j[k] for k in range(L)]
    a0 = [lst[ii[k]] if acc[k] else 0 for k in range(L)]
    l0j = [lst[j[k]] if acc[k] else 0 for k in range(L)]
    # bitmap OR with return, lanes in an arbitrary order
    lanes = [k for k in range(L) if acc[k]]
    if order_rng is not None:
        order_rng.shuffle(lanes)
    seen, dup = set(), [False] * L
    for k in lanes:
        dup[k] = j[k] in seen
        seen.add(j[k])
    A = list(a0)
    for k in range(L):  # ascending writers into the chunk's i range
        if acc[k] and slot[k] < m and slot[k] != t[k]:
            for x in range(L):
                if acc[x] and t[x] == slot[k]:
                    A[x] = A[k]
    B, notlast = list(l0j), set()
    D = [k for k in range(L) if dup[k]]
    while D:  # repeated-j groups, lowest flagged lane first
        jk = j[D[0]]
        G = [x for x in range(L) if acc[x] and j[x] == jk]
        D = [k for k in D if k not in G]
        notlast.update(G[:-1])
        for lo_, hi_ in zip(G, G[1:]):
            B[hi_] = A[lo_]
    for k in range(L):
        if acc[k] and k not in notlast:
            lst[j[k]] = A[k]
    for k in range(L):
        if acc[k]:
            lst[ii[k]] = B[k]
    return lst, si, consumed


def test_batched_fisher_yates_matches_sequential():
    rng = random.Random(7)
    orng = random.Random(8)
    stats = {"fast": 0, "amb": 0, "slow": 0}
    for _ in range(3000):
        n = rng.choice([2, 3, 5, 17, 64, 65, 100, 300, 1000, 4096])
        si = rng.randint(1, n - 1)
        L = rng.randint(1, 64)
        us = [rng.getrandbits(32) for _ in range(L)]
        lst = list(range(n))
        rng.shuffle(lst)
        assert batched(lst, us, si, orng, stats) == sequential(lst, us, si), (n, si, L)
    assert min(stats.values()) > 50, stats  # every acceptance path exercised


def test_repeated_targets_and_i_range_writers():
    """Small lists force many repeated j's and writers into the i range."""
    rng = random.Random(11)
    orng = random.Random(12)
    for _ in range(2000):
        n = rng.choice([66, 70, 80, 96, 128])
        si = rng.randint(64, n - 1)
        us = [rng.getrandbits(32) for _ in range(64)]
        lst = list(range(n))
        assert batched(lst, us, si, orng) == sequential(lst, us, si), (n, si)


@pytest.mark.parametrize("n", [1, 38, 75, 1000, 4096])
def test_chunks_compose_to_random_shuffle(n):
    """Chunk after chunk over a real MT stream == random.shuffle itself."""
    for seed in range(6):
        a = random.Random(seed)
        want = list(range(n))
        a.shuffle(want)
        b = random.Random(seed)
        lst, si = list(range(n)), n - 1
        while si >= 1:
            us = [b.getrandbits(32) for _ in range(64)]
            lst, si, used = batched(lst, us, si, random.Random(seed))
            assert used == 64 or si == 0
            if si == 0 and used < 64:  # the first unconsumed draw is the shuffle's next word
                assert a.getrandbits(32) == us[used]
        assert lst == want

