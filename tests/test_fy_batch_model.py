"""Model check of the batched Fisher-Yates step used by drl_reset_wave_kernel
(`fy_chunk`, dronerl_kernels.hip): a plain-Python restatement of its
algorithm -- ballot fixed point for acceptance, epoch tables for the i-slot
writers (p) and the double-hashed j writers (q), readlane loop over the
lanes that lose in both buckets, j writes then i writes -- must leave the list,
si and the consumed draw count exactly as Random.shuffle's one-draw-at-a-time
loop (random.py:380-395) does.  Bucket counts of 1 and 2 force the exact
collision path.  (The kernel itself is checked against the oracle in
test_gpu_parity.py; this pins the algorithm on CPU.)"""
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


def batched(lst, us, si0, nb):
    """fy_chunk over one chunk: lane k holds draw us[k]; nb buckets per hash."""
    lst, L = list(lst), len(us)
    S = [True] * L
    while True:  # acceptance fixed point
        t = [sum(S[:k]) for k in range(L)]
        s = [si0 - t[k] for k in range(L)]
        r = [us[k] >> (32 - (max(s[k], 1) + 1).bit_length()) for k in range(L)]
        acc = [s[k] >= 1 and r[k] <= s[k] for k in range(L)]
        if acc == S:
            break
        S = acc
    m = sum(S)
    if m == 0:
        return lst, si0, L
    j, ii = r, [si0 - t[k] for k in range(L)]
    a0 = [lst[ii[k]] if acc[k] else 0 for k in range(L)]
    l0j = [lst[j[k]] if acc[k] else 0 for k in range(L)]
    sh = max(1, nb.bit_length() - 1)
    h1 = lambda v: v % nb  # noqa: E731
    h2 = lambda v: ((v * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - sh) if nb > 1 else 0  # noqa: E731
    H1, H2, P = {}, {}, {}
    for k in range(L):
        if acc[k]:
            H1[h1(j[k])] = max(H1.get(h1(j[k]), -1), k)
            H2[h2(j[k])] = max(H2.get(h2(j[k]), -1), k)
            slot = si0 - j[k]
            if slot < m and slot != t[k]:
                P[slot] = max(P.get(slot, -1), k)
    p = [P.get(t[k], -1) if acc[k] else -1 for k in range(L)]
    f = [p[k] if p[k] >= 0 else k for k in range(L)]
    while True:  # pointer jumping to the chain roots
        f2 = [f[f[k]] for k in range(L)]
        if f2 == f:
            break
        f = f2
    A = [a0[f[k]] for k in range(L)]
    q, notlast = [-1] * L, set()
    for k in [k for k in range(L) if acc[k] and H1[h1(j[k])] != k and H2[h2(j[k])] != k]:
        later = [x for x in range(k + 1, L) if acc[x] and j[x] == j[k]]
        if later:
            notlast.add(k)
            for x in later:
                q[x] = k
    B = [A[q[k]] if q[k] >= 0 else l0j[k] for k in range(L)]
    for k in range(L):
        if acc[k] and k not in notlast:
            lst[j[k]] = A[k]
    for k in range(L):
        if acc[k]:
            lst[ii[k]] = B[k]
    si = si0 - m
    return lst, si, (max(k for k in range(L) if S[k]) + 1 if si == 0 else L)


@pytest.mark.parametrize("nb", [1, 2, 256])
def test_batched_fisher_yates_matches_sequential(nb):
    rng = random.Random(nb)
    for _ in range(1500):
        n = rng.choice([2, 3, 5, 17, 64, 65, 100, 300, 1000, 4096])
        si = rng.randint(1, n - 1)
        L = rng.randint(1, 64)
        us = [rng.getrandbits(32) for _ in range(L)]
        lst = list(range(n))
        rng.shuffle(lst)
        assert batched(lst, us, si, nb) == sequential(lst, us, si), (n, si, L)


def test_chunks_compose_to_random_shuffle():
    """Chunk after chunk over a real MT stream == random.shuffle itself."""
    for seed in range(20):
        n = 1 + seed * 37
        a = random.Random(seed)
        want = list(range(n))
        a.shuffle(want)
        b = random.Random(seed)
        lst, si = list(range(n)), n - 1
        while si >= 1:
            us = [b.getrandbits(32) for _ in range(64)]
            lst, si, used = batched(lst, us, si, 256)
            assert used == 64 or si == 0
            if si == 0 and used < 64:  # the first unconsumed draw is the shuffle's next word
                assert a.getrandbits(32) == us[used]
        assert lst == want
