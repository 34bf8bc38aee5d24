"""Pin the oracle (oracle/dronerl_oracle.c) before trusting it.

1. Its MT19937 / _randbelow / shuffle / sample against CPython's `random`
   (the stdlib the reference draws from: torch_impl/env/env.py:62,88,229-230).
2. The reference's own golden tests, restated as data (tests/golden/ref_tests.npz):
   test_windowedgridview.py:37-248, test_env_single_drone.py:13-109,
   test_env_multiple_drones.py:15-96.
3. Seeded trajectories of the reference itself (tests/golden/traj_*.npz,
   oracle/gen_golden.py): state, dict order, rewards (exact doubles), dones,
   MT index and observation windows, every step.
4. The RNG-free known-answer cases of jax_tests/test_env.py restated in
   torch_impl semantics.
"""
import random

import numpy as np
import pytest

from oracle.oracle import MT, OracleEnv, Params
from tests._golden import load_ref_tests, load_traj, oracle_params, traj_names


@pytest.mark.parametrize("seed", [0, 1, 7, 845, 2**31 - 1, 2**32, 2**40 + 3, 2**64 - 16, 2**64 - 1])
def test_mt_matches_cpython(seed):
    r, m = random.Random(seed), MT(seed)
    assert [r.getrandbits(32) for _ in range(1500)] == [m.genrand() for _ in range(1500)]
    for n in [1, 2, 3, 5, 8, 11, 16, 64, 100, 4096]:
        assert [r.randint(0, n - 1) for _ in range(50)] == [m.randint(0, n - 1) for _ in range(50)]
    for k in range(1, 33):
        assert r.getrandbits(k) == m.getrandbits(k)
    a = list(range(777))
    r.shuffle(a)
    assert a == m.shuffle(list(range(777)))
    for n, k in [(13, 4), (19, 2), (21, 5), (22, 1), (76, 8), (85, 10), (86, 10), (232, 8), (277, 64), (400, 64)]:
        pop = list(range(5, 5 + n))
        assert r.sample(pop, k) == m.sample(pop, k), (n, k)
    assert list(r.getstate()[1]) == m.getstate_words().tolist()


def _env_from_ref_params(n, charge_reward=-0.1, density=0.05):
    import math
    side = int(math.ceil(math.sqrt(n / density)))
    return OracleEnv(Params(side=side, n_drones=n, charge_reward=charge_reward))


def test_ref_windowedgridview():
    """test_windowedgridview.py:37-248 — seed 0, 2 drones, 3 scripted steps."""
    g = load_ref_tests()
    env = _env_from_ref_params(2, charge_reward=0.0)
    env.seed(0)
    env.reset()
    for t, a in enumerate(g["wgv_actions"]):
        env.step(a)
        ob = env.obs(radius=3, k=1)[0]
        np.testing.assert_array_equal(ob, g["wgv_windows"][t])


def test_ref_single_drone():
    """test_env_single_drone.py:13-109 (pickups at 3/8, deliveries 7/10, crash 13, battery death 23)."""
    g = load_ref_tests()
    env = _env_from_ref_params(1, charge_reward=0.0)
    env.seed(0)
    env.reset()
    for t, a in enumerate(g["single_actions"]):
        r, _ = env.step([a])
        s = env.state()
        assert s["charge"][0] == g["single_charge"][t]
        assert s["packet"][0] == g["single_carry"][t]
        assert r[0] == g["single_reward"][t]
    # the script's own asserted values
    assert g["single_carry"][3] and g["single_charge"][3] == 80
    assert not g["single_carry"][7] and g["single_charge"][7] == 70 and g["single_reward"][7] == 1
    assert g["single_charge"][13] == 100 and g["single_reward"][13] == -1
    assert g["single_charge"][23] == 100 and g["single_reward"][23] == -1


def test_ref_multiple_drones():
    """test_env_multiple_drones.py:15-96 (gym-PCG64 random actions captured)."""
    g = load_ref_tests()
    env = _env_from_ref_params(8)
    env.seed(0)
    env.reset()
    for t, a in enumerate(g["multi_actions"]):
        r, d = env.step(a)
        s = env.state()
        np.testing.assert_array_equal(s["charge"], g["multi_charge"][t])
        np.testing.assert_array_equal(s["packet"], g["multi_carry"][t])
        np.testing.assert_array_equal(r, g["multi_reward"][t])
        np.testing.assert_array_equal(d, g["multi_done"][t])
    assert g["multi_charge"][3].tolist() == [90, 60, 100, 60, 60, 60, 100, 60]
    assert g["multi_carry"][7].astype(int).tolist() == [0, 0, 0, 1, 1, 0, 0, 0]


def check_oracle_traj(name):
    d = load_traj(name)
    p = oracle_params(d)
    E, S, N = d["actions"].shape
    obs_steps = list(d["obs_steps"])
    for e in range(E):
        env = OracleEnv(p)
        env.seed(int(d["seeds"][e]))
        assert env.state()["mt"].tolist()[:624] == d["mt0"][e][:624].tolist()
        env.reset()
        for t in range(S + 1):
            if t > 0:
                r, dn = env.step(d["actions"][e, t - 1])
                np.testing.assert_array_equal(r, d["rewards"][e, t - 1])
                np.testing.assert_array_equal(dn, d["dones"][e, t - 1])
            s = env.state()
            ctx = f"{name} env {e} step {t}"
            np.testing.assert_array_equal(s["ground"], d["ground"][e, t], ctx)
            np.testing.assert_array_equal(s["order"], d["order"][e, t], ctx)
            np.testing.assert_array_equal(s["y"], d["y"][e, t], ctx)
            np.testing.assert_array_equal(s["x"], d["x"][e, t], ctx)
            np.testing.assert_array_equal(s["charge"], d["charge"][e, t], ctx)
            np.testing.assert_array_equal(s["packet"], d["packet"][e, t], ctx)
            assert s["mt"][624] == d["mtidx"][e, t], ctx
            if t in obs_steps:
                np.testing.assert_array_equal(env.obs(3), d["obs"][e, obs_steps.index(t)], ctx)


@pytest.mark.parametrize("name", traj_names())
def test_oracle_matches_reference_trajectory(name):
    check_oracle_traj(name)


# ---- jax_tests/test_env.py RNG-free known answers, torch_impl semantics ------
def _hand_env(n, G=8, charge=None):
    env = OracleEnv(Params(side=G, n_drones=n))
    env.seed(0)
    return env


def _set(env, ys, xs, ground=None, charge=None, packet=None):
    n = len(ys)
    G = env.p.side
    ground = np.zeros((G, G), np.uint8) if ground is None else ground
    env.set_state(ground, list(range(n)), ys, xs, charge or [100] * n, packet or [0] * n)


def test_kat_single_movements():
    """jax test_env.py:230-239: start (x=3,y=3); LEFT, DOWN, RIGHT, UP, STAY."""
    for a, (x, y) in zip(range(5), [(2, 3), (3, 4), (4, 3), (3, 2), (3, 3)]):
        env = _hand_env(1)
        _set(env, [3], [3])
        env.step([a])
        s = env.state()
        assert (s["x"][0], s["y"][0]) == (x, y)


def test_kat_collisions():
    """jax test_env.py:220-227: drones (x=1,y=3),(x=3,y=3) RIGHT/LEFT collide."""
    env = _hand_env(2)
    _set(env, [3, 3], [1, 3])
    r, d = env.step([2, 0])
    assert d.sum() == 2 and env.state()["charge"].sum() == 200
    assert (r == -1).all()


def test_kat_skyscrapers():
    """jax test_env.py:187-195: one drone into a skyscraper, one off the board."""
    env = _hand_env(2)
    g = np.zeros((8, 8), np.uint8)
    g[3, 4] = 2
    _set(env, [3, 3], [3, 0], ground=g)
    r, d = env.step([2, 0])
    assert d.sum() == 2 and r.sum() == -2
    assert env.state()["ground"][3, 4] == 2


def test_kat_charge_step1():
    """jax test_env.py:150-162 (first step)."""
    env = _hand_env(3)
    g = np.zeros((8, 8), np.uint8)
    g[3, 4] = 3
    _set(env, [0, 3, 0], [3, 3, 0], ground=g, charge=[50, 50, 10])
    r, d = env.step([2, 2, 2])
    s = env.state()
    assert s["charge"].tolist() == [40, 70, 100]
    assert d.tolist() == [False, False, True]
    assert r[0] == 0 and r[1] == -0.1 and r[2] == -1


def test_kat_packages():
    """jax test_env.py:199-217 (minus the threefry-dependent respawn cell)."""
    env = _hand_env(1)
    g = np.zeros((8, 8), np.uint8)
    g[3, 4], g[3, 5] = 5, 4
    _set(env, [3], [3], ground=g)
    r, _ = env.step([2])
    s = env.state()
    assert s["packet"][0] and s["x"][0] == 4 and s["y"][0] == 3 and s["ground"][3, 4] == 0 and r[0] == 0
    r, _ = env.step([2])
    s = env.state()
    assert not s["packet"][0] and s["x"][0] == 5 and r[0] == 1
    assert (s["ground"] > 0).sum() == 2  # one packet + one dropzone respawned


def test_kat_get_obs():
    """jax test_env.py:242-318 (get_obs, get_obs_v2, comprehensive), torch ch1 rule."""
    env = _hand_env(1)
    g = np.zeros((8, 8), np.uint8)
    g[3, 4], g[3, 5] = 5, 4
    _set(env, [3], [3], ground=g)
    for rad in [2, 3, 4]:
        o = env.obs(rad)
        assert o.shape == (1, 2 * rad + 1, 2 * rad + 1, 6)
        assert o[0, rad, rad, 0] == 1 and o[0, rad, rad + 1, 1] == 1 and o[0, rad, rad + 2, 2] == 1
    env = _hand_env(2)
    g = np.zeros((8, 8), np.uint8)
    g[2, 6] = g[6, 6] = 5
    g[1, 3] = g[2, 3] = 3
    g[6, 3] = 4
    g[0, 0] = 2
    _set(env, [3, 3], [1, 3], ground=g, charge=[80, 60], packet=[1, 0])
    o, R = env.obs(3), 3
    assert o[0, R, R, 0] == 1 and o[0, R, R + 2, 0] == 1
    assert o[0, R, R, 1] == 1 and o[1, R, R, 1] == 0
    assert o[1, 2, 6, 1] == 1 and o[1, 6, 6, 1] == 1
    assert o[0, R, R, 4] == np.float32(0.8) and o[1, R, R, 4] == np.float32(0.6)
    assert o[0, 0, 2, 5] == 1 and (o[0, :, :2, 5] == 1).all()
    assert o[0, :, :, 0].sum() == 2
    assert (o[:, :, :, 1:4].sum(-1) <= 1).all()
    for d in range(2):
        assert o[d, R, R, 5] == 0 and (o[d, :, :, 4] > 0).sum() == 2


@pytest.mark.parametrize("n,G", [(3, 8), (8, 16), (4, 8)])
def test_reset_object_counts(n, G):
    """jax test_env.py:117-133 restated: counts per object type after reset."""
    for seed in range(20):
        env = OracleEnv(Params(side=G, n_drones=n))
        env.seed(seed)
        env.reset()
        s = env.state()
        gr = s["ground"]
        assert (gr == 2).sum() == 3 * n and (gr == 3).sum() == 2 * n and (gr == 4).sum() == 2 * n
        assert (gr == 5).sum() + s["packet"].sum() == 3 * n
        assert (s["charge"] == 100).all()
        assert len(set(zip(s["y"].tolist(), s["x"].tolist()))) == n


def test_charge_div_true_division():
    """wrappers.py:18 stores (double)c/100 into an f32 grid; the f32 true
    division (float)c/100.0f that the HIP kernel uses is identical for every
    reachable charge 0..100 (the reciprocal multiply is not)."""
    c = np.arange(0, 101)
    ref = (c.astype(np.float64) / 100).astype(np.float32)
    assert (c.astype(np.float32) / np.float32(100) == ref).all()


def full_grid_delivery_state(G=4):
    """A delivery on a grid whose every other cell holds an object: the packet
    respawn takes the freed dropzone cell, and the dropzone respawn then finds
    no free cell, where the reference's _find_respawn_position
    (env.py:226-233) loops forever.  Drone 0 at (0,0) carries a packet and
    moves RIGHT onto the dropzone at (0,1)."""
    ground = np.full((G, G), 3, np.uint8)  # stations everywhere
    ground[0, 1] = 4                       # one dropzone
    return dict(ground=ground, order=[0], y=[0], x=[0], charge=[50], packet=[1]), [2]


def test_full_grid_respawn_detected_not_hung():
    from oracle.oracle import NoFreeCell
    st, act = full_grid_delivery_state()
    env = OracleEnv(Params(side=4, n_drones=1))
    env.seed(0)
    env.set_state(st["ground"], st["order"], st["y"], st["x"], st["charge"], st["packet"])
    with pytest.raises(NoFreeCell):
        env.step(np.array(act, np.int32))


# ---- C-3 items 3 and 4: committed reset states (seeds 0..15 per config) and
# MT19937 known answers, both generated from the reference / CPython
# (oracle/gen_reset_mt_golden.py), so the box-side checks need neither.
def test_mt_known_answers_fixture():
    from tests._golden import load_npz
    k = load_npz("mt_kat.npz")
    for i, s in enumerate(k["seeds"]):
        m = MT(int(s))
        assert [m.genrand() for _ in range(16)] == k["first16"][i].tolist()
        m = MT(int(s))
        assert [m.getrandbits(b) for b in range(1, 9)] == k["bits1_8"][i].tolist()
        for gi, G in enumerate(k["sides"]):
            m = MT(int(s))
            assert [m.randint(0, int(G) - 1) for _ in range(16)] == k["randint"][i, gi].tolist()
        assert MT(int(s)).shuffle(list(range(100))) == k["shuffle100"][i].tolist()
        assert MT(int(s)).sample(list(range(300)), 8) == k["sample_set_300_8"][i].tolist()
        assert MT(int(s)).sample(list(range(13)), 4) == k["sample_pool_13_4"][i].tolist()


@pytest.mark.parametrize("name", ["c1_g8_n4", "c3_g16_n8", "c4_g32_n16", "c5_g64_n32", "t_g5_n1", "t_g7_n2",
                                  "t_g11_n6", "t_g13_n8"])
def test_reset_states_fixture(name):
    from oracle.oracle import OracleMulti
    from tests._golden import load_npz, mt_sha
    d = load_npz("reset_states.npz")
    G, N = int(d[f"{name}__side"]), int(d[f"{name}__n"])
    seeds = d["seeds"]
    o = OracleMulti(Params(side=G, n_drones=N), len(seeds))
    o.reset(seeds)
    st = o.state()
    np.testing.assert_array_equal(st["ground"], d[f"{name}__ground"])
    np.testing.assert_array_equal(st["y"], d[f"{name}__y"])
    np.testing.assert_array_equal(st["x"], d[f"{name}__x"])
    np.testing.assert_array_equal(st["packet"], d[f"{name}__packet"])
    np.testing.assert_array_equal(st["order"], np.tile(np.arange(N), (len(seeds), 1)))
    np.testing.assert_array_equal(st["mt"][:, 624], d[f"{name}__mtidx"])
    for e in range(len(seeds)):
        np.testing.assert_array_equal(mt_sha(st["mt"][e]), d[f"{name}__mtsha"][e])
