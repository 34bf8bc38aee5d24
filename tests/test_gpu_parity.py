"""GPU parity: libdronerl.so (HIP, gfx950) vs the oracle and the reference's fixtures.

Bar (BASELINE.json north_star): grid state, dict order, done flags and the MT
stream bit-exact; rewards equal to float32(reference double) (|err| <= 1e-6
as stated, in practice 0); observations bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle.oracle import OracleMulti, Params as OParams
from tests._golden import load_ref_tests, load_traj, traj_names, traj_params

pytestmark = pytest.mark.gpu

REWARD_ATOL = 1e-6  # north_star tolerance for float rewards


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dronerl_amd._native import lib
    lib()  # must load: no fallback


def EnvParams(**kw):
    from dronerl_amd import EnvParams as P
    return P(**kw)


def Env(p, E, **kw):
    from dronerl_amd import BatchedDeliveryDrones
    return BatchedDeliveryDrones(p, E, **kw)


def oparams(p) -> OParams:
    return OParams(side=p.side, n_drones=p.n_drones, charge=p.charge, discharge=p.discharge,
                   packets_factor=p.packets_factor, dropzones_factor=p.dropzones_factor,
                   stations_factor=p.stations_factor, skyscrapers_factor=p.skyscrapers_factor,
                   pickup_reward=p.pickup_reward, delivery_reward=p.delivery_reward, crash_reward=p.crash_reward,
                   charge_reward=p.charge_reward)


def gpu_state(env, envs=None):
    d = env.decode()
    out = {k: d[k] for k in ["ground", "order", "y", "x", "charge", "carrying"]}
    out["mt"] = env.mt_words_device()  # the stream's getstate() words (drl_mt_get)
    if envs is not None:
        idx = torch.as_tensor(envs, device=env.device)
        out = {k: v.index_select(0, idx) for k, v in out.items()}
    out = {k: v.cpu().numpy() for k, v in out.items()}
    out["packet"] = out.pop("carrying").astype(bool)
    out["mt"] = out["mt"].astype(np.uint32)
    return out


def assert_state(g, o, ctx, mt_full=True):
    for k in ["ground", "order", "y", "x", "charge", "packet"]:
        if not np.array_equal(g[k], o[k]):
            bad = np.argwhere(np.asarray(g[k] != o[k]).reshape(len(g[k]), -1).any(1)).ravel()
            raise AssertionError(f"{ctx}: '{k}' differs in envs {bad[:10]} (of {len(bad)})")
    if mt_full:
        np.testing.assert_array_equal(g["mt"], o["mt"], err_msg=f"{ctx}: mt")
    else:
        np.testing.assert_array_equal(g["mt"][:, 624], o["mt"][:, 624], err_msg=f"{ctx}: mt index")


def assert_rewards(rg, ro, ctx):
    rg = np.asarray(rg, dtype=np.float32)
    np.testing.assert_array_equal(rg, ro.astype(np.float32), err_msg=f"{ctx}: rewards vs f32(ref)")
    assert np.abs(rg.astype(np.float64) - ro).max(initial=0) <= REWARD_ATOL


# --------------------------------------------------------------- fixtures --
@pytest.mark.parametrize("name", traj_names())
def test_reference_trajectory_on_gpu(name):
    """Replay the reference's own seeded trajectories (oracle/gen_golden.py)."""
    d = load_traj(name)
    tp = traj_params(d)
    p = EnvParams(n_drones=tp["n_drones"], grid_size=int(d["side"]), pickup_reward=tp["pickup_reward"],
                  delivery_reward=tp["delivery_reward"], crash_reward=tp["crash_reward"],
                  charge_reward=tp["charge_reward"], discharge=tp["discharge"], charge=tp["charge"],
                  packets_factor=tp["packets_factor"], dropzones_factor=tp["dropzones_factor"],
                  stations_factor=tp["stations_factor"], skyscrapers_factor=tp["skyscrapers_factor"])
    E, S, N = d["actions"].shape
    env = Env(p, E)
    env.set_mt_words(d["mt0"])           # random.seed(s) words, as captured from CPython
    env.reset(seed=None)                 # then env.reset() continues that stream
    obs_steps = list(d["obs_steps"])
    acts = torch.as_tensor(d["actions"].astype(np.int32)).cuda()
    for t in range(S + 1):
        if t > 0:
            want_obs = t in obs_steps
            out = env.step(acts[:, t - 1].contiguous(), obs_k=N if want_obs else 0)
            r, dn = out[0].cpu().numpy(), out[1].cpu().numpy().astype(bool)
            assert_rewards(r, d["rewards"][:, t - 1], f"{name} step {t}")
            np.testing.assert_array_equal(dn, d["dones"][:, t - 1], err_msg=f"{name} step {t} dones")
            if want_obs:
                np.testing.assert_array_equal(out[2].cpu().numpy(), d["obs"][:, obs_steps.index(t)],
                                              err_msg=f"{name} step {t} fused obs")
        g = gpu_state(env)
        ref = dict(ground=d["ground"][:, t], order=d["order"][:, t], y=d["y"][:, t], x=d["x"][:, t],
                   charge=d["charge"][:, t], packet=d["packet"][:, t],
                   mt=np.zeros((E, 625), np.uint32))
        ref["mt"][:, 624] = d["mtidx"][:, t]
        assert_state(g, ref, f"{name} step {t}", mt_full=False)
        if t in obs_steps:
            np.testing.assert_array_equal(env.get_obs().cpu().numpy(), d["obs"][:, obs_steps.index(t)],
                                          err_msg=f"{name} step {t} obs")
    env.check_errors()


@pytest.mark.parametrize("name", ["c2_g16_n8", "t_g11_n6", "t_pool_n2"])
def test_reseed_matches_cpython_seed(name):
    """drl_reset(reseed) == random.seed(s) (init_by_array) for the fixture seeds."""
    d = load_traj(name)
    tp = traj_params(d)
    p = EnvParams(n_drones=tp["n_drones"], grid_size=int(d["side"]), packets_factor=tp["packets_factor"],
                  dropzones_factor=tp["dropzones_factor"], stations_factor=tp["stations_factor"],
                  skyscrapers_factor=tp["skyscrapers_factor"])
    for e, s in enumerate(d["seeds"]):
        env = Env(p, 1)
        env.reset(seed=int(s))
        g = gpu_state(env)
        np.testing.assert_array_equal(g["ground"][0], d["ground"][e, 0])
        np.testing.assert_array_equal(g["y"][0], d["y"][e, 0])
        np.testing.assert_array_equal(g["x"][0], d["x"][e, 0])
        np.testing.assert_array_equal(g["packet"][0], d["packet"][e, 0])
        assert g["mt"][0, 624] == d["mtidx"][e, 0]


# ------------------------------------------------------------ vs oracle ---
CONFIGS = {
    "c1_8x8_n4": dict(n_drones=4, grid_size=8),
    "c2_16x16_n8": dict(n_drones=8, grid_size=16),
    "c4_32x32_n16": dict(n_drones=16, grid_size=32),
    "c5_64x64_n32": dict(n_drones=32, grid_size=64),
    "n1_5x5": dict(n_drones=1, grid_size=5),
    "n3_8x8": dict(n_drones=3, grid_size=8),
    "n6_11x11": dict(n_drones=6, grid_size=11),
    "n33_26x26": dict(n_drones=33, grid_size=26),
    "n64_36x36": dict(n_drones=64, grid_size=36),
    "pool_5x5_n2": dict(n_drones=2, grid_size=5, packets_factor=2, dropzones_factor=1, stations_factor=1),
    "dense_10x10_n8": dict(n_drones=8, grid_size=10, pickup_reward=0.5, charge_reward=-0.25, discharge=15,
                           charge=30),
    "bigside_128_n4": dict(n_drones=4, grid_size=128),
}


RESET_KERNELS = {
    "wave": {},                                                  # default: wave per env, batched shuffle
    "wave_serial": {"DRL_FY_BATCH_MIN": "1000000"},              # wave per env, one draw at a time
    "wave_fy64": {"DRL_FY_BATCH_MIN": "64"},                     # batched only while si >= 64 (no hot loop)
    "wave_ser0": {"DRL_FY_SERIAL": "0"},                         # i-range writers: slot table + pointer jumps
    "wave_ser64": {"DRL_FY_SERIAL": "64"},                       # i-range writers: readlane pass only
    "lane": {"DRL_RESET_WAVE": "0"},                             # lane per env
    "wave_wpb1": {"DRL_RESET_WPB": "1"},                         # 1, 2, 4, 8 envs (waves) per workgroup:
    "wave_wpb2": {"DRL_RESET_WPB": "2"},                         # every drl_reset_wave_kernel instance
    "wave_wpb4": {"DRL_RESET_WPB": "4"},
    "wave_wpb8": {"DRL_RESET_WPB": "8"},
}


@pytest.mark.parametrize("kernel", list(RESET_KERNELS))
@pytest.mark.parametrize("name", list(CONFIGS))
def test_reset_matches_oracle(name, kernel, monkeypatch):
    """Reseeded reset, then two resets continuing the stream (the second one
    starts mid-way through an MT block), on every reset kernel variant."""
    for k, v in RESET_KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    p = EnvParams(**CONFIGS[name])
    E = 300 if kernel == "wave" else 97
    env = Env(p, E)
    env.reset(seed=1000)
    o = OracleMulti(oparams(p), E)
    o.reset(1000 + np.arange(E))
    assert_state(gpu_state(env), o.state(), f"{name} reset")
    for r in range(2):
        env.reset(seed=None)
        o.reset(None)
        assert_state(gpu_state(env), o.state(), f"{name} reset {r + 2}")


@pytest.mark.parametrize("name,E,steps,every", [
    ("c1_8x8_n4", 1, 1000, 1),
    ("c2_16x16_n8", 4096, 300, 25),
    ("c4_32x32_n16", 1024, 150, 30),
    ("c5_64x64_n32", 256, 100, 25),
    ("n1_5x5", 333, 300, 20),
    ("n3_8x8", 500, 300, 20),
    ("n6_11x11", 257, 300, 20),
    ("n33_26x26", 97, 120, 20),
    ("n64_36x36", 65, 120, 20),
    ("pool_5x5_n2", 200, 300, 20),
    ("dense_10x10_n8", 600, 300, 20),
    ("bigside_128_n4", 40, 100, 50),
    # the benchmark shapes again on the runtime-geometry kernel instance
    ("c1_8x8_n4|rt", 64, 300, 50),
    ("c2_16x16_n8|rt", 1024, 200, 25),
    ("c4_32x32_n16|rt", 512, 120, 30),
    ("c5_64x64_n32|rt", 128, 80, 40),
])
def test_rollout_matches_oracle(name, E, steps, every, monkeypatch):
    """Benchmark shapes run compile-time-geometry instances; "|rt" forces the
    runtime-geometry one (DRL_SPECIALIZE=0) on the same shape."""
    name, _, rt = name.partition("|")
    if rt:
        monkeypatch.setenv("DRL_SPECIALIZE", "0")
    p = EnvParams(**CONFIGS[name])
    env = Env(p, E)
    env.reset(seed=7)
    o = OracleMulti(oparams(p), E)
    o.reset(7 + np.arange(E))
    for t in range(1, steps + 1):
        a = env.synth_actions(seed=99, step=t)
        check = (t % every == 0) or t == steps
        out = env.step(a, obs_k=1 if check else 0)
        ro, do = o.step(a.cpu().numpy())
        assert_rewards(out[0].cpu().numpy(), ro, f"{name} step {t}")
        np.testing.assert_array_equal(out[1].cpu().numpy().astype(bool), do, err_msg=f"{name} step {t} dones")
        if check:
            assert_state(gpu_state(env), o.state(), f"{name} step {t}")
            np.testing.assert_array_equal(out[2].cpu().numpy(), o.obs(3, 1), err_msg=f"{name} step {t} obs")
    env.check_errors()


@pytest.mark.parametrize("refill_kernel", ["list", "wave"])
@pytest.mark.parametrize("refill", [0, 1, 3])
@pytest.mark.parametrize("name,E,steps", [
    ("c1_8x8_n4", 256, 120),
    ("c2_16x16_n8", 1024, 150),
    ("dense_10x10_n8", 600, 150),
    ("c4_32x32_n16", 256, 80),
    ("c5_64x64_n32", 96, 60),
    ("bigside_128_n4", 40, 60),
])
def test_candidate_ring_cadence_matches_oracle(name, E, steps, refill, refill_kernel, monkeypatch):
    """The respawn-candidate ring never changes results: topped up every step
    (refill 1), every 3rd, or never after the reset's fill (0: it runs dry and
    every later respawn is drawn from the stream in the step, from the end of
    the ring's last entry, which may lie in the next MT block).  Rewards, dones
    and the full state, MT words included, equal the oracle at every step.
    refill_kernel "list": drl_refill's worklist form (the default), "wave": one
    wave per env (DRL_REFILL_LIST=0)."""
    if refill_kernel == "wave":
        monkeypatch.setenv("DRL_REFILL_LIST", "0")
    p = EnvParams(**CONFIGS[name])
    env = Env(p, E)
    env.refill_every = refill
    env.reset(seed=17)
    o = OracleMulti(oparams(p), E)
    o.reset(17 + np.arange(E))
    for t in range(1, steps + 1):
        a = env.synth_actions(seed=31, step=t)
        r, dn = env.step(a)
        ro, do = o.step(a.cpu().numpy())
        assert_rewards(r.cpu().numpy(), ro, f"{name} refill {refill} step {t}")
        np.testing.assert_array_equal(dn.cpu().numpy().astype(bool), do, err_msg=f"{name} step {t} dones")
        assert_state(gpu_state(env), o.state(), f"{name} refill {refill} step {t}")
    env.check_errors()


@pytest.mark.parametrize("k", [1, 8])
@pytest.mark.parametrize("E", [1, 2, 3, 7, 31, 33, 63, 65, 129, 1001])
def test_ragged_num_envs(E, k):
    p = EnvParams(n_drones=8, grid_size=16)
    env = Env(p, E)
    env.reset(seed=3)
    o = OracleMulti(oparams(p), E)
    o.reset(3 + np.arange(E))
    for t in range(1, 41):
        a = env.synth_actions(seed=5, step=t)
        r, dn, ob = env.step(a, obs_k=k)
        ro, do = o.step(a.cpu().numpy())
        assert_rewards(r.cpu().numpy(), ro, f"E={E} step {t}")
    assert_state(gpu_state(env), o.state(), f"E={E}")
    np.testing.assert_array_equal(ob.cpu().numpy(), o.obs(3, k))
    np.testing.assert_array_equal(env.get_obs(k).cpu().numpy(), o.obs(3, k))


@pytest.mark.parametrize("cfg,E", [(dict(n_drones=8, grid_size=16), 4096), (dict(n_drones=8, grid_size=16), 65),
                                   (dict(n_drones=16, grid_size=32), 300), (dict(n_drones=6, grid_size=11), 129)])
def test_streaming_obs_stores(cfg, E):
    """drl_step_ex(DRL_STEP_OBS_STREAM): identical observation, rewards and
    state to the cached-store step, step after step, and both equal to the
    oracle (rewards and dones every step, the observation every 5th, the
    final state)."""
    p = EnvParams(**cfg)
    envs = [Env(p, E), Env(p, E)]
    for env in envs:
        env.reset(seed=21)
    o = OracleMulti(oparams(p), E)
    o.reset(21 + np.arange(E))
    for t in range(1, 31):
        a = envs[0].synth_actions(seed=8, step=t)
        out = [env.step(a, obs_k=1, obs_stream=s) for env, s in zip(envs, (False, True))]
        for x, y in zip(out[0], out[1]):
            assert torch.equal(x, y), f"step {t}"
        ro, do = o.step(a.cpu().numpy())
        assert_rewards(out[1][0].cpu().numpy(), ro, f"streaming step {t}")
        np.testing.assert_array_equal(out[1][1].cpu().numpy().astype(bool), np.asarray(do).astype(bool))
        if t % 5 == 0:
            np.testing.assert_array_equal(out[1][2].cpu().numpy(), o.obs(p.window_radius, 1))
    assert_state(gpu_state(envs[1]), gpu_state(envs[0]), "streaming vs cached")
    assert_state(gpu_state(envs[1]), o.state(), "streaming vs oracle")
    envs[1].check_errors()


@pytest.mark.parametrize("radius", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("k", [1, 3, 8])
def test_obs_variants(radius, k):
    p = EnvParams(n_drones=8, grid_size=16, window_radius=radius)
    E = 130
    env = Env(p, E)
    env.reset(seed=11)
    o = OracleMulti(oparams(p), E)
    o.reset(11 + np.arange(E))
    for t in range(1, 13):
        a = env.synth_actions(seed=1, step=t)
        _, _, ob = env.step(a, obs_k=k)
        o.step(a.cpu().numpy())
    want = o.obs(radius, k)
    np.testing.assert_array_equal(ob.cpu().numpy(), want)
    np.testing.assert_array_equal(env.get_obs(k).cpu().numpy(), want)


def test_shard_invariance():
    """Two shards with env_offset == one unsharded run (train_jax.py:196-212 semantics)."""
    p = EnvParams(n_drones=8, grid_size=16)
    full = Env(p, 1000)
    halves = [Env(p, 500, env_offset=0), Env(p, 500, env_offset=500)]
    for e in [full] + halves:
        e.reset(seed=42)
    for t in range(1, 61):
        rf, df = full.step(full.synth_actions(seed=8, step=t))
        rh = [h.step(h.synth_actions(seed=8, step=t)) for h in halves]
        assert torch.equal(rf, torch.cat([x[0] for x in rh]))
        assert torch.equal(df, torch.cat([x[1] for x in rh]))
    for k in ["ground", "drones", "mt", "mt_index"]:
        assert torch.equal(getattr(full.state, k), torch.cat([getattr(h.state, k) for h in halves]))


@pytest.mark.parametrize("kernel", ["wave", "lane"])
def test_masked_reset_continues_stream(kernel, monkeypatch):
    for k, v in RESET_KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    p = EnvParams(n_drones=8, grid_size=16)
    E = 200
    env = Env(p, E)
    env.reset(seed=5)
    o = OracleMulti(oparams(p), E)
    o.reset(5 + np.arange(E))
    for t in range(1, 21):
        a = env.synth_actions(seed=2, step=t)
        env.step(a)
        o.step(a.cpu().numpy())
    mask = (torch.arange(E) % 3 == 0).to(torch.uint8)
    env.reset(seed=None, env_mask=mask)
    # oracle: reset (continuing the stream) only the masked envs
    st = o.state()
    o2 = OracleMulti(oparams(p), E)
    o2.set_state(st["ground"], st["order"], st["y"], st["x"], st["charge"], st["packet"], st["mt"])
    sel = np.nonzero(mask.numpy())[0]
    o3 = OracleMulti(oparams(p), len(sel))
    o3.set_state(st["ground"][sel], st["order"][sel], st["y"][sel], st["x"][sel], st["charge"][sel],
                 st["packet"][sel], st["mt"][sel])
    o3.reset(None)
    s3 = o3.state()
    want = {k: v.copy() for k, v in st.items()}
    for k in want:
        want[k][sel] = s3[k]
    assert_state(gpu_state(env), want, "masked reset")


def test_negative_and_bad_actions():
    """Python list indexing: -1..-5 wrap (STAY..LEFT); others raise (flag)."""
    p = EnvParams(n_drones=8, grid_size=16)
    E = 64
    env = Env(p, E)
    env.reset(seed=1)
    o = OracleMulti(oparams(p), E)
    o.reset(1 + np.arange(E))
    g = torch.Generator().manual_seed(0)
    for t in range(30):
        a = torch.randint(-5, 5, (E, 8), generator=g, dtype=torch.int32)
        r, _ = env.step(a.cuda())
        ro, _ = o.step(a.numpy())
        assert_rewards(r.cpu().numpy(), ro, f"neg step {t}")
    assert_state(gpu_state(env), o.state(), "negative actions")
    env.check_errors()
    bad = torch.full((E, 8), 4, dtype=torch.int32)
    bad[3, 2] = 5
    env.step(bad.cuda())
    from dronerl_amd._native import DroneRLError
    with pytest.raises(DroneRLError):
        env.check_errors()


def test_hand_built_states_kat():
    """jax_tests/test_env.py RNG-free known answers (torch semantics) on the GPU."""
    p = EnvParams(n_drones=3, grid_size=8)
    env = Env(p, 1)
    env.reset(seed=0)
    g = np.zeros((8, 8), np.uint8)
    g[3, 4] = 3
    env.set_state(g, [0, 1, 2], [0, 3, 0], [3, 3, 0], [50, 50, 10], [0, 0, 0])
    r, d = env.step(torch.tensor([[2, 2, 2]], dtype=torch.int32))
    s = gpu_state(env)
    assert s["charge"][0].tolist() == [40, 70, 100]
    assert d[0].tolist() == [0, 0, 1]
    assert r[0].tolist() == [0.0, np.float32(-0.1), -1.0]
    # single movements
    p1 = EnvParams(n_drones=1, grid_size=8)
    for a, (x, y) in zip(range(5), [(2, 3), (3, 4), (4, 3), (3, 2), (3, 3)]):
        e1 = Env(p1, 1)
        e1.reset(seed=0)
        e1.set_state(np.zeros((8, 8)), [0], [3], [3], [100], [0])
        e1.step(torch.tensor([[a]], dtype=torch.int32))
        s = gpu_state(e1)
        assert (s["x"][0, 0], s["y"][0, 0]) == (x, y)
    # packages: pickup then delivery, two objects respawned
    e1 = Env(p1, 1)
    e1.reset(seed=0)
    g = np.zeros((8, 8), np.uint8)
    g[3, 4], g[3, 5] = 5, 4
    e1.set_state(g, [0], [3], [3], [100], [0])
    r, _ = e1.step(torch.tensor([[2]], dtype=torch.int32))
    s = gpu_state(e1)
    assert s["packet"][0, 0] and s["ground"][0, 3, 4] == 0 and r.item() == 0
    r, _ = e1.step(torch.tensor([[2]], dtype=torch.int32))
    s = gpu_state(e1)
    assert not s["packet"][0, 0] and r.item() == 1 and (s["ground"][0] > 0).sum() == 2


# Full-size parity over every env (C3-C5) and the C5 train-loop segment are
# in tests/test_gpu_fullsize.py.


# -------------------------------------------------- torch_impl drop-in API ---
def test_compat_reference_golden_scripts():
    """The reference's golden scripts, driven through dronerl_amd.compat exactly
    as they drive torch_impl (set_seed -> reset -> step dicts)."""
    from dronerl_amd.compat import DeliveryDrones, WindowedGridView, set_seed
    g = load_ref_tests()
    base = {'drone_density': 0.05, 'pickup_reward': 0, 'delivery_reward': 1, 'crash_reward': -1,
            'charge_reward': -0.1, 'discharge': 10, 'charge': 20, 'packets_factor': 3, 'dropzones_factor': 2,
            'stations_factor': 2, 'skyscrapers_factor': 3, 'rgb_render_rescale': 1.0}
    # test_windowedgridview.py
    env = WindowedGridView(DeliveryDrones(dict(base, n_drones=2, charge_reward=0.0)), radius=3)
    set_seed(env, 0)
    env.reset()
    for t, a in enumerate(g["wgv_actions"]):
        st, _, _, _, _ = env.step({0: int(a[0]), 1: int(a[1])})
        np.testing.assert_array_equal(st[0].astype(np.float32), g["wgv_windows"][t])
        assert st[0].dtype == np.float64 and st[0].shape == (7, 7, 6)
    # test_env_single_drone.py
    env = WindowedGridView(DeliveryDrones(dict(base, n_drones=1, charge_reward=0.0)), radius=3)
    set_seed(env, 0)
    env.reset()
    for t, a in enumerate(g["single_actions"]):
        _, r, _, _, _ = env.step({0: int(a)})
        d0 = env.drones_list[0]
        assert d0.charge == g["single_charge"][t] and d0.packet == g["single_carry"][t] and r[0] == g["single_reward"][t]
    # test_env_multiple_drones.py (gym-sampled actions captured in the fixture)
    env = WindowedGridView(DeliveryDrones(dict(base, n_drones=8)), radius=3)
    set_seed(env, 0)
    env.reset()
    for t, a in enumerate(g["multi_actions"]):
        _, r, d, _, _ = env.step({i: int(a[i]) for i in range(8)})
        ch = [dr.charge for dr in sorted(env.drones_list, key=lambda z: z.index)]
        assert ch == g["multi_charge"][t].tolist()
        assert [r[i] for i in range(8)] == g["multi_reward"][t].tolist()
    # the action space reproduces gym 0.25.2 sampling (RandomAgent, 8 draws per step)
    from dronerl_amd.compat import Discrete
    sp = Discrete(5)
    sp.seed(0)
    for t in range(len(g["multi_actions"])):
        draws = [sp.sample() for _ in range(8)]
        assert draws[1:] == g["multi_actions"][t][1:].tolist()


def test_gpu_eval_runner_matches_oracle():
    """eval_jax-style sharded evaluation on the GPU env == oracle episodes."""
    from dronerl_amd.distributed import evaluate_sharded, gpu_episode_runner
    from tests.test_distributed import oracle_runner
    p = EnvParams(n_drones=3, grid_size=8)
    g_agent, g_rnd, g_table = evaluate_sharded(gpu_episode_runner(p, 50, 100), num_evals=7)
    o_agent, o_rnd, o_table = evaluate_sharded(oracle_runner(3, 8, 50, 100), num_evals=7)
    np.testing.assert_allclose(g_table.cpu().numpy(), o_table.numpy(), rtol=0, atol=1e-6)


# ------------------------------------------------------ env handles (B2) ---
def test_env_handle_matches_oracle_and_roundtrips_state():
    """drl_env_* (library-owned state) == oracle; get_state/set_state round trip
    continues bit-identically; set_seed re-seeds like random.seed."""
    from dronerl_amd.handle import DrlEnvHandle
    p = EnvParams(n_drones=8, grid_size=16)
    E, off = 257, 1000
    h = DrlEnvHandle(p, E, env_offset=off, base_seed=5)
    h.reset()
    o = OracleMulti(oparams(p), E)
    o.reset(5 + off + np.arange(E))
    from dronerl_amd import BatchedDeliveryDrones
    helper = BatchedDeliveryDrones(p, E, env_offset=off)   # synthetic actions only
    for t in range(1, 31):
        a = helper.synth_actions(seed=3, step=t)
        r, dn, ob = h.step(a, obs_k=1)
        ro, do = o.step(a.cpu().numpy())
        assert_rewards(r.cpu().numpy(), ro, f"handle step {t}")
        np.testing.assert_array_equal(dn.cpu().numpy().astype(bool), do)
        np.testing.assert_array_equal(ob.cpu().numpy(), o.obs(3, 1))
    st = h.get_state()
    want = o.state()
    np.testing.assert_array_equal(st["ground"].cpu().numpy(), want["ground"])
    np.testing.assert_array_equal(st["order"].cpu().numpy(), want["order"])
    np.testing.assert_array_equal(st["y"].cpu().numpy(), want["y"])
    np.testing.assert_array_equal(st["x"].cpu().numpy(), want["x"])
    np.testing.assert_array_equal(st["charge"].cpu().numpy(), want["charge"])
    np.testing.assert_array_equal(st["carry"].cpu().numpy().astype(bool), want["packet"])
    np.testing.assert_array_equal(st["mt"].cpu().numpy().astype(np.uint32), want["mt"])
    np.testing.assert_array_equal(h.obs(2).cpu().numpy(), o.obs(3, 2))
    # round trip into a second handle, then both continue identically
    h2 = DrlEnvHandle(p, E, env_offset=off)
    h2.set_state(st)
    for t in range(31, 41):
        a = helper.synth_actions(seed=3, step=t)
        r1, d1 = h.step(a)
        r2, d2 = h2.step(a)
        assert torch.equal(r1, r2) and torch.equal(d1, d2)
    for k in st:
        assert torch.equal(h.get_state()[k], h2.get_state()[k]), k
    # masked reset continues the stream; seed() makes the next reset re-seed
    mask = torch.zeros(E, dtype=torch.uint8, device="cuda")
    mask[::3] = 1
    h.reset(mask)
    h.seed(5)
    h.reset()
    o2 = OracleMulti(oparams(p), E)
    o2.reset(5 + off + np.arange(E))
    np.testing.assert_array_equal(h.get_state()["ground"].cpu().numpy(), o2.state()["ground"])
    assert h.errors() == 0
    bad = torch.full((E, 8), 7, dtype=torch.int32, device="cuda")
    h.step(bad)
    assert h.errors() == 1 and h.errors() == 0
    h.close()
    h2.close()


def test_env_handle_argument_errors():
    from dronerl_amd._native import DroneRLError
    from dronerl_amd.handle import DrlEnvHandle
    p = EnvParams(n_drones=4, grid_size=8)
    with pytest.raises(DroneRLError, match="num_envs"):
        DrlEnvHandle(p, 0)
    with pytest.raises(DroneRLError, match="device"):
        DrlEnvHandle(p, 4, device=99)
    h = DrlEnvHandle(p, 4)
    with pytest.raises(DroneRLError, match="before the first reset"):
        h.step(torch.zeros((4, 4), dtype=torch.int32, device="cuda"))
    with pytest.raises(DroneRLError, match="first reset"):
        h.reset(torch.ones(4, dtype=torch.uint8, device="cuda"))
    h.close()


# ----------------------------------------------------------- GridView (A13) --
def base_grid(ground, y, x, charge, packet):
    """wrappers.py:10-31 _create_base_grid restated in numpy (checker)."""
    G = ground.shape[0]
    g = np.zeros((G, G, 6), np.float32)
    for i in range(len(y)):
        g[y[i], x[i], 0] = 1
        if packet[i]:
            g[y[i], x[i], 1] = 1
        g[y[i], x[i], 4] = np.float32(charge[i] / 100)
    g[ground == 5, 1] = 1
    g[ground == 4, 2] = 1
    g[ground == 3, 3] = 1
    g[ground == 2, 5] = 1
    return g


@pytest.mark.parametrize("name", ["c1_g8_n4", "t_g11_n6", "c2_g16_n8"])
def test_grid_obs_on_reference_trajectory_states(name):
    """The grid of the reference's recorded states (tests/golden/traj_*)."""
    d = load_traj(name)
    tp = traj_params(d)
    p = EnvParams(n_drones=tp["n_drones"], grid_size=int(d["side"]))
    E, S, N = d["actions"].shape
    env = Env(p, E)
    for t in [0, S // 2, S]:
        env.set_state(torch.as_tensor(d["ground"][:, t]).cuda(), torch.as_tensor(d["order"][:, t]).cuda(),
                      torch.as_tensor(d["y"][:, t]).cuda(), torch.as_tensor(d["x"][:, t]).cuda(),
                      torch.as_tensor(d["charge"][:, t]).cuda(), torch.as_tensor(d["packet"][:, t]).cuda())
        grid = env.get_grid().cpu().numpy()
        for e in range(E):
            want = base_grid(d["ground"][e, t], d["y"][e, t], d["x"][e, t], d["charge"][e, t], d["packet"][e, t])
            np.testing.assert_array_equal(grid[e], want, err_msg=f"{name} env {e} step {t}")


def test_grid_obs_vs_oracle_state_and_compat_gridview():
    p = EnvParams(n_drones=8, grid_size=16)
    E = 300
    env = Env(p, E)
    env.reset(seed=21)
    o = OracleMulti(oparams(p), E)
    o.reset(21 + np.arange(E))
    for t in range(25):
        a = env.synth_actions(seed=4, step=t)
        env.step(a)
        o.step(a.cpu().numpy())
    st = o.state()
    grid = env.get_grid().cpu().numpy()
    for e in range(E):
        np.testing.assert_array_equal(grid[e], base_grid(st["ground"][e], st["y"][e], st["x"][e], st["charge"][e],
                                                         st["packet"][e]))
    from dronerl_amd.compat import DeliveryDrones, GridView, set_seed
    g = GridView(DeliveryDrones({"n_drones": 3}))
    set_seed(g, 5)
    obs = g.reset()
    st, _, _, _, _ = g.env.step({0: 1, 1: 2, 2: 4})
    obs = g.observation(None)
    assert list(obs) == [dr.index for dr in g.drones.values()]   # dict order
    grid0 = obs[0]
    assert grid0.dtype == np.float32 and grid0.shape == (g.side_size, g.side_size, 6)
    for (y, x), dr in g.drones.items():
        assert grid0[y, x, 0] == 1 and grid0[y, x, 4] == np.float32(dr.charge / 100)


# ------------------------------------------------------------- rollout ---
@pytest.mark.parametrize("name,E,T,k", [
    ("c1_8x8_n4", 64, 40, 1),
    ("c2_16x16_n8", 1000, 60, 1),
    ("c2_16x16_n8", 257, 30, 0),
    ("c2_16x16_n8", 65, 25, 3),
    # P >= 16 (the on-chip rollout kernel): long enough to use up the rings
    # and continue from the streams within the launch
    ("c4_32x32_n16", 300, 90, 1),
    ("c4_32x32_n16|rt", 100, 70, 0),
    ("c5_64x64_n32", 64, 70, 1),
    ("n6_11x11", 129, 50, 2),
    ("n33_26x26", 33, 60, 1),
    ("pool_5x5_n2", 100, 80, 1),
    ("dense_10x10_n8", 200, 60, 1),
    ("c2_16x16_n8|rt", 333, 30, 1),
    # P = 8 without observations: the on-chip kernel (ring entries discarded),
    # long enough for several MT twists per env
    ("c2_16x16_n8", 129, 120, 0),
    ("c2_16x16_n8|rt", 200, 40, 0),
])
def test_rollout_equals_steps(name, E, T, k, monkeypatch):
    """drl_rollout (T steps per launch, state on chip) == T drl_step calls:
    per-step rewards, dones and observations, and the final state."""
    name, _, rt = name.partition("|")
    if rt:
        monkeypatch.setenv("DRL_SPECIALIZE", "0")
    p = EnvParams(**CONFIGS[name])
    a_env, b_env = Env(p, E), Env(p, E)
    a_env.reset(seed=21)
    b_env.reset(seed=21)
    for t in range(3):  # some history first
        acts = a_env.synth_actions(seed=4, step=100 + t)
        a_env.step(acts)
        b_env.step(acts)
    acts = torch.stack([a_env.synth_actions(seed=4, step=t) for t in range(T)])
    out = b_env.rollout(acts, obs_k=k)
    for t in range(T):
        r = a_env.step(acts[t], obs_k=k)
        assert torch.equal(r[0], out[0][t]), f"{name} step {t} rewards"
        assert torch.equal(r[1], out[1][t]), f"{name} step {t} dones"
        if k:
            assert torch.equal(r[2], out[2][t]), f"{name} step {t} obs"
    for f in ["ground", "drones"]:
        assert torch.equal(getattr(a_env.state, f), getattr(b_env.state, f)), f"{name} final {f}"
    # the streams (the rings may differ: refills at other points)
    assert torch.equal(a_env.mt_words_device(), b_env.mt_words_device()), f"{name} final MT state"
    a_env.check_errors()
    b_env.check_errors()


def test_rollout_last_step_outputs_and_oracle():
    """every_step=False keeps the last step's outputs; the final state matches the oracle."""
    p = EnvParams(**CONFIGS["c2_16x16_n8"])
    E, T = 500, 40
    env = Env(p, E)
    env.reset(seed=9)
    o = OracleMulti(oparams(p), E)
    o.reset(9 + np.arange(E))
    acts = torch.stack([env.synth_actions(seed=6, step=t) for t in range(T)])
    r, d, ob = env.rollout(acts, obs_k=1, every_step=False)
    for t in range(T):
        ro, do = o.step(acts[t].cpu().numpy())
    assert_rewards(r.cpu().numpy(), ro, "last step")
    np.testing.assert_array_equal(d.cpu().numpy().astype(bool), do)
    np.testing.assert_array_equal(ob.cpu().numpy(), o.obs(3, 1))
    assert_state(gpu_state(env), o.state(), "rollout final")


def test_train_segment_parallel_matches_serial():
    """bench.TrainSegment: synthetic actions and replay add_many on parallel
    stream branches (3 rotating buffers), and the one-stream loop with the
    synthetic actions fused into the act launch, leave the same env state,
    replay buffer, next observation and learner state as the plain calls on
    one stream."""
    from bench import TrainSegment
    p = EnvParams(n_drones=8, grid_size=16)
    E, seg = 3000, 13
    runs = []
    for parallel, fused in ((False, False), (True, False), (False, True), (True, True)):
        env = Env(p, E)
        env.reset(seed=5)
        loop = TrainSegment(env, seg, parallel=parallel, fused=fused)
        loop.run()
        loop.run()
        torch.cuda.synchronize()
        env.check_errors()
        runs.append((gpu_state(env), loop))
    g0, l0 = runs[0]
    for name, (g1, l1) in zip(("parallel", "fused", "parallel fused"), runs[1:]):
        assert_state(g1, g0, f"{name} vs serial segments")
        for k in ("obs", "next_obs", "actions", "rewards", "dones"):
            assert torch.equal(getattr(l0.rb, k), getattr(l1.rb, k)), (name, k)
        assert l0.rb.cursor == l1.rb.cursor
        assert torch.equal(l0.obs[0], l1.obs[0]), name
        # the learner: the parallel loop trains from the step's own buffers (drl_dqn_train_fresh) while the
        # add runs beside it; the serial loop after the add -- the same learned state, bit for bit
        for k in ("online", "target", "m", "v"):
            for (w0, b0), (w1, b1) in zip(l0.learner.params(k), l1.learner.params(k)):
                assert torch.equal(w0, w1) and torch.equal(b0, b1), (name, k)
        assert l0.learner.counters() == l1.learner.counters(), name
        assert torch.equal(l0.net.packed, l1.net.packed), name


def test_train_segment_code_fused_replay_matches_separate_add():
    """bench.TrainSegment on policy codes: the step that lands its transitions
    in the ring itself (drl_step_code_replay, the one-stream default) leaves
    the same env state, ring, learner and packed net as the separate replay
    add (one stream) and as the parallel branches (learner on fresh rows)."""
    from bench import TrainSegment
    p = EnvParams(n_drones=8, grid_size=16)
    E, seg = 3000, 13
    runs = []
    for parallel, fuse in ((False, False), (False, True), (True, False)):
        env = Env(p, E)
        env.reset(seed=6)
        loop = TrainSegment(env, seg, parallel=parallel, input="code", capacity=20000, fuse_replay=fuse)
        assert loop.fuse_replay == fuse
        loop.run()
        loop.run()
        torch.cuda.synchronize()
        env.check_errors()
        runs.append((gpu_state(env), loop))
    g0, l0 = runs[0]
    for name, (g1, l1) in zip(("fused replay", "parallel"), runs[1:]):
        assert_state(g1, g0, f"{name} vs separate add")
        for k in ("obs", "next_obs", "actions", "rewards", "dones"):
            assert torch.equal(getattr(l0.rb, k), getattr(l1.rb, k)), (name, k)
        assert l0.rb.cursor == l1.rb.cursor and l0.rb.size == l1.rb.size
        for k in ("online", "target", "m", "v"):
            for (w0, b0), (w1, b1) in zip(l0.learner.params(k), l1.learner.params(k)):
                assert torch.equal(w0, w1) and torch.equal(b0, b1), (name, k)
        assert l0.learner.counters() == l1.learner.counters(), name
        assert torch.equal(l0.net.packed, l1.net.packed), name


@pytest.mark.parametrize("G,N,E", [(16, 8, 3000), (64, 32, 600)])
def test_train_segment_synth_branch_graph_matches_fused(G, N, E):
    """bench.TrainSegment(synth_branch=True): the synthetic actions of step
    t + 1 on their own graph branch beside learner t (drl_synth_actions,
    joined before act t + 1), captured and replayed as train_loop_bench does,
    leave the same env state, ring, learner and packed net as the fused act
    (drl_qnet_act_synth) run eagerly: two segments each."""
    from bench import TrainSegment
    p = EnvParams(n_drones=N, grid_size=G)
    seg = 13
    runs = []
    for branch in (False, True):
        env = Env(p, E)
        env.reset(seed=6)
        loop = TrainSegment(env, seg, input="code", capacity=5000, fused=not branch, synth_branch=branch)
        if branch:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                loop.run()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                loop.run()
            g.replay()
        else:
            loop.run()
            loop.run()
        torch.cuda.synchronize()
        env.check_errors()
        loop.net.check_errors()
        runs.append((gpu_state(env), loop))
    (g0, l0), (g1, l1) = runs
    assert_state(g1, g0, "synth branch (graph) vs fused")
    for k in ("obs", "next_obs", "actions", "rewards", "dones"):
        assert torch.equal(getattr(l0.rb, k), getattr(l1.rb, k)), k
    assert l0.rb.cursor == l1.rb.cursor and l0.rb.size == l1.rb.size
    for b in range(2):  # (drone 0's column: the fused run draws the others inside its step)
        assert torch.equal(l0.acts[b][:, 0], l1.acts[b][:, 0]), b
    for k in ("online", "target", "m", "v"):
        for (w0, b0), (w1, b1) in zip(l0.learner.params(k), l1.learner.params(k)):
            assert torch.equal(w0, w1) and torch.equal(b0, b1), k
    assert l0.learner.counters() == l1.learner.counters()
    assert torch.equal(l0.net.packed, l1.net.packed)


@pytest.mark.parametrize("kernel", list(RESET_KERNELS))
@pytest.mark.parametrize("name", ["c1_g8_n4", "c3_g16_n8", "c4_g32_n16", "c5_g64_n32", "t_g5_n1", "t_g7_n2",
                                  "t_g11_n6", "t_g13_n8"])
def test_reset_states_fixture_on_gpu(name, kernel, monkeypatch):
    """C-3 item 3: random.seed(s); env.reset() of the reference for s = 0..15
    (tests/golden/reset_states.npz): env g of reset(seed=0) is seeded g."""
    from tests._golden import load_npz, mt_sha
    for k, v in RESET_KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    d = load_npz("reset_states.npz")
    G, N = int(d[f"{name}__side"]), int(d[f"{name}__n"])
    E = len(d["seeds"])
    env = Env(EnvParams(n_drones=N, grid_size=G), E)
    env.reset(seed=0)
    g = gpu_state(env)
    np.testing.assert_array_equal(g["ground"], d[f"{name}__ground"])
    np.testing.assert_array_equal(g["y"], d[f"{name}__y"])
    np.testing.assert_array_equal(g["x"], d[f"{name}__x"])
    np.testing.assert_array_equal(g["packet"], d[f"{name}__packet"])
    np.testing.assert_array_equal(g["order"], np.tile(np.arange(N), (E, 1)))
    np.testing.assert_array_equal(g["mt"][:, 624], d[f"{name}__mtidx"])
    for e in range(E):
        np.testing.assert_array_equal(mt_sha(g["mt"][e]), d[f"{name}__mtsha"][e], err_msg=f"{name} seed {e} MT")


@pytest.mark.parametrize("name", ["c1_8x8_n4", "c2_16x16_n8", "c5_64x64_n32", "bigside_128_n4", "n6_11x11",
                                  "n1_5x5"])
@pytest.mark.parametrize("refill_kernel", ["list", "wave"])
def test_candidate_ring_holds_the_streams_randint_pairs(name, refill_kernel, monkeypatch):
    """drl_refill's ring, entry by entry, against CPython's own generator:
    entry k is the k-th (randint(0, side-1), randint(0, side-1)) pair drawn
    from the env's stream (random.setstate of its getstate words), with the MT
    index after the pair and its block (flipped once the stream passes a
    twist); the ring-end word is the position after the last entry; the ring
    reaches through the end of the block after the stream's (the next pair
    would end two blocks on) unless it is full; that next block sits twisted
    in the other block's words.  Checked after the reset's conversion and
    again mid-run (partly consumed, wrapped, converted again)."""
    import random
    if refill_kernel == "wave":
        monkeypatch.setenv("DRL_REFILL_LIST", "0")
    from dronerl_amd._native import DRL_CAND_SLOTS as CAP, DRL_MT_RING as RING, DRL_MT_RING_END as RING_END
    p = EnvParams(**CONFIGS[name])
    G, E = p.side, 48
    kb = G.bit_length()
    env = Env(p, E)
    env.reset(seed=13)
    for phase in range(3):
        if phase:
            for t in range(37 if phase == 1 else 160):
                env.step(env.synth_actions(seed=3 + phase, step=t))
            env.refill()
        words = env.mt_words().numpy()
        mi = env.state.mt_index.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        mt = env.state.mt.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        for e in range(E):
            head, cnt, tpar = (mi[e] >> 11) & (CAP - 1), (mi[e] >> 20) & 0x3FF, (mi[e] >> 10) & 1
            r = random.Random()
            r.setstate((3, tuple(int(v) for v in words[e]), None))
            pos = int(words[e, 624])  # absolute stream position (words drawn since block 0 of the stream's)

            def randint():  # _randbelow(G) one getrandbits(kb) word at a time, counting words
                nonlocal pos
                while True:
                    pos += 1
                    v = r.getrandbits(kb)
                    if v < G:
                        return v
            last = None
            for k in range(cnt):
                y, x = randint(), randint()
                blk = (pos - 1) // 624  # block of the pair's last word (0: the stream's)
                idx = pos - 624 * blk
                want = (y * G + x) | (idx << 16) | ((tpar ^ (blk & 1)) << 26)
                got = mt[e, RING + (head + k) % CAP]
                assert got == want, f"{name} phase {phase} env {e} entry {k}/{cnt}: {got:#x} != {want:#x}"
                last = idx | ((tpar ^ (blk & 1)) << 10)
                assert blk <= 1
            if last is not None:
                assert mt[e, RING_END] == last, f"{name} env {e}: ring-end word"
            if cnt < CAP:  # converted through the end of the next block: the next pair ends two blocks on
                randint(), randint()
                assert (pos - 1) // 624 >= 2, f"{name} phase {phase} env {e}: ring stops short ({cnt} entries)"
            # the next block, twisted into the other block's words: CPython's words after the first twist
            r2 = random.Random()
            r2.setstate((3, tuple(int(v) for v in words[e][:624]) + (624,), None))
            r2.getrandbits(1)
            np.testing.assert_array_equal(mt[e, (1 - tpar) * 624:(2 - tpar) * 624],
                                          np.array(r2.getstate()[1][:624], dtype=np.int64),
                                          err_msg=f"{name} env {e}: next block")
    env.check_errors()
