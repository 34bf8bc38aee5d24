"""Policy code (include/dronerl.h drl_step_code / drl_obs_code /
drl_qnet_act_code): drone index 0's window as one u16 per cell, the input of
the f32 act kernel that does not read the f32 observation.

The oracle here is the observation itself (the GPU step is bit-exact with the
reference's WindowedGridView, tests/test_gpu_parity.py): the code decoded on
the host with the channel rules of wrappers.py:10-31 must give drone 0's
observation bit for bit, and the code-input act must give the Q values of an
f32 forward of that observation (Q_TOL below, as tests/test_dqn.py's f32 act).
"""
import ctypes

import numpy as np
import pytest
import torch

from dronerl_amd._native import DroneRLError, lib

gpu = pytest.mark.gpu
Q_TOL = 1e-5  # relative to 1 + max |Q| of the row (tests/test_dqn.py Q_TOL_EXACT)
OBJ_SKYSCRAPER, OBJ_STATION, OBJ_DROPZONE, OBJ_PACKET = 2, 3, 4, 5  # include/dronerl.h


def _cpg(W):
    cpg = -(-W * W // 4)
    return cpg, -(-cpg // 8) * 8


@pytest.mark.parametrize("radius", range(1, 9))
def test_policy_code_bytes(radius):
    W = 2 * radius + 1
    _, cpg8 = _cpg(W)
    assert lib().drl_policy_code_bytes(radius) == 4 * cpg8 * 2
    assert lib().drl_policy_code_bytes(radius) % 16 == 0


def test_policy_code_bytes_rejects_bad_radius():
    assert lib().drl_policy_code_bytes(0) == -1
    assert lib().drl_policy_code_bytes(9) == -1


def _desc(in_features, precision, inp, hidden=(64, 32)):
    from dronerl_amd.dqn import DrlQnetDesc, _bind
    _bind(lib())
    h = list(hidden) + [0] * (3 - len(hidden))
    return DrlQnetDesc(in_features, len(hidden), (ctypes.c_int32 * 3)(*h), 5, precision, inp)


@pytest.mark.parametrize("inf,precision,inp,ok", [(294, 1, 1, True), (150, 1, 1, True), (486, 1, 1, True),
                                                  (294, 0, 1, False), (300, 1, 1, False), (54, 1, 1, False),
                                                  (294, 1, 2, False), (294, 0, 0, True)])
def test_code_net_desc_validation(inf, precision, inp, ok):
    """A code-input net: f32, a 5x5, 7x7 or 9x9 window (no GPU needed)."""
    n = ctypes.c_int64()
    rc = lib().drl_qnet_packed_bytes(ctypes.byref(_desc(inf, precision, inp)), ctypes.byref(n))
    assert (rc == 0) == ok, lib().drl_last_error()


def decode_code(code: np.ndarray, W: int) -> np.ndarray:
    """Host decoder of the policy code -> f32 [E, W, W, 6] with the channel
    rules of wrappers.py:10-31 (as include/dronerl.h documents the code)."""
    E = code.shape[0]
    cells = W * W
    cpg, cpg8 = _cpg(W)
    c = code.view(np.uint16).reshape(E, 4, cpg8)
    h = np.zeros((E, cells), np.uint32)
    for g in range(4):
        n = min(cpg, cells - g * cpg)
        h[:, g * cpg:g * cpg + n] = c[:, g, :n]
        assert (c[:, g, n:] == 0).all(), "padding codes must be zero"
    obj, air = h & 7, h >> 3
    out = np.zeros((E, cells, 6), np.float32)
    out[..., 0] = air != 0
    out[..., 1] = (obj == OBJ_PACKET) | ((air & 0x80) != 0)
    out[..., 2] = obj == OBJ_DROPZONE
    out[..., 3] = obj == OBJ_STATION
    charge = ((air & 0x7F).astype(np.int64) - 1).astype(np.float32) / np.float32(100.0)
    out[..., 4] = np.where(air != 0, charge, np.float32(0.0))
    out[..., 5] = obj == OBJ_SKYSCRAPER
    return out.reshape(E, W, W, 6)


def _env(side, n, radius, E, seed=0, env_offset=0):
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    env = BatchedDeliveryDrones(EnvParams(n_drones=n, grid_size=side, window_radius=radius), E, env_offset=env_offset)
    env.reset(seed=seed)
    return env


@gpu
@pytest.mark.parametrize("side,n,radius,E,k", [(16, 8, 3, 1000, 1), (16, 8, 3, 4096, 2), (32, 16, 3, 333, 1),
                                               (8, 3, 2, 777, 1), (16, 8, 4, 500, 3), (64, 32, 3, 256, 1),
                                               (10, 5, 1, 300, 1), (16, 8, 5, 200, 1)])
def test_step_code_decodes_to_drone0_observation(side, n, radius, E, k):
    """drl_step_code's code == drone 0's observation, bit for bit, over steps
    with deaths, pickups and respawns; drl_obs_code writes the same code."""
    env = _env(side, n, radius, E, seed=side + n)
    W = 2 * radius + 1
    code, code2 = env.new_code(), env.new_code()
    obs2 = torch.empty((E, k, W, W, 6), device="cuda")
    for t in range(12):
        code.fill_(0xAB)
        _, _, obs = env.step(env.synth_actions(seed=3, step=t), obs_k=k, code=code)
        dec = decode_code(code.cpu().numpy(), W)
        assert np.array_equal(dec.view(np.uint32), obs[:, 0].cpu().numpy().view(np.uint32)), t
        code2.fill_(0xCD)
        env.get_obs(k, out=obs2, code=code2)
        assert torch.equal(code2, code)
        assert torch.equal(obs2, obs)
    env.check_errors()


@gpu
@pytest.mark.parametrize("side,n,radius,E", [(16, 8, 3, 4096), (32, 16, 3, 1000), (64, 32, 3, 300), (8, 3, 2, 777),
                                             (16, 8, 4, 500), (10, 5, 1, 300), (16, 8, 8, 64), (24, 20, 3, 129)])
def test_code_only_step_equals_step_with_obs(side, n, radius, E):
    """drl_step_code without the observation (obs_k = 0): the same code, the
    same rewards / dones and the same state as the step that also writes the
    observation."""
    a, b = _env(side, n, radius, E, seed=5), _env(side, n, radius, E, seed=5)
    ca, cb = a.new_code(), b.new_code()
    for t in range(10):
        acts = a.synth_actions(seed=4, step=t)
        ra, da = a.step(acts, code=ca)
        rb, db, _ = b.step(acts, obs_k=1, code=cb)
        assert torch.equal(ca, cb), t
        assert torch.equal(ra, rb) and torch.equal(da, db), t
    for f in ("ground", "drones", "mt", "mt_index"):
        assert torch.equal(getattr(a.state, f), getattr(b.state, f)), f
    a.check_errors()


@gpu
def test_step_code_needs_obs_and_shape():
    env = _env(16, 8, 3, 64)
    acts = env.synth_actions(seed=1, step=0)
    with pytest.raises(ValueError, match="code"):
        env.step(acts, obs_k=1, code=torch.empty((64, 64), dtype=torch.uint8, device="cuda"))
    with pytest.raises(ValueError, match="code"):
        env.step(acts, obs_k=1, code=torch.empty((64, 128), dtype=torch.int32, device="cuda"))


def _nets(in_features, hidden, seed):
    from dronerl_amd.dqn import QNetwork
    g = torch.Generator().manual_seed(seed)
    cnet = QNetwork(in_features, hidden, generator=g, precision="f32", input="code")
    gb = torch.Generator(device="cuda").manual_seed(seed + 1)
    for b in cnet.biases:
        b.normal_(0, 0.1, generator=gb)
    cnet.pack()
    onet = QNetwork(in_features, hidden, precision="f32")
    onet.load(cnet.weights, cnet.biases)
    return cnet, onet


def _f32_forward(net, x):
    ref = x.cpu()
    for i, (w, b) in enumerate(zip(net.weights, net.biases)):
        ref = ref @ w.cpu().t() + b.cpu()
        if i < len(net.weights) - 1:
            ref = torch.relu(ref)
    return ref


@gpu
@pytest.mark.parametrize("side,n,radius,E,hidden", [(16, 8, 3, 65536, (128, 64)), (16, 8, 3, 1000, (32, 32)),
                                                    (32, 16, 3, 4096, (64,)), (16, 8, 3, 333, (128, 128, 128)),
                                                    (8, 3, 2, 777, (96, 32)), (16, 8, 4, 2048, (64, 32)),
                                                    (16, 8, 4, 500, (96, 32)), (16, 8, 2, 31, (64, 64, 32)),
                                                    (8, 3, 2, 777, (128, 64)), (16, 8, 3, 100, (128, 64)),
                                                    (32, 16, 3, 131072, (128, 64))])
@pytest.mark.parametrize("kernel", ["auto", "code2"])
def test_qnet_act_code_matches_f32_forward(side, n, radius, E, hidden, kernel, monkeypatch):
    """Q from the code == an f32 forward of drone 0's observation (and the
    obs-input f32 kernel's Q) within Q_TOL; greedy = the f32 argmax wherever
    the top two are further apart than the tolerance, else within it.
    kernel "code2": DRL_QN_CODE=2 (read per call) routes the 128 -> 64 nets
    through drl_qnet_act_code2_kernel, which no packable net reaches at
    32-bit code offsets (a 9x9 window's 128-unit layer 0 overflows the LDS)."""
    if kernel == "code2":
        if tuple(hidden) != (128, 64):
            pytest.skip("the two-tile kernel serves the 128 -> 64 nets")
        monkeypatch.setenv("DRL_QN_CODE", "2")
    env = _env(side, n, radius, E, seed=E)
    code = env.new_code()
    for t in range(6):
        _, _, obs = env.step(env.synth_actions(seed=2, step=t), obs_k=1, code=code)
    x = obs.reshape(E, -1)
    cnet, onet = _nets(x.shape[1], hidden, seed=len(hidden) * 100 + E)
    q, qo = torch.empty((E, 5), device="cuda"), torch.empty((E, 5), device="cuda")
    a = cnet.act(code, epsilon=0.0, q_out=q)
    onet.act(x, epsilon=0.0, q_out=qo)
    cnet.check_errors()
    ref = _f32_forward(onet, x)
    scale = 1.0 + ref.abs().amax(dim=1, keepdim=True)
    assert ((q.cpu() - ref).abs() / scale).max().item() <= Q_TOL
    assert ((q.cpu() - qo.cpu()).abs() / scale).max().item() <= 2 * Q_TOL
    act = a[:, 0].cpu().long()
    assert torch.equal(act, torch.argmax(q.cpu(), dim=1))
    top2 = torch.topk(ref, 2, dim=1).values
    tol = 2 * Q_TOL * scale[:, 0]
    clear = (top2[:, 0] - top2[:, 1]) > tol
    assert clear.float().mean() > 0.99
    assert torch.equal(act[clear], torch.argmax(ref, dim=1)[clear])
    assert torch.all(ref.gather(1, act[:, None])[:, 0] >= top2[:, 0] - tol)


@gpu
@pytest.mark.parametrize("E,N,off", [(777, 8, 5000), (4096, 32, 123), (31, 3, 0)])
def test_qnet_act_code_exploration_and_synth(E, N, off):
    """The exploration stream and the synth columns are the obs act's: with
    the same Q argmax the actions agree exactly (drl_qnet_act_synth)."""
    side = 16 if N <= 8 else 32
    env = _env(side, N, 3, E, seed=9)
    code = env.new_code()
    _, _, obs = env.step(env.synth_actions(seed=2, step=0), obs_k=1, code=code)
    x = obs.reshape(E, -1)
    cnet, onet = _nets(x.shape[1], (128, 64), seed=77)
    got = torch.full((E, N), -1, dtype=torch.int32, device="cuda")
    ref = torch.full((E, N), -1, dtype=torch.int32, device="cuda")
    q, qo = torch.empty((E, 5), device="cuda"), torch.empty((E, 5), device="cuda")
    cnet.act(code, epsilon=0.3, seed=7, step=3, env_offset=off, actions=got, q_out=q, synth=(2024, 9))
    onet.act(x, epsilon=0.3, seed=7, step=3, env_offset=off, actions=ref, q_out=qo, synth=(2024, 9))
    same_greedy = torch.argmax(q, dim=1) == torch.argmax(qo, dim=1)
    assert same_greedy.float().mean() > 0.99
    assert torch.equal(got[same_greedy], ref[same_greedy])
    assert torch.equal(got[:, 1:], ref[:, 1:])


@gpu
def test_qnet_code_input_checks():
    from dronerl_amd.dqn import QNetwork
    with pytest.raises(ValueError, match="code"):
        QNetwork(294, (64,), precision="bf16", input="code")
    with pytest.raises(ValueError, match="code"):
        QNetwork(300, (64,), precision="f32", input="code")
    net = QNetwork(294, (64,), precision="f32", input="code")
    with pytest.raises(ValueError, match="code"):
        net.act(torch.zeros((10, 294), device="cuda"), epsilon=0.0)
    with pytest.raises(ValueError, match="code"):
        net.act(torch.zeros((10, 64), dtype=torch.uint8, device="cuda"), epsilon=0.0)
    onet = QNetwork(294, (64,), precision="f32")
    lib_ = onet.L
    # an obs-input net refuses the code entry point and vice versa (C-ABI checks)
    code = torch.zeros((10, 128), dtype=torch.uint8, device="cuda")
    acts = torch.zeros((10, 1), dtype=torch.int32, device="cuda")
    rc = lib_.drl_qnet_act_code(ctypes.byref(onet.desc), ctypes.c_void_p(onet.packed.data_ptr()),
                                ctypes.c_void_p(code.data_ptr()), 10, 0.0, 0, 0, 0,
                                ctypes.c_void_p(acts.data_ptr()), 1, 0, 0, 0, None, None,
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc != 0 and b"INPUT_CODE" in lib_.drl_last_error()
    with pytest.raises(DroneRLError):
        obs = torch.zeros((10, 294), device="cuda")
        from dronerl_amd.dqn import _check
        _check(lib_, lib_.drl_qnet_act(ctypes.byref(net.desc), ctypes.c_void_p(net.packed.data_ptr()),
                                       ctypes.c_void_p(obs.data_ptr()), 10, 294, 0.0, 0, 0, 0,
                                       ctypes.c_void_p(acts.data_ptr()), 1, None, None,
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))


@gpu
@pytest.mark.parametrize("side,n,radius,E", [(16, 8, 3, 1000), (8, 3, 2, 777), (16, 8, 4, 500), (10, 5, 1, 300),
                                             (16, 8, 8, 64), (64, 32, 3, 129)])
def test_code_decode_and_get_code(side, n, radius, E):
    """drl_code_decode(code) == drone 0's observation bit for bit; get_code ==
    the code the step wrote."""
    from dronerl_amd.dqn import decode_policy_code
    env = _env(side, n, radius, E, seed=3)
    code = env.new_code()
    for t in range(5):
        _, _, obs = env.step(env.synth_actions(seed=8, step=t), obs_k=1, code=code)
    dec = decode_policy_code(code, radius)
    assert torch.equal(dec.view(torch.int32), obs[:, 0].reshape(E, -1).view(torch.int32))
    assert torch.equal(env.get_code(), code)


@gpu
def test_code_replay_buffer_samples_decode_to_obs_buffer():
    """A replay buffer of code rows holds the same transitions as one of f32
    rows: sample() with the same generator returns identical tensors."""
    from dronerl_amd.dqn import ReplayBuffer
    E, cap = 3000, 5000
    env = _env(16, 8, 3, E, seed=1)
    D = 294
    rb_f = ReplayBuffer(cap, D, torch.device("cuda"))
    rb_c = ReplayBuffer(cap, D, torch.device("cuda"), code_radius=3)
    code = [env.new_code(), env.new_code()]
    obs = [torch.empty((E, 1, 7, 7, 6), device="cuda"), torch.empty((E, 1, 7, 7, 6), device="cuda")]
    env.get_obs(1, out=obs[0], code=code[0])
    for t in range(4):
        a = env.synth_actions(seed=6, step=t)
        r, d, _ = env.step(a, obs_k=1, obs=obs[(t + 1) & 1], code=code[(t + 1) & 1])
        rb_f.add_many(obs[t & 1], a, r, obs[(t + 1) & 1], d)
        rb_c.add_many(code[t & 1], a, r, code[(t + 1) & 1], d)
    assert rb_f.cursor == rb_c.cursor and rb_f.size == rb_c.size
    sf = rb_f.sample(256, generator=torch.Generator(device="cuda").manual_seed(9))
    sc = rb_c.sample(256, generator=torch.Generator(device="cuda").manual_seed(9))
    for k in sf:
        assert torch.equal(sf[k], sc[k]), k


@gpu
@pytest.mark.parametrize("side,n,radius,E,cap,cursor0", [
    (16, 8, 3, 4096, 10000, 0),      # the C3 geometry (compile-time instance), no wrap in the first steps
    (16, 8, 3, 3000, 7001, 6000),    # the ring wraps inside a call
    (16, 8, 3, 2000, 1500, 700),     # num_envs > capacity: only the last `capacity` envs land
    (24, 5, 3, 777, 2000, 1999),     # runtime geometry, n_drones % 4 != 0 (byte dones)
    (32, 16, 2, 333, 1000, 10),      # 5x5 window (64-B code rows)
    (64, 32, 4, 129, 300, 250),      # 9x9 window (192-B rows), C5's grid
    (64, 32, 3, 6000, 5000, 4500),   # the C5 compile-time instance with num_envs > capacity (c5.train_loop)
])
@pytest.mark.parametrize("synth", [False, True])
def test_step_code_replay_equals_step_then_add_many(side, n, radius, E, cap, cursor0, synth):
    """drl_step_code_replay (env.step(..., replay=rb, replay_obs=prev)): the
    step's outputs and state and the whole ring -- obs, next_obs, actions,
    rewards, dones, cursor, size -- equal drl_step_code followed by
    drl_replay_add of the same transitions, bit for bit, over steps that wrap
    the ring.  synth: drl_step_code_replay_synth (env.step(..., synth=(seed,
    t))) draws drone indices >= 1 itself; its actions' other columns hold an
    invalid action (9) that must not be read (env_offset 1000: the draws
    follow the global env index)."""
    from dronerl_amd.dqn import ReplayBuffer
    D = (2 * radius + 1) ** 2 * 6
    off = 1000 if synth else 0
    a, b = _env(side, n, radius, E, seed=11, env_offset=off), _env(side, n, radius, E, seed=11, env_offset=off)
    ra_ = ReplayBuffer(cap, D, torch.device("cuda"), code_radius=radius)
    rb_ = ReplayBuffer(cap, D, torch.device("cuda"), code_radius=radius)
    for r in (ra_, rb_):
        r.cursor = cursor0
        for f in ("obs", "next_obs"):
            getattr(r, f).fill_(0x5A)  # (stale rows: every landing row must be overwritten)
    ca, cb = [a.new_code(), a.new_code()], [b.new_code(), b.new_code()]
    a.get_obs(1, code=ca[0])
    b.get_obs(1, code=cb[0])
    for t in range(6):
        acts = a.synth_actions(seed=8, step=t)
        if synth:
            only0 = torch.full_like(acts, 9)
            only0[:, 0] = acts[:, 0]
            rw_a, dn_a = a.step(only0, code=ca[(t + 1) & 1], replay=ra_, replay_obs=ca[t & 1], synth=(8, t))
            assert (only0[:, 1:] == 9).all()  # (neither read nor written)
        else:
            rw_a, dn_a = a.step(acts, code=ca[(t + 1) & 1], replay=ra_, replay_obs=ca[t & 1])
        rw_b, dn_b = b.step(acts, code=cb[(t + 1) & 1])
        rb_.add_many(cb[t & 1], acts, rw_b, cb[(t + 1) & 1], dn_b)
        assert torch.equal(rw_a, rw_b) and torch.equal(dn_a, dn_b), t
        assert torch.equal(ca[(t + 1) & 1], cb[(t + 1) & 1]), t
        assert ra_.cursor == rb_.cursor and ra_.size == rb_.size, t
        for f in ("obs", "next_obs", "actions", "rewards", "dones"):
            assert torch.equal(getattr(ra_, f), getattr(rb_, f)), (t, f)
        assert ra_.last_batch.n == E and ra_.last_batch.cursor == (cursor0 + t * E) % cap
    for f in ("ground", "drones", "mt", "mt_index"):
        assert torch.equal(getattr(a.state, f), getattr(b.state, f)), f
    a.check_errors()


@gpu
def test_step_code_replay_argument_checks():
    from dronerl_amd.dqn import ReplayBuffer
    env = _env(16, 8, 3, 64)
    rb = ReplayBuffer(100, 294, torch.device("cuda"), code_radius=3)
    c0, c1 = env.new_code(), env.new_code()
    acts = env.synth_actions(seed=1, step=0)
    since = env._since_refill = env.refill_every - 1  # a refused call must not consume the refill cadence
    with pytest.raises(ValueError):  # the act's rows must be another buffer
        env.step(acts, code=c0, replay=rb, replay_obs=c0)
    assert env._since_refill == since
    with pytest.raises(ValueError):  # no f32 observation with the ring
        env.step(acts, obs_k=1, code=c0, replay=rb, replay_obs=c1)
    with pytest.raises(ValueError):  # a buffer of f32 rows
        env.step(acts, code=c0, replay=ReplayBuffer(100, 294, torch.device("cuda")), replay_obs=c1)
    with pytest.raises(ValueError):  # another window radius
        env.step(acts, code=c0, replay=ReplayBuffer(100, 150, torch.device("cuda"), code_radius=2), replay_obs=c1)
    assert env._since_refill == since and rb.cursor == 0 and rb.size == 0
    assert rb.cursor == 0 and rb.size == 0
