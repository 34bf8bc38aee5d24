"""DQN consumer: Q-network act on MFMA + replay add_many.

Reference: jax_impl/agents/dqn.py:47-63,132-146; jax_impl/buffers.py:57-93;
train_jax.py:42-64.  Numerics (precision="bf16", the opt-in): the kernel uses
bf16 operands with f32 accumulation, so Q is checked against a torch fp32 forward with the same
bf16 rounding of weights/inputs/activations (tolerance below) and, looser,
against the plain fp32 forward; greedy actions must match wherever the
reference's top-two margin exceeds the tolerance.  The exploration draws come
from our counter hash (the reference's threefry stream is jax-only: parity
unpinned for the random branch; checked against a numpy restatement).
"""
import ctypes

import numpy as np
import pytest
import torch

Q_TOL_BF16 = 2e-2   # |Q - Q_ref(bf16 operands)| <= tol * (1 + |Q_ref|): f32 sum order + activation rounding
Q_TOL_F32 = 8e-2    # vs the plain fp32 forward (bf16 operand rounding)


def _desc(in_features, hidden, n_actions=5, precision=0):
    from dronerl_amd.dqn import DrlQnetDesc
    h = list(hidden) + [0] * (3 - len(hidden))
    return DrlQnetDesc(in_features, len(hidden), (ctypes.c_int32 * 3)(*h), n_actions, precision)


@pytest.mark.parametrize("inf,hidden,ok", [
    (294, (128, 64), True), (294, (32, 32), True), (294, (128, 128, 128), True), (150, (64,), True),
    (293, (32,), False), (294, (100,), False), (294, (256,), False), (294, (), False), (600, (32,), False),
    (512, (128, 128, 128), False),   # does not fit LDS
])
def test_qnet_desc_validation(inf, hidden, ok):
    from dronerl_amd._native import lib
    from dronerl_amd.dqn import _bind
    L = _bind(lib())
    nb = ctypes.c_int64()
    rc = L.drl_qnet_packed_bytes(ctypes.byref(_desc(inf, hidden)), ctypes.byref(nb))
    assert (rc == 0) == ok, L.drl_last_error()
    if ok:
        assert nb.value % 16 == 0 and nb.value <= 160 * 1024


def test_qnet_packed_size_formula():
    from dronerl_amd._native import lib
    from dronerl_amd.dqn import _bind
    L = _bind(lib())
    nb = ctypes.c_int64()
    assert L.drl_qnet_packed_bytes(ctypes.byref(_desc(294, (128, 64))), ctypes.byref(nb)) == 0
    frags = 8 * 10 + 4 * 4 + 1 * 2          # (16-row tiles x 32-wide K-slices) per layer, 1 KB each
    biases = (128 + 64 + 16) * 4
    status = 16  # drl_qnet_pack's range flag vector ends the packed net
    assert nb.value == frags * 1024 + biases + status
    # DRL_QNET_F32: fp16 hi fragments, biases, the later layers' lo fragments (the LDS image), then layer 0's lo
    assert L.drl_qnet_packed_bytes(ctypes.byref(_desc(294, (128, 64), precision=1)), ctypes.byref(nb)) == 0
    assert nb.value == 2 * frags * 1024 + biases + status
    assert L.drl_qnet_packed_bytes(ctypes.byref(_desc(294, (128, 64), precision=2)), ctypes.byref(nb)) != 0
    assert b"precision" in L.drl_last_error()
    # f32 with layer 0's hi + lo fragments alone in LDS (160 KB at 294 -> 128), the later layers in global
    # memory: three 128-wide hidden layers pack (same total bytes, another order)
    assert L.drl_qnet_packed_bytes(ctypes.byref(_desc(294, (128, 128, 128), precision=1)), ctypes.byref(nb)) == 0
    frags3 = 8 * 10 + 8 * 4 + 8 * 4 + 1 * 4
    assert nb.value == 2 * frags3 * 1024 + (128 * 3 + 16) * 4 + status
    # 486 inputs (radius 4) at 128 units: neither layout fits the LDS
    assert L.drl_qnet_packed_bytes(ctypes.byref(_desc(486, (128, 128), precision=1)), ctypes.byref(nb)) != 0


def _hash_explore(seed, step, genv, n_actions, eps):
    M = (1 << 64) - 1

    def sm(z):
        z = (z + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)
    h = sm(seed ^ sm(((step << 40) ^ (genv << 8) ^ 0xA5) & M))
    u = np.float32(h >> 40) * np.float32(1.0 / 16777216.0)
    return bool(u < np.float32(eps)), ((h & 0xFFFFFFFF) * n_actions) >> 32


gpu = pytest.mark.gpu


def _obs_batch(E, seed=0, radius=3):
    """Real observations from the env (C3 shape)."""
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    env = BatchedDeliveryDrones(EnvParams(n_drones=8, grid_size=16, window_radius=radius), E)
    env.reset(seed=seed)
    for t in range(5):
        env.step(env.synth_actions(seed=1, step=t))
    return env.get_obs(1).reshape(E, -1).contiguous(), env


@gpu
@pytest.mark.parametrize("hidden", [(128, 64), (32, 32), (64,), (128, 128, 128), (96, 32)])
@pytest.mark.parametrize("E", [4096, 1000, 31])
def test_qnet_greedy_matches_torch_reference(hidden, E):
    from dronerl_amd.dqn import QNetwork
    obs, _ = _obs_batch(E)
    g = torch.Generator().manual_seed(len(hidden) * 1000 + E)
    net = QNetwork(obs.shape[1], hidden, generator=g, precision="bf16")
    gb = torch.Generator(device="cuda").manual_seed(E + 3)
    for b in net.biases:
        b.normal_(0, 0.1, generator=gb)
    net.pack()
    q = torch.empty((E, 5), device="cuda")
    a = net.act(obs, epsilon=0.0, q_out=q)
    ref = net.reference_q(obs, bf16_operands=True)
    ref32 = net.reference_q(obs)
    assert torch.all((q - ref).abs() <= Q_TOL_BF16 * (1 + ref.abs())), (q - ref).abs().max()
    assert torch.all((q - ref32).abs() <= Q_TOL_F32 * (1 + ref32.abs())), (q - ref32).abs().max()
    # greedy = first argmax of the kernel's own Q, always
    assert torch.equal(a[:, 0].long(), torch.argmax(q, dim=1))
    # and the reference's argmax wherever its margin is safe
    top2 = torch.topk(ref, 2, dim=1).values
    safe = (top2[:, 0] - top2[:, 1]) > 2 * Q_TOL_BF16 * (1 + top2[:, 0].abs())
    assert safe.float().mean() > 0.5
    assert torch.equal(a[safe, 0].long(), torch.argmax(ref, dim=1)[safe])


# DRL_QNET_F32 (the reference's f32 nets): Q against an f32 forward, relative
# to the row's scale, and the greedy action against the f32 argmax everywhere.
Q_TOL_EXACT = 1e-5


# Layouts: layer 0's hi + lo fragments fit the LDS (every 294-input net here,
# and 486 inputs at 64 units) -> layer 0 alone in LDS, the rest from L2; at 486
# inputs with 96 units they do not -> layer 0's lo fragments from L2.
@gpu
@pytest.mark.parametrize("hidden,E,radius", [((128, 64), 65536, 3), ((128, 64), 1000, 3), ((32, 32), 4096, 3),
                                             ((64,), 31, 3), ((96, 32), 4096, 3), ((128, 128), 333, 3),
                                             ((64, 64, 32), 4096, 3), ((128, 128, 128), 2048, 3), ((96, 32), 2048, 4),
                                             ((64, 32), 777, 4)])
def test_qnet_f32_matches_fp32_forward(hidden, E, radius):
    from dronerl_amd.dqn import QNetwork
    obs, _ = _obs_batch(E, radius=radius)
    g = torch.Generator().manual_seed(len(hidden) * 1000 + E)
    net = QNetwork(obs.shape[1], hidden, generator=g, precision="f32")
    gb = torch.Generator(device="cuda").manual_seed(E + 7)
    for b in net.biases:
        b.normal_(0, 0.1, generator=gb)
    net.pack()
    q = torch.empty((E, 5), device="cuda")
    a = net.act(obs, epsilon=0.0, q_out=q)
    # f32 forward on the host (plain IEEE f32 matmuls) and an f64 one
    x = obs.cpu()
    ref32, ref64 = x.clone(), x.double()
    for i, (w, b) in enumerate(zip(net.weights, net.biases)):
        ref32 = ref32 @ w.cpu().t() + b.cpu()
        ref64 = ref64 @ w.cpu().double().t() + b.cpu().double()
        if i < len(net.weights) - 1:
            ref32, ref64 = torch.relu(ref32), torch.relu(ref64)
    qc = q.cpu()
    scale = 1.0 + ref32.abs().amax(dim=1, keepdim=True)
    err = ((qc - ref32).abs() / scale).max().item()
    assert err <= Q_TOL_EXACT, err
    assert ((qc.double() - ref64).abs() / scale.double()).max().item() <= Q_TOL_EXACT
    # greedy action == torch.argmax of the f32 reference (first maximum) on every env whose top two
    # Q values are further apart than the tolerance (two f32 forwards that sum in different orders may
    # order a closer pair either way); on the others the chosen action's reference Q is within the
    # tolerance of the maximum
    act = a[:, 0].cpu().long()
    top2 = torch.topk(ref32, 2, dim=1).values
    tol = 2 * Q_TOL_EXACT * scale[:, 0]
    clear = (top2[:, 0] - top2[:, 1]) > tol
    assert clear.float().mean() > 0.99
    assert torch.equal(act[clear], torch.argmax(ref32, dim=1)[clear])
    chosen = ref32.gather(1, act[:, None])[:, 0]
    assert torch.all(chosen >= top2[:, 0] - tol)
    assert torch.equal(act, torch.argmax(q.cpu(), dim=1))  # and always the first argmax of its own Q


@gpu
def test_qnet_f32_weight_range_checked():
    from dronerl_amd.dqn import QNetwork
    net = QNetwork(294, (32,), precision="f32")
    w = [t.clone() for t in net.weights]
    w[0][0, 0] = 70000.0
    with pytest.raises(ValueError, match="65504"):
        net.load(w, net.biases)
    b = [t.clone() for t in net.biases]
    b[0][3] = float("inf")
    with pytest.raises(ValueError, match="finite"):
        net.load(net.weights, b)
    # only a code net's layer-0 bias is split into fp16 pieces; the
    # obs net's biases stay f32, so a large finite bias is a valid net
    b = [t.clone() for t in net.biases]
    b[0][3], b[1][2] = 1e6, -2e5
    net.load(net.weights, b)
    cnet = QNetwork(294, (32,), precision="f32", input="code")
    with pytest.raises(ValueError, match="65504"):
        cnet.load(cnet.weights, b)
    b = [t.clone() for t in cnet.biases]
    b[1][2] = 1e6
    cnet.load(cnet.weights, b)


@gpu
@pytest.mark.parametrize("where", ["input", "hidden", "nan", "packed_weight", "ok"])
def test_qnet_f32_activation_range_flagged(where):
    """an input or hidden activation beyond fp16's split range
    (|v| >= 65520) would become inf/NaN in the hi/lo split; the kernel flags
    DRL_ERR_QNET_RANGE instead of returning an arbitrary action silently."""
    from dronerl_amd._native import DroneRLError
    from dronerl_amd.dqn import QNetwork
    E = 100
    obs, _ = _obs_batch(E)
    net = QNetwork(obs.shape[1], (64, 32), generator=torch.Generator().manual_seed(5), precision="f32")
    x = obs.clone()
    if where == "input":
        x[17, 3] = 1.0e5
    elif where == "nan":
        x[42, 0] = float("nan")
    elif where == "hidden":  # weights in range, activations of layer 0 beyond it
        w = [t.clone() for t in net.weights]
        w[0][:, :] = 3000.0
        net.load(w, net.biases)
    elif where == "packed_weight":  # a weight outside the split range packed through the C ABI (no host check)
        w = [t.clone() for t in net.weights]
        w[2][1, 0] = 1.0e6
        net.weights = w
        from dronerl_amd.dqn import _check, _stream, _vp
        n = len(w)
        wp = (_vp * n)(*[t.data_ptr() for t in w])
        bp = (_vp * n)(*[t.data_ptr() for t in net.biases])
        _check(net.L, net.L.drl_qnet_pack(ctypes.byref(net.desc), wp, bp, _vp(net.packed.data_ptr()),
                                          _stream(net.device)))
    net.act(x, epsilon=0.0)
    if where == "ok":
        net.check_errors()
        return
    with pytest.raises(DroneRLError, match="fp16 split range"):
        net.check_errors()
    net.check_errors()  # cleared


@gpu
def test_qnet_exploration_stream_and_column_write():
    from dronerl_amd.dqn import QNetwork
    E, N = 777, 8
    obs, _ = _obs_batch(E)
    net = QNetwork(obs.shape[1], (128, 64), generator=torch.Generator().manual_seed(3))
    acts = torch.full((E, N), 9, dtype=torch.int32, device="cuda")
    q = torch.empty((E, 5), device="cuda")
    eps, seed, step, off = 0.3, 12345, 17, 5000
    net.act(obs, epsilon=eps, seed=seed, step=step, env_offset=off, actions=acts, q_out=q)
    a = acts.cpu().numpy()
    assert (a[:, 1:] == 9).all()               # other drones untouched
    greedy = torch.argmax(q, dim=1).cpu().numpy()
    n_exp = 0
    for e in range(E):
        exp, rnd = _hash_explore(seed, step, off + e, 5, eps)
        n_exp += exp
        assert a[e, 0] == (rnd if exp else greedy[e]), e
    assert 0.2 < n_exp / E < 0.4
    net.act(obs, epsilon=1.0, seed=seed, step=step + 1, actions=acts)
    assert set(np.unique(acts[:, 0].cpu().numpy())) == set(range(5))


@gpu
@pytest.mark.parametrize("precision", ["bf16", "f32"])
@pytest.mark.parametrize("E,N,off", [(777, 8, 5000), (31, 3, 0), (4096, 32, 123), (100, 1, 7), (65536, 8, 0)])
def test_qnet_act_synth_equals_synth_then_act(E, N, off, precision):
    """drl_qnet_act_synth == drl_synth_actions followed by drl_qnet_act (the
    fused launch of bench.TrainSegment), Q included."""
    from dronerl_amd import _native
    from dronerl_amd.dqn import QNetwork
    obs, env = _obs_batch(E)
    net = QNetwork(obs.shape[1], (128, 64), generator=torch.Generator().manual_seed(11), precision=precision)
    ref = torch.empty((E, N), dtype=torch.int32, device="cuda")
    assert _native.lib().drl_synth_actions(2024, 9, off, E, N, ref.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream) == 0
    q0, q1 = torch.empty((E, 5), device="cuda"), torch.empty((E, 5), device="cuda")
    net.act(obs, epsilon=0.25, seed=7, step=3, env_offset=off, actions=ref, q_out=q0)
    got = torch.full((E, N), -1, dtype=torch.int32, device="cuda")
    net.act(obs, epsilon=0.25, seed=7, step=3, env_offset=off, actions=got, q_out=q1, synth=(2024, 9))
    assert torch.equal(got, ref)
    assert torch.equal(q0, q1)


@gpu
def test_qnet_load_repacks():
    from dronerl_amd.dqn import QNetwork
    obs, _ = _obs_batch(256)
    net = QNetwork(obs.shape[1], (64, 32), generator=torch.Generator().manual_seed(1))
    net2 = QNetwork(obs.shape[1], (64, 32), generator=torch.Generator().manual_seed(2))
    net.load(net2.weights, net2.biases)
    q1, q2 = torch.empty((256, 5), device="cuda"), torch.empty((256, 5), device="cuda")
    net.act(obs, 0.0, q_out=q1)
    net2.act(obs, 0.0, q_out=q2)
    assert torch.equal(q1, q2)
    with pytest.raises(ValueError):
        net.load(net2.weights[:1], net2.biases[:1])


def _seq_add(buf, obs, acts, rews, nobs, dones, cursor, cap):
    for i in range(obs.shape[0]):
        s = (cursor + i) % cap
        buf["obs"][s], buf["next_obs"][s] = obs[i], nobs[i]
        buf["actions"][s], buf["rewards"][s], buf["dones"][s] = acts[i], rews[i], dones[i]


@gpu
@pytest.mark.parametrize("cap,batches", [(10000, [4096, 4096, 4096]), (100, [37, 250, 5, 64]), (7, [3])])
def test_replay_add_many_matches_sequential_add(cap, batches):
    from dronerl_amd.dqn import ReplayBuffer
    D, N = 294, 8
    rb = ReplayBuffer(cap, D, torch.device("cuda"))
    ref = dict(obs=np.zeros((cap, D), np.float32), next_obs=np.zeros((cap, D), np.float32),
               actions=np.zeros(cap, np.int32), rewards=np.zeros(cap, np.float32), dones=np.zeros(cap, np.uint8))
    g = torch.Generator(device="cuda").manual_seed(0)
    cursor, size = 0, 0
    for n in batches:
        obs = torch.rand((n, 1, 7, 7, 6), device="cuda", generator=g)
        nobs = torch.rand((n, 1, 7, 7, 6), device="cuda", generator=g)
        acts = torch.randint(0, 5, (n, N), dtype=torch.int32, device="cuda", generator=g)
        rews = torch.rand((n, N), device="cuda", generator=g)
        dones = (torch.rand((n, N), device="cuda", generator=g) < 0.2).to(torch.uint8)
        rb.add_many(obs, acts, rews, nobs, dones)
        _seq_add(ref, obs.reshape(n, -1).cpu().numpy(), acts[:, 0].cpu().numpy(), rews[:, 0].cpu().numpy(),
                 nobs.reshape(n, -1).cpu().numpy(), dones[:, 0].cpu().numpy(), cursor, cap)
        cursor, size = (cursor + n) % cap, min(size + n, cap)
        assert rb.cursor == cursor and rb.size == size
    for k in ref:
        np.testing.assert_array_equal(getattr(rb, k).cpu().numpy(), ref[k], err_msg=k)
    b = rb.sample(64, generator=g)
    assert b["obs"].shape == (64, D) and rb.can_sample(64) == (size >= 64)


@gpu
def test_replay_add_two_float_rows():
    """Rows of one float2 (obs_floats 2): drl_replay_add_rows_kernel, the
    block-per-row form, against a sequential add() loop."""
    from dronerl_amd.dqn import ReplayBuffer
    cap, D = 50, 2
    rb = ReplayBuffer(cap, D, torch.device("cuda"))
    ref = dict(obs=np.zeros((cap, D), np.float32), next_obs=np.zeros((cap, D), np.float32),
               actions=np.zeros(cap, np.int32), rewards=np.zeros(cap, np.float32), dones=np.zeros(cap, np.uint8))
    g = torch.Generator(device="cuda").manual_seed(1)
    cursor = 0
    for n in (30, 40, 77):
        obs, nobs = torch.rand((n, D), device="cuda", generator=g), torch.rand((n, D), device="cuda", generator=g)
        acts = torch.randint(0, 5, (n,), dtype=torch.int32, device="cuda", generator=g)
        rews = torch.rand((n,), device="cuda", generator=g)
        dones = (torch.rand((n,), device="cuda", generator=g) < 0.3).to(torch.uint8)
        rb.add_many(obs, acts, rews, nobs, dones)
        _seq_add(ref, obs.cpu().numpy(), acts.cpu().numpy(), rews.cpu().numpy(), nobs.cpu().numpy(),
                 dones.cpu().numpy(), cursor, cap)
        cursor = (cursor + n) % cap
    for k in ref:
        np.testing.assert_array_equal(getattr(rb, k).cpu().numpy(), ref[k], err_msg=k)


@gpu
def test_train_loop_shape_step_act_add():
    """train_jax.py:42-64 loop shape: act on obs -> step(+obs) -> add_many."""
    from dronerl_amd.dqn import QNetwork, ReplayBuffer
    E = 2048
    obs, env = _obs_batch(E)
    net = QNetwork(obs.shape[1], (128, 64), generator=torch.Generator().manual_seed(0))
    rb = ReplayBuffer(10000, obs.shape[1], torch.device("cuda"))
    for t in range(20):
        a = env.synth_actions(seed=7, step=t)
        net.act(obs, epsilon=0.1, seed=1, step=t, actions=a)
        r, d, nobs = env.step(a, obs_k=1)
        nobs = nobs.reshape(E, -1)
        rb.add_many(obs, a, r, nobs, d)
        obs = nobs
    env.check_errors()
    assert rb.size == 10000 and rb.cursor == (20 * E) % 10000
