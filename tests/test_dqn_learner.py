"""DQN learner (SURVEY.md §8 F1's train half): drl_dqn_train.

Reference: jax_impl/agents/dqn.py:147-200 (train_step, update_target,
update_epsilon), train_jax.py:68-98 (the scan body's learner block),
jax_impl/buffers.py:79-93 (sample, can_sample), optax.adam.

Oracle: oracle/dqn_learner.py, a numpy f32 restatement in the kernel's fixed
arithmetic order -- the GPU learner must equal it BIT FOR BIT (parameters,
target, Adam moments, loss, counters) over many steps.  The restatement
itself is pinned here on the CPU against an independent fp32 PyTorch
restatement (autograd for the gradient, optax's Adam formula written out):
within REL_TOL per step.  jax/optax are not importable, so
agreement with optax's own code stays parity unpinned; the row draw is the
build's counter hash (the reference's jax.random stream is jax-only).
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import dqn_learner as O

gpu = pytest.mark.gpu
REL_TOL = 2e-5  # oracle vs the torch restatement: different summation orders, f32


def _rand_net(sizes, seed):
    g = np.random.default_rng(seed)
    out = []
    for i in range(len(sizes) - 1):
        std = (2.0 / sizes[i]) ** 0.5
        out.append((g.normal(0, std, (sizes[i + 1], sizes[i])).astype(np.float32),
                    g.normal(0, 0.05, sizes[i + 1]).astype(np.float32)))
    return out


def _rand_replay(cap, n_in, seed, code_window=0):
    g = np.random.default_rng(seed)
    if code_window:
        W = code_window
        cells = W * W
        cpg = -(-cells // 4)
        cpg8 = -(-cpg // 8) * 8
        codes = np.zeros((2, cap, 4, cpg8), np.uint16)
        for t in range(2):
            for grp in range(4):
                k = min(cpg, cells - grp * cpg)
                obj = g.choice([0, 0, 0, 2, 3, 4, 5], size=(cap, k))
                air = np.where(g.random((cap, k)) < 0.2, g.integers(1, 102, (cap, k)) | (g.integers(0, 2, (cap, k)) << 7), 0)
                codes[t, :, grp, :k] = (obj | (air << 3)).astype(np.uint16)
        obs = codes[0].reshape(cap, -1).view(np.uint8).reshape(cap, -1)
        nxt = codes[1].reshape(cap, -1).view(np.uint8).reshape(cap, -1)
    else:
        obs = (g.random((cap, n_in)) < 0.15).astype(np.float32)
        nxt = (g.random((cap, n_in)) < 0.15).astype(np.float32)
        obs[:, 4::6] *= g.integers(0, 101, (cap, n_in // 6)).astype(np.float32) / np.float32(100)
        nxt[:, 4::6] *= g.integers(0, 101, (cap, n_in // 6)).astype(np.float32) / np.float32(100)
    return {"obs": obs, "next_obs": nxt, "actions": g.integers(0, 5, cap).astype(np.int32),
            "rewards": g.choice(np.array([0.0, 1.0, -1.0, -0.1], np.float32), cap),
            "dones": (g.random(cap) < 0.1).astype(np.uint8)}


def _torch_forward(ps, X):
    a = X
    for i in range(0, len(ps), 2):
        a = a @ ps[i].t() + ps[i + 1]
        if i < len(ps) - 2:
            a = torch.relu(a)
    return a


def _torch_step(st, hp, X, Xn, act, rew, done):
    """fp32 PyTorch restatement of train_step + optax.adam (independent of the
    oracle's order): autograd gradient, the optax formula written out."""
    ps = [torch.tensor(t).requires_grad_() for wb in st["online"] for t in wb]
    tg = [torch.tensor(t) for wb in st["target"] for t in wb]
    q = _torch_forward(ps, torch.tensor(X))
    qa = q.gather(1, torch.tensor(act, dtype=torch.long)[:, None])[:, 0]
    with torch.no_grad():
        mx = _torch_forward(tg, torch.tensor(Xn)).max(dim=1).values
        td = torch.tensor(rew) + hp.gamma * mx * (1 - torch.tensor(done, dtype=torch.float32))
    loss = ((qa - td) ** 2).mean()
    loss.backward()
    st["t"] += 1
    t = st["t"]
    new_p, new_m, new_v = [], [], []
    for p, m, v in zip(ps, [x for wb in st["m"] for x in wb], [x for wb in st["v"] for x in wb]):
        g = p.grad
        m = (1 - hp.beta1) * g + hp.beta1 * torch.tensor(m)
        v = (1 - hp.beta2) * g * g + hp.beta2 * torch.tensor(v)
        u = (m / (1 - hp.beta1 ** t)) / (torch.sqrt(v / (1 - hp.beta2 ** t)) + hp.adam_eps)
        new_p.append((p.detach() - hp.learning_rate * u).numpy())
        new_m.append(m.numpy())
        new_v.append(v.numpy())
    pair = lambda xs: [(xs[i], xs[i + 1]) for i in range(0, len(xs), 2)]  # noqa: E731
    st["online"], st["m"], st["v"] = pair(new_p), pair(new_m), pair(new_v)
    return float(loss.detach())


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / (1e-3 + np.max(np.abs(b))))


@pytest.mark.parametrize("sizes,batch,code_window", [((294, 128, 64, 5), 8, 7), ((150, 64, 5), 4, 0),
                                                     ((96, 32, 32, 32, 5), 16, 0)])
def test_oracle_learner_matches_torch_restatement(sizes, batch, code_window):
    """The oracle's learner step == autograd + optax's Adam formula (fp32
    PyTorch) within REL_TOL: loss, parameters and moments, step by step, with
    the target update (tau 0.7 every 3 steps) and the epsilon schedule."""
    hp = O.HParams(batch=batch, tau=0.7, target_update_interval=3, epsilon_decay=0.97, epsilon_decay_every=2,
                   sample_seed=11)
    cap = 300
    rep = _rand_replay(cap, sizes[0], seed=len(sizes) + batch, code_window=code_window)
    online, target = _rand_net(sizes, 1), _rand_net(sizes, 2)
    st = O.LearnerState.start(online, target, epsilon_start=1.0)
    ts = {"online": [(w.copy(), b.copy()) for w, b in online], "target": [(w.copy(), b.copy()) for w, b in target],
          "m": [(np.zeros_like(w), np.zeros_like(b)) for w, b in online],
          "v": [(np.zeros_like(w), np.zeros_like(b)) for w, b in online], "t": 0}
    eps = np.float32(1.0)
    for step in range(12):
        info = O.learner_step(st, hp, rep["obs"], rep["next_obs"], rep["actions"], rep["rewards"], rep["dones"],
                              cap, code_window)
        idx = info["rows"]
        if code_window:
            X, Xn = O.decode_code_rows(rep["obs"][idx], code_window), O.decode_code_rows(rep["next_obs"][idx],
                                                                                        code_window)
        else:
            X, Xn = rep["obs"][idx], rep["next_obs"][idx]
        loss = _torch_step(ts, hp, X, Xn, rep["actions"][idx], rep["rewards"][idx], rep["dones"][idx])
        assert abs(float(info["loss"]) - loss) <= REL_TOL * (1e-3 + abs(loss)), step
        if step % hp.target_update_interval == 0:
            ts["target"] = [(hp.tau * w + (1 - hp.tau) * tw, hp.tau * b + (1 - hp.tau) * tb)
                            for (w, b), (tw, tb) in zip(ts["online"], ts["target"])]
        for k in ("online", "target", "m", "v"):
            for (a, b), (c, d) in zip(getattr(st, k), ts[k]):
                assert _rel(a, c) <= REL_TOL and _rel(b, d) <= REL_TOL, (step, k)
        if step % hp.epsilon_decay_every == 0:
            eps = max(np.float32(eps * np.float32(hp.epsilon_decay)), np.float32(hp.epsilon_end))
        assert st.epsilon == eps and st.step == step + 1 and st.count == step + 1
        # resynchronise the torch side on the oracle (the comparison is per step)
        for k in ("online", "target", "m", "v"):
            ts[k] = [(w.copy(), b.copy()) for w, b in getattr(st, k)]


def test_oracle_learner_without_sample_only_schedules():
    """size < batch: no train_step (loss 0, parameters unchanged, Adam count
    unchanged) but the target update and the epsilon decay still run."""
    hp = O.HParams(batch=8, tau=0.5, target_update_interval=1)
    online, target = _rand_net((30, 32, 5), 3), _rand_net((30, 32, 5), 4)
    st = O.LearnerState.start(online, target, 1.0)
    rep = _rand_replay(16, 30, 5)
    info = O.learner_step(st, hp, rep["obs"], rep["next_obs"], rep["actions"], rep["rewards"], rep["dones"], 7)
    assert not info["trained"] and info["loss"] == 0 and st.count == 0 and st.step == 1
    for (w, b), (w0, b0) in zip(st.online, online):
        assert np.array_equal(w, w0) and np.array_equal(b, b0)
    for (tw, _), (w0, _), (t0, _) in zip(st.target, online, target):
        assert np.array_equal(tw, np.float32(0.5) * w0 + np.float32(0.5) * t0)
    assert st.epsilon == np.float32(np.float32(1.0) * np.float32(hp.epsilon_decay))


def test_train_jax_epsilon_decay_formula():
    """train_jax.py:133-134: half-way to epsilon_end after 20 % of the steps
    (per decay call, as the reference computes it)."""
    d = O.train_jax_epsilon_decay(1000)
    assert abs(d ** 200 - 0.505) < 1e-9


def test_sample_indices_in_range_and_uniform():
    rows = np.array([O.sample_indices(7, s, 64, 1000) for s in range(200)]).ravel()
    assert rows.min() >= 0 and rows.max() < 1000
    hist = np.bincount(rows // 100, minlength=10)
    assert hist.min() > 0.8 * rows.size / 10


# ------------------------------------------------------------ C ABI (CPU) ---
def _desc(in_features, hidden, inp=0, precision=1):
    from dronerl_amd.dqn import DrlQnetDesc
    h = list(hidden) + [0] * (3 - len(hidden))
    return DrlQnetDesc(in_features, len(hidden), (ctypes.c_int32 * 3)(*h), 5, precision, inp)


def test_dqn_layout_query():
    """The agent block: four parameter sets in torch state_dict order, 16-B
    aligned sections, the counters, the scratch; batch bounds; LDS fit."""
    from dronerl_amd._native import lib
    from dronerl_amd.dqn import DrlDqnLayout, _bind
    L = _bind(lib())
    lay = DrlDqnLayout()
    assert L.drl_dqn_layout_query(ctypes.byref(_desc(294, (128, 64), 1)), 8, ctypes.byref(lay)) == 0
    n = 294 * 128 + 128 + 128 * 64 + 64 + 64 * 8  # (the 5-row output layer padded to 4 floats: 320 -> 320, bias 5 -> 8)
    assert lay.weight_off[0] == 0 and lay.bias_off[0] == 294 * 128
    assert lay.weight_off[1] == 294 * 128 + 128 and lay.weight_off[2] == 294 * 128 + 128 + 128 * 64 + 64
    assert lay.n_params == 294 * 128 + 128 + 128 * 64 + 64 + 320 + 8 and n > 0
    assert (lay.online_off, lay.target_off, lay.m_off, lay.v_off) == tuple(i * 4 * lay.n_params for i in range(4))
    assert lay.counters_off == 16 * lay.n_params and lay.scratch_off == lay.counters_off + 64
    assert lay.bytes % 16 == 0 and lay.grad_workgroups == 2 + 2 * 128 // 4 and lay.grad_lds_bytes <= 159 * 1024
    for b, ok in ((0, False), (1, True), (64, True), (65, False)):
        assert (L.drl_dqn_layout_query(ctypes.byref(_desc(294, (128, 64), 1)), b, ctypes.byref(lay)) == 0) == ok
    # 8-unit layer-0 tiles: the widest input the nets take (512) fits a batch of 64 within 150 KB
    assert L.drl_dqn_layout_query(ctypes.byref(_desc(512, (64,), 0, 0)), 64, ctypes.byref(lay)) == 0
    assert lay.grad_lds_bytes <= 150 * 1024


def test_dqn_train_argument_checks():
    """drl_dqn_train validates before it launches (no GPU work reached)."""
    from dronerl_amd._native import lib
    from dronerl_amd.dqn import DrlDqnHParams, DrlReplay, _bind
    L = _bind(lib())
    d = _desc(294, (128, 64), 1)
    hp = DrlDqnHParams(8, 10, 5, 0, 0.9, 1e-3, 0.9, 0.999, 1e-8, 1.0, 0.999, 0.01, 0)
    fake = ctypes.c_void_p(1 << 20)
    rep = DrlReplay(1000, 32, 1 << 20, 1 << 20, 1 << 20, 1 << 20, 1 << 20)

    def call(h=hp, agent=fake, packed=fake, r=rep, size=100):
        return L.drl_dqn_train(ctypes.byref(d), ctypes.byref(h), agent, packed, ctypes.byref(r), size, None)
    assert call(size=1001) != 0 and b"size" in L.drl_last_error()
    assert call(size=-1) != 0
    assert call(agent=None) != 0 and b"agent" in L.drl_last_error()
    assert call(packed=ctypes.c_void_p((1 << 20) + 4)) != 0 and b"packed" in L.drl_last_error()
    bad = DrlDqnHParams(8, 0, 5, 0, 0.9, 1e-3, 0.9, 0.999, 1e-8, 1.0, 0.999, 0.01, 0)
    assert call(h=bad) != 0 and b"interval" in L.drl_last_error()
    bad = DrlDqnHParams(8, 10, 5, 0, 0.9, 1e-3, 1.0, 0.999, 1e-8, 1.0, 0.999, 0.01, 0)
    assert call(h=bad) != 0 and b"beta" in L.drl_last_error()
    wrong_rows = DrlReplay(1000, 294, 1 << 20, 1 << 20, 1 << 20, 1 << 20, 1 << 20)  # f32 rows for a code net
    assert call(r=wrong_rows) != 0 and b"policy code" in L.drl_last_error()


# ------------------------------------------------------------------- GPU ---
def _learner_setup(sizes, inp, hp_kw, E=64, cap=300, seed=0):
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    from dronerl_amd.dqn import DQNHParams, DQNLearner, QNetwork, ReplayBuffer
    radius = 3
    env = BatchedDeliveryDrones(EnvParams(n_drones=8, grid_size=16, window_radius=radius), E)
    env.reset(seed=seed)
    g = torch.Generator().manual_seed(seed + 5)
    net = QNetwork(sizes[0], sizes[1:-1], generator=g, precision="f32", input=inp)
    gb = torch.Generator(device="cuda").manual_seed(seed + 6)
    for b in net.biases:
        b.normal_(0, 0.05, generator=gb)
    net.pack()
    hp = DQNHParams(**hp_kw)
    target = ([torch.randn(w.shape, generator=g) * 0.1 for w in net.weights],
              [torch.randn(b.shape, generator=g) * 0.05 for b in net.biases])
    learner = DQNLearner(net, hp, target=target)
    rb = ReplayBuffer(cap, sizes[0], torch.device("cuda"), code_radius=radius if inp == "code" else 0)
    return env, net, learner, rb, hp


def _host(t):
    return t.detach().cpu().numpy().copy()


def state_from_learner(learner):
    st = O.LearnerState.start([(_host(w), _host(b)) for w, b in learner.params("online")],
                              [(_host(w), _host(b)) for w, b in learner.params("target")], 1.0)
    st.m = [(_host(w), _host(b)) for w, b in learner.params("m")]
    st.v = [(_host(w), _host(b)) for w, b in learner.params("v")]
    c = learner.counters()
    st.step, st.count, st.epsilon = c["step"], c["count"], np.float32(c["epsilon"])
    st.beta1_pow, st.beta2_pow = c["beta1_pow"], c["beta2_pow"]
    return st


class DevRows:
    """A device tensor read on demand by the oracle (rows it indexes only):
    the learner oracle gathers its 8 sampled rows of a 100,000-slot ring
    without copying the ring."""

    def __init__(self, t):
        self.t = t

    def __getitem__(self, idx):
        if isinstance(idx, tuple):
            return self[idx[0]][(slice(None),) + idx[1:]]
        if isinstance(idx, (int, np.integer)):
            return self.t[int(idx)].item()
        return self.t[torch.as_tensor(np.asarray(idx), device=self.t.device)].cpu().numpy()


def oracle_hparams(hp):
    return O.HParams(batch=hp.batch, gamma=hp.gamma, learning_rate=hp.learning_rate, beta1=hp.beta1, beta2=hp.beta2,
                     adam_eps=hp.adam_eps, tau=hp.tau, target_update_interval=hp.target_update_interval,
                     epsilon_decay=hp.decay(), epsilon_end=hp.epsilon_end,
                     epsilon_decay_every=hp.epsilon_decay_every, sample_seed=hp.sample_seed)


def oracle_step_on_ring(st, ohp, rb, code_window):
    """The oracle's learner step on the device ring's current contents."""
    return O.learner_step(st, ohp, DevRows(rb.obs), DevRows(rb.next_obs), DevRows(rb.actions), DevRows(rb.rewards),
                          DevRows(rb.dones), rb.size, code_window)


def assert_same(learner, st, where):
    for k in ("online", "target", "m", "v"):
        for l, ((w, b), (ow, ob)) in enumerate(zip(learner.params(k), getattr(st, k))):
            assert np.array_equal(_host(w).view(np.uint32), ow.view(np.uint32)), (where, k, l, "W")
            assert np.array_equal(_host(b).view(np.uint32), ob.view(np.uint32)), (where, k, l, "b")
    c = learner.counters()
    assert c["step"] == st.step and c["count"] == st.count, where
    assert np.float32(c["epsilon"]) == st.epsilon and np.float32(c["loss"]) == st.loss, where
    assert c["beta1_pow"] == st.beta1_pow and c["beta2_pow"] == st.beta2_pow, where


@gpu
@pytest.mark.parametrize("sizes,inp,hp_kw,E,cap", [
    ((294, 128, 64, 5), "code", dict(batch=8, num_steps=1000), 64, 300),                      # train_jax defaults
    ((294, 128, 64, 5), "obs", dict(batch=8, tau=0.6, target_update_interval=3), 50, 257),
    ((294, 64, 5), "code", dict(batch=1, epsilon_decay=0.9, epsilon_decay_every=1), 16, 100),
    ((294, 96, 32, 32, 5), "code", dict(batch=32, learning_rate=3e-3, gamma=0.95), 40, 500),
    ((294, 128, 64, 5), "code", dict(batch=64, target_update_interval=7, sample_seed=99), 24, 96),
    # narrow layer 0, wide later layers: the tails stage those weights layer by layer (no prefetch) and the
    # target-side shares exceed the registers' 8 per thread (the batched fallback update)
    ((294, 32, 128, 128, 5), "code", dict(batch=8, tau=0.5, target_update_interval=2), 32, 200),
])
def test_learner_matches_oracle_bit_exact(sizes, inp, hp_kw, E, cap):
    """The train_jax.py loop shape with the learner on: act (device epsilon)
    -> step -> replay add_many -> drl_dqn_train, 40 steps.  Before each train
    the ring is copied to the host and the oracle takes the same learner step:
    parameters, target, moments, loss and counters equal bit for bit after
    every step (including the first steps, where a batch larger than the
    ring's size skips train_step: buffers.py can_sample)."""
    env, net, learner, rb, hp = _learner_setup(sizes, inp, hp_kw, E=E, cap=cap)
    st = state_from_learner(learner)
    ohp = oracle_hparams(hp)
    W = 7
    cur = env.new_code() if inp == "code" else torch.empty((E, 1, W, W, 6), device="cuda")
    nxt = env.new_code() if inp == "code" else torch.empty((E, 1, W, W, 6), device="cuda")
    if inp == "code":
        env.get_code(out=cur)
    else:
        env.get_obs(1, out=cur)
    acts = torch.empty((E, 8), dtype=torch.int32, device="cuda")
    trained = 0
    for t in range(40):
        x = cur if inp == "code" else cur.reshape(E, -1)
        eps_before = float(learner.epsilon.item())
        assert np.float32(eps_before) == st.epsilon
        net.act(x, learner.epsilon, seed=3, step=t, actions=acts, synth=(5, t))
        if inp == "code":
            r, d = env.step(acts, code=nxt)
        else:
            r, d, _ = env.step(acts, obs_k=1, obs=nxt)
        rb.add_many(cur, acts, r, nxt, d)
        rep = {"obs": _host(rb.obs), "next_obs": _host(rb.next_obs), "actions": _host(rb.actions),
               "rewards": _host(rb.rewards), "dones": _host(rb.dones)}
        info = O.learner_step(st, ohp, rep["obs"], rep["next_obs"], rep["actions"], rep["rewards"], rep["dones"],
                              rb.size, W if inp == "code" else 0)
        trained += info["trained"]
        learner.train(rb)
        torch.cuda.synchronize()
        assert_same(learner, st, t)
        cur, nxt = nxt, cur
    net.check_errors()
    env.check_errors()
    assert trained >= 30
    # the act's packed image is the online net's: a fresh drl_qnet_pack of the same parameters is byte-identical
    after = net.packed.clone()
    net.pack()
    assert torch.equal(after, net.packed)


@gpu
def test_learner_act_reads_device_epsilon():
    """drl_qnet_act_eps == drl_qnet_act with the same epsilon value (both
    inputs, with and without the synthetic columns)."""
    from dronerl_amd.dqn import QNetwork
    env, net, learner, rb, hp = _learner_setup((294, 128, 64, 5), "code", dict(epsilon_start=0.37), E=777)
    code = env.new_code()
    _, _, obs = env.step(env.synth_actions(seed=1, step=0), obs_k=1, code=code)
    a1 = torch.full((777, 8), -1, dtype=torch.int32, device="cuda")
    a2 = a1.clone()
    net.act(code, learner.epsilon, seed=5, step=2, actions=a1, synth=(9, 4))
    net.act(code, float(learner.epsilon.item()), seed=5, step=2, actions=a2, synth=(9, 4))
    assert torch.equal(a1, a2)
    onet = QNetwork(294, (128, 64), precision="f32")
    onet.load(net.weights, net.biases)
    x = obs.reshape(777, -1)
    b1 = torch.empty((777, 1), dtype=torch.int32, device="cuda")
    b2 = b1.clone()
    onet.act(x, learner.epsilon, seed=5, step=2, actions=b1)
    onet.act(x, 0.37, seed=5, step=2, actions=b2)
    assert torch.equal(b1, b2)


@gpu
@pytest.mark.parametrize("cap,E", [(300, 64), (100, 160)])
def test_learner_fresh_batch_equals_serial(cap, E):
    """drl_dqn_train_fresh (the learner reads the latest add's rows from that
    add's own buffers, so the add may overlap it) leaves the same state, bit
    for bit, as drl_dqn_train after the add; also when the add overwrites the
    whole ring (E > capacity)."""
    from dronerl_amd.dqn import DQNHParams, DQNLearner, QNetwork, ReplayBuffer
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    env = BatchedDeliveryDrones(EnvParams(n_drones=8, grid_size=16), E)
    env.reset(seed=4)
    nets = [QNetwork(294, (128, 64), generator=torch.Generator().manual_seed(8), input="code") for _ in range(2)]
    hp = DQNHParams(batch=16, target_update_interval=3)
    lrs = [DQNLearner(n, hp, generator=torch.Generator().manual_seed(9)) for n in nets]
    rb = ReplayBuffer(cap, 294, torch.device("cuda"), code_radius=3)
    cur, nxt = env.new_code(), env.new_code()
    env.get_code(out=cur)
    acts = torch.empty((E, 8), dtype=torch.int32, device="cuda")
    for t in range(12):
        nets[0].act(cur, lrs[0].epsilon, seed=1, step=t, actions=acts, synth=(2, t))
        r, d = env.step(acts, code=nxt)
        batch = rb.add_many(cur, acts, r, nxt, d)
        lrs[0].train(rb)
        lrs[1].train(rb, fresh=batch)
        cur, nxt = nxt, cur
    torch.cuda.synchronize()
    for k in ("online", "target", "m", "v"):
        for (w0, b0), (w1, b1) in zip(lrs[0].params(k), lrs[1].params(k)):
            assert torch.equal(w0, w1) and torch.equal(b0, b1), k
    assert lrs[0].counters() == lrs[1].counters()
    assert torch.equal(nets[0].packed, nets[1].packed)
    for lr in lrs:
        lr.check_errors()


@gpu
def test_sample_slots_are_the_learners_draws():
    """DQNLearner.sample_slots (drl_dqn_sample_rows) == the slots the next
    train() draws (the oracle's sample_indices at the device step), step after
    step, for growing sizes; refused for an empty ring."""
    from dronerl_amd.handle import DroneRLError
    env, net, learner, rb, hp = _learner_setup((294, 128, 64, 5), "code", dict(batch=8, sample_seed=77), E=40,
                                               cap=300)
    cur, nxt = env.new_code(), env.new_code()
    env.get_code(out=cur)
    acts = torch.empty((40, 8), dtype=torch.int32, device="cuda")
    for t in range(12):
        net.act(cur, learner.epsilon, seed=3, step=t, actions=acts, synth=(5, t))
        r, d = env.step(acts, code=nxt)
        rb.add_many(cur, acts, r, nxt, d)
        slots = learner.sample_slots(rb.size)
        assert slots.cpu().tolist() == O.sample_indices(77, t, 8, rb.size), t
        learner.train(rb)
        cur, nxt = nxt, cur
    torch.cuda.synchronize()
    assert learner.counters()["step"] == 12
    with pytest.raises(DroneRLError):
        learner.sample_slots(0)


@gpu
def test_learner_handoff_timeout_is_reported_and_refused(monkeypatch):
    """a launch whose workgroup gives up on a hand-off sets the
    error flag; DQNLearner.check_errors raises; every later launch returns at
    once (parameters, moments, packed image and counters frozen: an aborted
    step's stale granules carry the same epoch and are never read); restart()
    (drl_dqn_init) zeroes the scratch and clears the flag, and training then
    matches the oracle again.  The hand-off is dropped with the debug knob
    DRL_DQN_DEBUG_DROP_HANDOFF (the online tail omits the epoch word)."""
    from dronerl_amd.handle import DroneRLError
    env, net, learner, rb, hp = _learner_setup((294, 128, 64, 5), "code", dict(batch=8), E=64, cap=300)
    cur, nxt = env.new_code(), env.new_code()
    env.get_code(out=cur)
    acts = torch.empty((64, 8), dtype=torch.int32, device="cuda")

    def fill(t):
        net.act(cur, learner.epsilon, seed=3, step=t, actions=acts, synth=(5, t))
        r, d = env.step(acts, code=nxt)
        rb.add_many(cur, acts, r, nxt, d)
        cur.copy_(nxt)

    fill(0)
    learner.train(rb)
    torch.cuda.synchronize()
    learner.check_errors()
    monkeypatch.setenv("DRL_DQN_DEBUG_DROP_HANDOFF", "1")
    learner.train(rb)
    torch.cuda.synchronize()
    monkeypatch.delenv("DRL_DQN_DEBUG_DROP_HANDOFF")
    with pytest.raises(DroneRLError):
        learner.check_errors()
    frozen = learner.block.clone()
    packed = net.packed.clone()
    for t in range(1, 4):
        fill(t)
        learner.train(rb)
    torch.cuda.synchronize()
    assert torch.equal(learner.block, frozen) and torch.equal(net.packed, packed)
    with pytest.raises(DroneRLError):
        learner.check_errors()
    # restart: counters from zero, the flag cleared, the granules zeroed; then bit-exact training again
    learner.restart()
    torch.cuda.synchronize()
    lay = learner.layout
    assert int(learner.block[lay.counters_off + 52:lay.counters_off + 56].view(torch.int32).item()) == 0
    learner.check_errors()
    st, ohp = state_from_learner(learner), oracle_hparams(hp)
    assert st.step == 0 and st.count == 0
    for t in range(4, 9):
        fill(t)
        O.learner_step(st, ohp, _host(rb.obs), _host(rb.next_obs), _host(rb.actions), _host(rb.rewards),
                       _host(rb.dones), rb.size, 7)
        learner.train(rb)
        torch.cuda.synchronize()
        assert_same(learner, st, f"after restart, step {t}")
    learner.check_errors()


@gpu
def test_learner_beside_co_running_kernels():
    """the learner's workgroups hand off to each other, so
    they must all become resident.  Each learner step here is launched on its
    own stream while a second stream keeps the device full: C5-sized env steps
    (131,072 envs, one-wave workgroups holding LDS on every CU) and a 1 GiB
    copy.  Every step still completes bit-exact against the oracle, with no
    hand-off timeout."""
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    env, net, learner, rb, hp = _learner_setup((294, 128, 64, 5), "code", dict(batch=8), E=64, cap=300)
    st, ohp = state_from_learner(learner), oracle_hparams(hp)
    big = BatchedDeliveryDrones(EnvParams(n_drones=32, grid_size=64), 131072)
    big.reset(seed=2)
    src = torch.empty(1 << 28, dtype=torch.float32, device="cuda").fill_(1.0)
    dst = torch.empty_like(src)
    busy, side = torch.cuda.Stream(), torch.cuda.Stream()
    cur, nxt = env.new_code(), env.new_code()
    env.get_code(out=cur)
    acts = torch.empty((64, 8), dtype=torch.int32, device="cuda")
    for t in range(6):
        net.act(cur, learner.epsilon, seed=3, step=t, actions=acts, synth=(5, t))
        r, d = env.step(acts, code=nxt)
        rb.add_many(cur, acts, r, nxt, d)
        torch.cuda.synchronize()
        O.learner_step(st, ohp, _host(rb.obs), _host(rb.next_obs), _host(rb.actions), _host(rb.rewards),
                       _host(rb.dones), rb.size, 7)
        # even steps: the learner goes in while the env steps run (the host
        # enqueues faster than they execute); odd steps: behind the copy
        for k in range(12):
            with torch.cuda.stream(busy):
                if t % 2 and k == 0:
                    dst.copy_(src)
                big.step(big.synth_actions(seed=9, step=12 * t + k))
            if k == 6:
                with torch.cuda.stream(side):
                    learner.train(rb)
        torch.cuda.synchronize()
        learner.check_errors()
        assert_same(learner, st, f"co-running, step {t}")
        cur, nxt = nxt, cur
    big.check_errors()
    assert learner.counters()["count"] == 6


@gpu
@pytest.mark.parametrize("inp", ["code", "obs"])
def test_learner_matches_torch_restatement_50_steps(inp):
    """VERDICT r4 item 1's check: 50 device learner steps (train_jax defaults:
    batch 8, lr 1e-3, gamma 0.9, tau 1.0 every 10, decay every 5) on a fixed,
    full replay; the rows of each step are the counter hash's
    (oracle.sample_indices reproduces them).  After every step the device's
    weights, target, both Adam moments and the loss equal an fp32 PyTorch
    restatement (autograd + optax's Adam formula written out, _torch_step)
    within 1e-5 relative; the torch side is then resynchronised on the
    device state (a per-step comparison, as optax itself is not importable:
    agreement with optax's code stays parity unpinned)."""
    tol = 1e-5
    env, net, learner, rb, hp = _learner_setup((294, 128, 64, 5), inp, dict(batch=8, num_steps=1000), E=64, cap=300)
    W = 7
    cur = env.new_code() if inp == "code" else torch.empty((64, 1, W, W, 6), device="cuda")
    nxt = env.new_code() if inp == "code" else torch.empty((64, 1, W, W, 6), device="cuda")
    if inp == "code":
        env.get_code(out=cur)
    else:
        env.get_obs(1, out=cur)
    for t in range(5):  # fill the 300-slot ring with 5 x 64 transitions (no adds during the 50 steps)
        acts = env.synth_actions(seed=9, step=t)
        if inp == "code":
            r, d = env.step(acts, code=nxt)
        else:
            r, d, _ = env.step(acts, obs_k=1, obs=nxt)
        rb.add_many(cur, acts, r, nxt, d)
        cur, nxt = nxt, cur
    assert rb.size == 300
    ohp = oracle_hparams(hp)
    obs, nobs = _host(rb.obs), _host(rb.next_obs)
    act_all, rew_all, done_all = _host(rb.actions), _host(rb.rewards), _host(rb.dones)

    def dev_state():
        return {k: [(_host(w), _host(b)) for w, b in learner.params(k)] for k in ("online", "target", "m", "v")}

    ts = dev_state()
    ts["t"] = 0
    for step in range(50):
        assert learner.counters()["step"] == step
        idx = O.sample_indices(hp.sample_seed, step, hp.batch, rb.size)
        if inp == "code":
            X, Xn = O.decode_code_rows(obs[idx], W), O.decode_code_rows(nobs[idx], W)
        else:
            X, Xn = obs[idx, :294], nobs[idx, :294]
        loss = _torch_step(ts, ohp, X, Xn, act_all[idx], rew_all[idx], done_all[idx])
        if step % hp.target_update_interval == 0:
            ts["target"] = [(ohp.tau * w + (1 - ohp.tau) * tw, ohp.tau * b + (1 - ohp.tau) * tb)
                            for (w, b), (tw, tb) in zip(ts["online"], ts["target"])]
        learner.train(rb)
        dev = dev_state()
        c = learner.counters()
        assert abs(c["loss"] - loss) <= tol * (1e-3 + abs(loss)), step
        for k in ("online", "target", "m", "v"):
            for l, ((a, b), (e, f)) in enumerate(zip(dev[k], ts[k])):
                assert _rel(a, e) <= tol and _rel(b, f) <= tol, (step, k, l)
        dev["t"] = ts["t"]
        ts = dev  # resynchronise on the device state
    learner.check_errors()
