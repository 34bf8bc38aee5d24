"""Full-size parity against the oracle over EVERY env.

1. C3 / C4 / C5 per-GPU shares (65,536 / 65,536 / 131,072 envs): the HIP
   path and the threaded oracle rollout (oracle/dronerl_oracle.c
   orc_rollout: random.seed(123 + g), torch_impl reset, synthetic actions)
   run the same steps; the final state of every env (ground, dict order,
   positions, charge, carry, all 625 MT words) is compared bit for bit, with
   every env's done count and reward sum.  Size-independent invariants are
   checked over every env as well.
   The last step runs the headline kernel instance (fused obs(K=1)), and every
   env's observation is compared with the oracle's.
2. The C5 scan-style train-loop segment (train_jax.py:38-115, reset every
   100 steps :359): per step, synthetic actions for drones 1..N-1 plus the
   epsilon-greedy DQN action of drone 0 (one drl_qnet_act_synth launch),
   step + fused obs(K=1), replay add_many of the drone-0 transition; after
   100 steps a reset of every env and its observation.  The oracle is driven
   by the kernel's actions; env state, rewards, dones and the observation are
   compared every step, and the replay ring at the end against the ring the
   oracle's transitions give.
3. The exact loops bench.py times (`train_loop` and `c5.train_loop`): C3 at
   65,536 envs on the 100,000-slot ring, and C5's 64x64 / 32-drone compile-time
   instance with more envs than ring slots (8,192 into 5,000, the regime of
   131,072 into 100,000); f32 nets on drone 0's policy code, the fused replay
   add, the device learner, bench.TrainSegment's own calls, then its reset.
   The oracle is driven by the kernel's actions; every step compares rewards,
   dones and the code the step wrote (decoded on the host) with the oracle's
   observation, and the learner with oracle/dqn_learner.py bit for bit; the
   state every 10 steps; the act's Q on the step's code against an f32
   forward of the oracle's observation; the code ring and sample()'s decoded
   rows against the oracle's transitions; the reset's state and first code.
"""
import os

import numpy as np
import pytest
import torch

from oracle.oracle import OracleMulti, Params as OParams, rollout
from tests.test_gpu_parity import EnvParams, Env, assert_rewards, assert_state, gpu_state, oparams

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.mark.parametrize("cfg,E,steps", [
    (dict(n_drones=8, grid_size=16), 65536, 200),       # C3 on one GPU
    (dict(n_drones=16, grid_size=32), 65536, 100),      # C4 per-GPU share (262144 / 4)
    (dict(n_drones=32, grid_size=64), 131072, 60),      # C5 per-GPU share (2**20 / 8)
])
def test_full_size_every_env_matches_oracle(cfg, E, steps):
    p = EnvParams(**cfg)
    N, G = p.n_drones, p.side
    env = Env(p, E)
    env.reset(seed=123)
    rsum = torch.zeros(E, dtype=torch.float64, device=env.device)
    dsum = torch.zeros(E, dtype=torch.int64, device=env.device)
    for t in range(steps):
        # the last step is the headline kernel instance: fused obs(K=1)
        out = env.step(env.synth_actions(seed=77, step=t), obs_k=1 if t == steps - 1 else 0)
        r, dn = out[0], out[1]
        rsum += r.double().sum(1)
        dsum += dn.sum(1)
    obs = out[2]
    torch.cuda.synchronize()
    env.check_errors()
    o = rollout(oparams(p), E, steps, seed0=123, action_seed=77, nthreads=THREADS)
    assert_state(gpu_state(env), o, f"{G}x{G}/{N}, {E} envs x {steps} steps")
    # every env's observation of drone 0 after the last step, against the oracle's WindowedGridView of its
    # own final state (wrappers.py:10-31,55-73)
    om = OracleMulti(oparams(p), E)
    om.set_state(o["ground"], o["order"], o["y"], o["x"], o["charge"], o["packet"], o["mt"])
    want = om.obs(3, 1)
    got = obs.cpu().numpy()
    if not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
        bad = np.argwhere((got != want).reshape(E, -1).any(1)).ravel()
        raise AssertionError(f"obs differs in envs {bad[:10]} (of {len(bad)})")
    del om, want, got
    np.testing.assert_array_equal(dsum.cpu().numpy(), o["done_sum"])
    assert np.abs(rsum.cpu().numpy() - o["reward_sum"]).max() <= steps * N * 1e-6
    # size-independent invariants over every env
    d = env.decode()
    gr = d["ground"]
    cnt = lambda v: (gr == v).sum(dim=(1, 2))  # noqa: E731
    assert torch.all(cnt(2) == 3 * N) and torch.all(cnt(3) == 2 * N) and torch.all(cnt(4) == 2 * N)
    assert torch.all(cnt(5) + d["carrying"].sum(1) == 3 * N)
    cells = d["y"].long() * G + d["x"].long()
    assert torch.all(cells.sort(1).values.diff(dim=1) > 0)  # distinct cells
    assert not (torch.gather(gr.view(E, -1), 1, cells) == 2).any()
    assert torch.all((d["charge"] >= 1) & (d["charge"] <= 100))
    assert torch.all(d["order"].sort(1).values == torch.arange(N, device=env.device))
    assert torch.all(d["mt_index"] <= 624)


@pytest.mark.parametrize("E,seg", [(4096, 100)])
def test_c5_train_loop_segment_matches_oracle(E, seg):
    from dronerl_amd.dqn import QNetwork, ReplayBuffer
    p = EnvParams(n_drones=32, grid_size=64)
    N = p.n_drones
    dev = torch.device("cuda:0")
    env = Env(p, E)
    env.reset(seed=3)
    o = OracleMulti(oparams(p), E)
    o.reset(3 + np.arange(E))
    W = env.layout.obs_window
    D = W * W * 6
    net = QNetwork(D, (128, 64), device=dev, generator=torch.Generator().manual_seed(0))
    cap = 10000
    rb = ReplayBuffer(cap, D, dev)
    obs = [torch.empty((E, 1, W, W, 6), device=dev) for _ in range(2)]
    acts = torch.empty((E, N), dtype=torch.int32, device=dev)
    rew = torch.empty((E, N), device=dev)
    don = torch.empty((E, N), dtype=torch.uint8, device=dev)
    env.get_obs(1, out=obs[0])
    np.testing.assert_array_equal(obs[0].cpu().numpy(), o.obs(3, 1), err_msg="first obs")
    hist = {}  # drone-0 transitions of the steps the ring keeps, from the oracle
    t_keep = (seg * E - cap) // E
    o_prev = o.obs(3, 1)
    for t in range(seg):
        cur, nxt = obs[t & 1], obs[(t + 1) & 1]
        net.act(cur.reshape(E, -1), 0.1, seed=7, step=t, actions=acts, synth=(2024, t))
        env.step(acts, obs_k=1, rewards=rew, dones=don, obs=nxt)
        rb.add_many(cur, acts, rew, nxt, don)
        a = acts.cpu().numpy()
        # drones 1..N-1 follow the synthetic stream; drone 0 the policy
        np.testing.assert_array_equal(a[:, 1:], env.synth_actions(seed=2024, step=t).cpu().numpy()[:, 1:])
        assert ((a[:, 0] >= 0) & (a[:, 0] < 5)).all()
        ro, do = o.step(a, nthreads=THREADS)
        ctx = f"C5 loop step {t}"
        assert_rewards(rew.cpu().numpy(), ro, ctx)
        np.testing.assert_array_equal(don.cpu().numpy().astype(bool), do, err_msg=ctx)
        o_next = o.obs(3, 1)
        np.testing.assert_array_equal(nxt.cpu().numpy(), o_next, err_msg=f"{ctx} obs")
        if t % 10 == 9 or t == seg - 1:
            assert_state(gpu_state(env), o.state(), ctx)
        if t >= t_keep:
            hist[t] = (o_prev.reshape(E, -1), a[:, 0].copy(), ro[:, 0].astype(np.float32), o_next.reshape(E, -1),
                       do[:, 0])
        o_prev = o_next
    env.check_errors()
    # replay ring (buffers.py:57-80): transition i (step i // E, env i % E) in slot i % cap, later writes win
    torch.cuda.synchronize()
    assert rb.cursor == (seg * E) % cap and rb.size == cap
    first = seg * E - cap
    slots = np.arange(first, seg * E)
    tt, ee = slots // E, slots % E
    want_obs = np.stack([hist[t][0][e] for t, e in zip(tt, ee)])
    want_next = np.stack([hist[t][3][e] for t, e in zip(tt, ee)])
    order = slots % cap
    np.testing.assert_array_equal(rb.obs.cpu().numpy()[order], want_obs)
    np.testing.assert_array_equal(rb.next_obs.cpu().numpy()[order], want_next)
    np.testing.assert_array_equal(rb.actions.cpu().numpy()[order], [hist[t][1][e] for t, e in zip(tt, ee)])
    np.testing.assert_array_equal(rb.rewards.cpu().numpy()[order], [hist[t][2][e] for t, e in zip(tt, ee)])
    np.testing.assert_array_equal(rb.dones.cpu().numpy()[order].astype(bool), [hist[t][4][e] for t, e in zip(tt, ee)])
    # reset_env_every: a reset of every env continuing each stream, then its observation
    env.reset(seed=None)
    o.reset(None)
    assert_state(gpu_state(env), o.state(), "C5 loop reset")
    np.testing.assert_array_equal(env.get_obs(1).cpu().numpy(), o.obs(3, 1), err_msg="C5 loop reset obs")


@pytest.mark.parametrize("name,G,N,E,seg,cap", [
    ("C3", 16, 8, 65536, 100, 100_000),   # the bench's train_loop: 65,536 envs, the reference's 100,000-slot ring
    # the bench's c5.train_loop instance (drl_step_kernel<32, Geo<64,32,3,1>, ..., fused replay>) in its
    # E > capacity regime (131,072 envs into 100,000 slots there)
    ("C5", 64, 32, 8192, 40, 5000),
])
def test_code_train_loop_matches_oracle(name, G, N, E, seg, cap):
    """bench.TrainSegment's own calls (C3: 65,536 envs x 100 steps; C5's
    64x64 / 32-drone instance with more envs than ring slots): the env against
    the env oracle every step, the act against an f32 forward of the live
    (learning) net, the learner (drl_dqn_train; train_jax.py:173 ring) against
    oracle/dqn_learner.py bit for bit every step, the code ring, sample() and
    the reset."""
    import bench
    from tests.test_dqn_learner import assert_same, oracle_hparams, oracle_step_on_ring, state_from_learner
    from tests.test_policy_code import decode_code
    p = EnvParams(n_drones=N, grid_size=G)
    env = Env(p, E)
    env.reset(seed=5)
    o = OracleMulti(oparams(p), E)
    o.reset(5 + np.arange(E))
    # the bench's own loop (one stream, fused act + fused replay add)
    loop = bench.TrainSegment(env, seg, precision="f32", input="code", capacity=cap)
    assert loop.input == "code" and loop.net.precision == "f32" and loop.rb.code_radius == 3
    assert loop.rb.capacity == cap and loop.learner is not None
    assert loop.fuse_replay  # the ring is written by the step itself (drl_step_code_replay; _replay is a no-op)
    lst, ohp = state_from_learner(loop.learner), oracle_hparams(loop.learner.hp)
    W = env.layout.obs_window
    want0 = o.obs(3, 1)[:, 0]
    assert np.array_equal(decode_code(loop.code[0].cpu().numpy(), W), want0), "first code"
    cap = loop.rb.capacity
    t_keep = (seg * E - cap) // E
    hist, prev = {}, want0
    for t in range(seg):
        b, nb = t % loop.NB, (t + 1) % loop.NB
        assert np.float32(loop.learner.epsilon.item()) == lst.epsilon
        loop._act_step(t)
        loop._replay(t)
        info = oracle_step_on_ring(lst, ohp, loop.rb, W)
        assert info["trained"]  # E >= batch transitions from the first step on: can_sample
        loop._learn()
        assert_same(loop.learner, lst, f"{name} learner step {t}")
        a = loop.acts[b].cpu().numpy()
        syn = env.synth_actions(seed=2024, step=t).cpu().numpy()
        if loop.synth_in_step:  # the step drew drones 1..N-1 itself (drl_step_code_replay_synth)
            a = np.concatenate([a[:, :1], syn[:, 1:]], 1)
        else:
            np.testing.assert_array_equal(a[:, 1:], syn[:, 1:])
        assert ((a[:, 0] >= 0) & (a[:, 0] < 5)).all()
        ro, do = o.step(a, nthreads=THREADS)
        ctx = f"{name} code loop step {t}"
        assert_rewards(loop.rewards[b].cpu().numpy(), ro, ctx)
        np.testing.assert_array_equal(loop.dones[b].cpu().numpy().astype(bool), do, err_msg=ctx)
        nxt = o.obs(3, 1)[:, 0]
        got = decode_code(loop.code[nb].cpu().numpy(), W)
        if not np.array_equal(got.view(np.uint32), nxt.view(np.uint32)):
            bad = np.argwhere((got != nxt).reshape(E, -1).any(1)).ravel()
            raise AssertionError(f"{ctx}: code differs from the oracle's observation in envs {bad[:10]}")
        if t % 10 == 9:
            assert_state(gpu_state(env), o.state(), ctx)
        if t in (0, seg // 2 + 7, seg - 1):  # the act on the step's code == an f32 forward of the oracle's observation
            q = torch.empty((E, 5), device=env.device)
            tmp = torch.empty((E, 1), dtype=torch.int32, device=env.device)
            loop.net.act(loop.code[nb], 0.0, actions=tmp, q_out=q)
            x = torch.from_numpy(nxt.reshape(E, -1))
            ref = x
            for i, (w, bias) in enumerate(zip(loop.net.weights, loop.net.biases)):
                ref = ref @ w.cpu().t() + bias.cpu()
                if i < len(loop.net.weights) - 1:
                    ref = torch.relu(ref)
            scale = 1.0 + ref.abs().amax(dim=1, keepdim=True)
            assert ((q.cpu() - ref).abs() / scale).max().item() <= 1e-5, ctx
        if t >= t_keep:
            hist[t] = (prev, a[:, 0].copy(), ro[:, 0].astype(np.float32), nxt, do[:, 0])
        prev = nxt
    torch.cuda.synchronize()
    env.check_errors()
    loop.net.check_errors()
    # the code ring (buffers.py:57-80): transition i (step i // E, env i % E) in slot i % cap, decoded
    rb = loop.rb
    assert rb.cursor == (seg * E) % cap and rb.size == cap
    slots = np.arange(seg * E - cap, seg * E)
    tt, ee, order = slots // E, slots % E, slots % cap
    want_obs = np.stack([hist[t][0][e] for t, e in zip(tt, ee)])
    want_next = np.stack([hist[t][3][e] for t, e in zip(tt, ee)])
    np.testing.assert_array_equal(decode_code(rb.obs.cpu().numpy(), W)[order], want_obs)
    np.testing.assert_array_equal(decode_code(rb.next_obs.cpu().numpy(), W)[order], want_next)
    np.testing.assert_array_equal(rb.actions.cpu().numpy()[order], [hist[t][1][e] for t, e in zip(tt, ee)])
    np.testing.assert_array_equal(rb.rewards.cpu().numpy()[order], [hist[t][2][e] for t, e in zip(tt, ee)])
    np.testing.assert_array_equal(rb.dones.cpu().numpy()[order].astype(bool), [hist[t][4][e] for t, e in zip(tt, ee)])
    # sample(): the device decode of the drawn rows == the oracle's transitions
    idx = torch.randint(0, rb.size, (256,), device=env.device,
                        generator=torch.Generator(device=env.device).manual_seed(3))  # what sample() draws
    smp = rb.sample(256, generator=torch.Generator(device=env.device).manual_seed(3))
    slot_of = np.empty(cap, np.int64)
    slot_of[order] = np.arange(cap)
    k = slot_of[idx.cpu().numpy()]
    np.testing.assert_array_equal(smp["obs"].cpu().numpy(), want_obs[k].reshape(256, -1))
    np.testing.assert_array_equal(smp["next_obs"].cpu().numpy(), want_next[k].reshape(256, -1))
    acts_want = np.asarray([hist[t][1][e] for t, e in zip(tt, ee)])
    np.testing.assert_array_equal(smp["actions"].cpu().numpy(), acts_want[k])
    # reset_env_every (train_jax.py:101-113), as TrainSegment.run ends: every stream continues; first code
    env.reset(seed=None)
    loop._first_obs()
    o.reset(None)
    assert_state(gpu_state(env), o.state(), f"{name} code loop reset")
    assert np.array_equal(decode_code(loop.code[0].cpu().numpy(), W), o.obs(3, 1)[:, 0]), "reset code"
