"""The global learner's host logic on the CPU (dronerl_amd.global_learner;
VERDICT r5 item 6).  Reference: train_jax.py:59-82 (one add_many of every
env's drone-0 transition into one ring, one train_step per step),
:196-212 (envs sharded over devices), jax_impl/buffers.py:57-90.

1. shard_add_plan + slot_owner against a simulated global ring: for every
   slot, the rank the owner function names holds, in its own image, exactly
   the transition the global ring holds (world 1-8, the ring wrapping inside an
   add, adds larger than the ring).
2. exchange_rows over a gloo world-size-2 group: every rank ends with the
   owners' rows, bit for bit.
3. The whole scheme with the learner oracle (oracle/dqn_learner.py) standing
   in for drl_dqn_train: two gloo ranks with half the envs each end, after 20
   steps, with parameters, moments and counters equal bit for bit to one
   learner over the concatenated ring.  (The same scheme on the device
   learner: tests/test_gpu_multirank.py::test_global_learner_two_ranks_equal_one_learner.)
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from dronerl_amd.global_learner import exchange_rows, shard_add_plan, slot_owner


@pytest.mark.parametrize("E,world,cap,steps", [
    (8, 1, 20, 7), (8, 2, 20, 7), (12, 4, 25, 9), (16, 8, 1000, 5),
    (64, 2, 50, 4),    # one add overfills the ring: only the last 50 envs land
    (64, 4, 40, 5),    # ... and whole shards land nothing
    (30, 3, 31, 12),   # capacity coprime with the add size
])
def test_shard_add_plan_and_owner_match_global_ring(E, world, cap, steps):
    Er = E // world
    gid = np.full(cap, -1, np.int64)
    img = np.full((world, cap), -1, np.int64)
    n = 0
    for _ in range(steps):
        first = max(0, E - cap)
        for j in range(first, E):  # buffers.py add_many: row j at (cursor + j) % cap, the last `cap` kept
            gid[(n + j) % cap] = n + j
        for r in range(world):
            lo, cur = shard_add_plan(n, cap, E, r * Er, Er)
            for k in range(Er - lo):
                img[r, (cur + k) % cap] = n + r * Er + lo + k
        n += E
        filled = np.flatnonzero(gid >= 0)
        owner = slot_owner(torch.from_numpy(filled), n, cap, E, world).numpy()
        assert np.array_equal(owner, (gid[filled] % E) // Er)
        assert np.array_equal(img[owner, filled], gid[filled])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _exchange_worker(rank, world, port, out):
    dist = _init(rank, world, port)
    try:
        g = np.random.default_rng(5)
        owner = torch.from_numpy(g.integers(0, world, 16))
        truth = torch.from_numpy(g.integers(-2**31, 2**31 - 1, (16, 11)).astype(np.int32))
        junk = torch.from_numpy(np.random.default_rng(100 + rank).integers(-2**31, 2**31 - 1, (16, 11)).astype(np.int32))
        mine = torch.where((owner == rank)[:, None], truth, junk)
        out[rank] = (exchange_rows(mine, owner, world).numpy(), truth.numpy())
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    with ctx.Manager() as man:
        out = man.dict()
        port = _free_port()
        procs = [ctx.Process(target=target, args=(r, world, port, *args, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
            assert p.exitcode == 0, p.exitcode
        return dict(out)


def test_exchange_rows_gloo_two_ranks():
    res = _spawn(_exchange_worker, 2)
    for r in range(2):
        got, truth = res[r]
        assert np.array_equal(got, truth)


# --------------------------------------- the scheme with the learner oracle ---
E_TOT, N_IN, STEPS = 64, 48, 20


def _transitions(t):
    """Step t's drone-0 transitions of every env (a stand-in for the env)."""
    g = np.random.default_rng(1000 + t)
    return {"obs": (g.random((E_TOT, N_IN)) < 0.3).astype(np.float32),
            "next_obs": (g.random((E_TOT, N_IN)) < 0.3).astype(np.float32),
            "actions": g.integers(0, 5, E_TOT).astype(np.int32),
            "rewards": g.choice(np.array([0.0, 1.0, -1.0, -0.1], np.float32), E_TOT),
            "dones": (g.random(E_TOT) < 0.1).astype(np.uint8)}


def _oracle_run(rank, world, cap):
    from oracle import dqn_learner as O
    from tests.test_dqn_learner import _rand_net
    hp = O.HParams(batch=8, gamma=0.9, learning_rate=1e-3, beta1=0.9, beta2=0.999, adam_eps=1e-8, tau=1.0,
                   target_update_interval=3, epsilon_decay=0.99, epsilon_end=0.01, epsilon_decay_every=5,
                   sample_seed=4)
    st = O.LearnerState.start(_rand_net((N_IN, 32, 5), 1), _rand_net((N_IN, 32, 5), 2), 1.0)
    ring = {"obs": np.zeros((cap, N_IN), np.float32), "next_obs": np.zeros((cap, N_IN), np.float32),
            "actions": np.zeros(cap, np.int32), "rewards": np.zeros(cap, np.float32), "dones": np.zeros(cap, np.uint8)}
    Er, off = E_TOT // world, rank * (E_TOT // world)
    n = 0
    for t in range(STEPS):
        tr = _transitions(t)
        lo, cur = shard_add_plan(n, cap, E_TOT, off, Er)  # this shard's rows (world 1: every env)
        for k in range(Er - lo):
            for f in ring:
                ring[f][(cur + k) % cap] = tr[f][off + lo + k]
        n += E_TOT
        size = min(n, cap)
        if world > 1 and size >= hp.batch:
            slots = torch.tensor(O.sample_indices(hp.sample_seed, st.step, hp.batch, size), dtype=torch.int64)
            owner = slot_owner(slots, n, cap, E_TOT, world)
            s = slots.numpy()
            packed = torch.from_numpy(np.concatenate(
                [ring["obs"][s].view(np.int32), ring["next_obs"][s].view(np.int32), ring["actions"][s][:, None],
                 ring["rewards"][s].view(np.int32)[:, None], ring["dones"][s].astype(np.int32)[:, None]], 1))
            rows = exchange_rows(packed, owner, world).numpy()
            ring["obs"][s] = rows[:, :N_IN].view(np.float32)
            ring["next_obs"][s] = rows[:, N_IN:2 * N_IN].view(np.float32)
            ring["actions"][s] = rows[:, 2 * N_IN]
            ring["rewards"][s] = rows[:, 2 * N_IN + 1].view(np.float32)
            ring["dones"][s] = rows[:, 2 * N_IN + 2].astype(np.uint8)
        O.learner_step(st, hp, ring["obs"], ring["next_obs"], ring["actions"], ring["rewards"], ring["dones"], size, 0)
    return {"online": O.flat(st.online), "target": O.flat(st.target), "m": O.flat(st.m), "v": O.flat(st.v),
            "counters": (st.step, st.count, float(st.epsilon), float(st.loss))}


def _oracle_worker(rank, world, port, cap, out):
    dist = _init(rank, world, port)
    try:
        out[rank] = _oracle_run(rank, world, cap)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cap", [200, 40])  # the ring wraps; one add (64 envs) overfills it
def test_global_learner_scheme_two_ranks_equal_one_learner_oracle(cap):
    ref = _oracle_run(0, 1, cap)
    assert ref["counters"][1] == STEPS
    res = _spawn(_oracle_worker, 2, cap)
    for r in range(2):
        for k in ("online", "target", "m", "v"):
            assert np.array_equal(res[r][k].view(np.uint32), ref[k].view(np.uint32)), (r, k)
        assert res[r]["counters"] == ref["counters"]


def test_train_cli_mirrors_train_jax():
    """dronerl_amd.train's command line: train_jax.py's option names and
    defaults (:335-390), its epsilon-decay formula (:133-134) and its
    validations (:393-402)."""
    from dronerl_amd import train as T
    a = T.parse_args([])
    assert (a.n_drones, a.grid_size, a.window_radius, a.num_envs, a.num_steps, a.batch_size) == (4, 9, 3, 1, 1000, 8)
    assert (a.memory_size, a.gamma, a.target_update_interval, a.reset_env_every, a.tau) == (100_000, 0.9, 10, 100, 1.0)
    hp = T.hparams_of(a)
    assert hp.epsilon_decay == pytest.approx((1 - 0.5 * (1 - 0.01 / 1.0)) ** (1 / (0.2 * 1000)), rel=0, abs=0)
    assert hp.batch == 8 and hp.learning_rate == 1e-3 and hp.epsilon_decay_every == 5
    p = T.env_params_of(T.parse_args(["--eval_grid_size", "16", "--eval_n_drones", "8"]), eval_env=True)
    assert (p.side, p.n_drones) == (16, 8)
    for bad in (["--num_envs", "0"], ["--num_steps", "0"], ["--use_sharding", "--num_envs", "1"]):
        with pytest.raises(ValueError):
            T.parse_args(bad)
