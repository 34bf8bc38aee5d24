"""Multi-rank runs of the HIP env, on the one-GPU box.

Two processes share cuda:0 over a gloo process group (the driver's
multi-GPU runs use nccl = RCCL, one device per rank; the data path is the
same: contiguous env shards with env_offset = rank * E / world, train_jax.py
:196-212, and one all-reduce of the eval table, :270-319).

1. evaluate_sharded with gpu_episode_runner (greedy DQN for drone 0, f32
   numerics) on 2 ranks == the one-process table, bit for bit.
2. Sharded stepping: each rank steps its shard; the concatenated final
   states == one process stepping every env.
3. bench.py under torch.distributed.run with 2 ranks (DRL_DIST_BACKEND=gloo)
   prints one whole-job JSON line.
4. The global learner (dronerl_amd.global_learner): 2 ranks with half the
   envs each == one learner over every env, bit for bit.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NUM_EVALS, EVAL_STEPS, EVAL_SEED = 9, 60, 845
STEP_E, STEP_T = 2048, 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _params():
    from dronerl_amd import EnvParams
    return EnvParams(n_drones=8, grid_size=16)


def _policy():
    from dronerl_amd.dqn import QNetwork
    net = QNetwork(294, (128, 64), device="cuda:0", generator=torch.Generator().manual_seed(5), precision="f32")

    def act(obs):
        a = torch.empty((obs.shape[0], 1), dtype=torch.int32, device=obs.device)
        net.act(obs.contiguous(), 0.0, actions=a)
        return a[:, 0]
    return act


def _shard_states(rank, world):
    from dronerl_amd import BatchedDeliveryDrones
    from dronerl_amd.distributed import shard_envs
    sh = shard_envs(STEP_E, rank, world)
    env = BatchedDeliveryDrones(_params(), sh.num_envs, device="cuda:0", env_offset=sh.env_offset)
    env.reset(seed=11)
    for t in range(STEP_T):
        env.step(env.synth_actions(seed=3, step=t))
    torch.cuda.synchronize()
    env.check_errors()
    d = env.decode()
    return {k: d[k].cpu().numpy() for k in ("ground", "order", "y", "x", "charge", "carrying", "mt_index")}


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from dronerl_amd.distributed import evaluate_sharded, gpu_episode_runner
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        runner = gpu_episode_runner(_params(), EVAL_STEPS, EVAL_SEED, policy=_policy(), device="cuda:0")
        agent, rnd, table = evaluate_sharded(runner, NUM_EVALS, rank=rank, world=world)
        out[rank] = (agent, rnd, table.cpu().numpy(), _shard_states(rank, world))
    finally:
        dist.destroy_process_group()


def test_two_ranks_eval_and_shards_match_one_process():
    from dronerl_amd.distributed import evaluate_sharded, gpu_episode_runner
    runner = gpu_episode_runner(_params(), EVAL_STEPS, EVAL_SEED, policy=_policy(), device="cuda:0")
    ref_agent, ref_rnd, ref_table = evaluate_sharded(runner, NUM_EVALS)
    ref_states = _shard_states(0, 1)
    ctx = mp.get_context("spawn")
    with ctx.Manager() as man:
        out = man.dict()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
            assert p.exitcode == 0, p.exitcode
        res = dict(out)
    for r in range(2):
        agent, rnd, table, _ = res[r]
        np.testing.assert_array_equal(table, ref_table.cpu().numpy())
        assert (agent, rnd) == (ref_agent, ref_rnd)
    for k, v in ref_states.items():
        np.testing.assert_array_equal(np.concatenate([res[0][3][k], res[1][3][k]]), v, err_msg=k)


def test_bench_two_ranks_gloo_whole_job_json():
    env = dict(os.environ, DRL_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", DRL_BENCH_PMC="0")
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "20", "--warmup", "5", "--envs", "4096", "--no-cpu-baseline", "--no-dqn",
           "--no-reset-bench", "--rollout-chunk", "0", "--loop-segments", "0", "--cached-steps", "10",
           "--c5-envs", "1024", "--strong-envs", "4096"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 20
    assert d["config"]["num_envs_total"] == 2 * 4096 and d["config"]["parallelism"] == "env-shard x2"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value = every rank's env-steps over the slowest rank's wall time
    assert d["value"] == pytest.approx(2 * 4096 * 20 / (d["ms_per_step"] * 20 / 1e3), rel=1e-6)
    assert d["streaming_obs"]["value"] > 0 and d["config"]["obs_stores"] == "cached"
    # the north-star sub-record: whole-job envs over both ranks, the same timing rule
    c5 = d["c5"]
    assert c5["config"]["num_envs_total"] == 2 * 1024 and c5["steps"] >= 200 and c5["n_gpus"] == 2
    assert c5["value"] == pytest.approx(2 * 1024 * c5["steps"] / (c5["ms_per_step"] * c5["steps"] / 1e3), rel=1e-6)
    # the strong-scaling sub-record: 4096 envs over the job, 2048 per rank
    st = d["strong"]
    assert st["scaling"] == "strong" and st["num_envs_total"] == 4096 and st["num_envs_per_gpu"] == 2048
    assert st["value"] == pytest.approx(4096 * 20 / (st["ms_per_step"] * 20 / 1e3), rel=1e-6)


def test_bench_gpus2_launches_its_own_ranks():
    """a plain `bench.py --gpus 2` (no torchrun) starts
    its own 2 ranks (here gloo, both on the one GPU) and relays rank 0's one
    whole-job line: n_gpus 2, 2x the envs, and the north-star C5 sub-record
    at 131,072 envs per rank (262,144 over the job)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(DRL_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", DRL_BENCH_PMC="0")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
           "--envs", "4096", "--no-cpu-baseline", "--no-dqn", "--no-reset-bench", "--rollout-chunk", "0",
           "--loop-segments", "0", "--cached-steps", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith('{"metric"'), r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["num_envs_total"] == 2 * 4096
    assert d["config"]["parallelism"] == "env-shard x2"
    assert d["c5"]["config"]["num_envs_total"] == 262144 and d["c5"]["n_gpus"] == 2
    assert "torch.distributed.run" in r.stderr  # the launcher's own line


# ------------------------------------------------- the global learner (N > 1) ---
GL_STEPS = 20


def _learner_run(rank, world, E, cap):
    """train_jax.py's loop over one shard (world > 1: ShardedReplay + gather
    before every learner step) or over every env (world == 1: the plain ring)."""
    from dronerl_amd import BatchedDeliveryDrones
    from dronerl_amd.distributed import shard_envs
    from dronerl_amd.dqn import DQNHParams, DQNLearner, QNetwork, ReplayBuffer
    from dronerl_amd.global_learner import ShardedReplay
    sh = shard_envs(E, rank, world)
    env = BatchedDeliveryDrones(_params(), sh.num_envs, device="cuda:0", env_offset=sh.env_offset)
    env.reset(seed=21)
    net = QNetwork(294, (128, 64), device="cuda:0", generator=torch.Generator().manual_seed(3), input="code")
    learner = DQNLearner(net, DQNHParams(batch=8, target_update_interval=3), generator=torch.Generator().manual_seed(4))
    if world > 1:
        sr = ShardedReplay(cap, 294, torch.device("cuda:0"), E, sh.env_offset, sh.num_envs, rank, world, code_radius=3)
        ring = sr.ring
    else:
        sr = ring = ReplayBuffer(cap, 294, torch.device("cuda:0"), code_radius=3)
    cur, nxt = env.new_code(), env.new_code()
    env.get_code(out=cur)
    acts = torch.empty((sh.num_envs, 8), dtype=torch.int32, device="cuda:0")
    for t in range(GL_STEPS):
        net.act(cur, learner.epsilon, seed=9, step=t, env_offset=sh.env_offset, actions=acts, synth=(13, t))
        r, d = env.step(acts, code=nxt)
        sr.add_many(cur, acts, r, nxt, d)
        if world > 1:
            sr.gather(learner)
        learner.train(ring)
        cur, nxt = nxt, cur
    torch.cuda.synchronize()
    learner.check_errors()
    out = {k: learner.sets[k].cpu().numpy().copy() for k in ("online", "target", "m", "v")}
    out["counters"] = learner.counters()
    out["packed"] = net.packed.cpu().numpy().copy()
    return out


def _gl_worker(rank, world, port, E, cap, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out[rank] = _learner_run(rank, world, E, cap)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("E,cap", [(512, 3000), (512, 300)])  # the ring wraps; one add overfills it (E > cap)
def test_global_learner_two_ranks_equal_one_learner(E, cap):
    """two ranks, each with half the envs, its own image of
    the global ring and the row exchange before every learner step, end with
    parameters, target, Adam moments, counters and packed image all equal, bit
    for bit, to one learner over every env's transitions in one ring
    (train_jax.py:59-82, :196-212; buffers.py:57-90), over 20 steps."""
    ref = _learner_run(0, 1, E, cap)
    assert ref["counters"]["count"] == GL_STEPS
    ctx = mp.get_context("spawn")
    with ctx.Manager() as man:
        out = man.dict()
        port = _free_port()
        procs = [ctx.Process(target=_gl_worker, args=(r, 2, port, E, cap, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
            assert p.exitcode == 0, p.exitcode
        res = dict(out)
    for r in range(2):
        for k in ("online", "target", "m", "v", "packed"):
            assert np.array_equal(res[r][k].view(np.uint32), ref[k].view(np.uint32)), (r, k)
        assert res[r]["counters"] == ref["counters"], r


def _train_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from dronerl_amd import EnvParams
    from dronerl_amd.dqn import DQNHParams
    from dronerl_amd.train import train
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = train(EnvParams(n_drones=4, grid_size=9), 256, 30, hp=DQNHParams(num_steps=30), reset_env_every=10,
                    memory_size=1000, device="cuda:0", rank=rank, world=world)
        out[rank] = {k: res.learner.sets[k].cpu().numpy().copy() for k in ("online", "target", "m", "v")}
    finally:
        dist.destroy_process_group()


def test_train_use_sharding_equals_one_process():
    """dronerl_amd.train.train with world = 2 (train_jax.py --use_sharding:
    the envs sharded, the one replay ring sharded, the same learner on every
    rank) == world = 1 over the same 256 envs, bit for bit, through resets."""
    from dronerl_amd import EnvParams
    from dronerl_amd.dqn import DQNHParams
    from dronerl_amd.train import train
    ref = train(EnvParams(n_drones=4, grid_size=9), 256, 30, hp=DQNHParams(num_steps=30), reset_env_every=10,
                memory_size=1000, device="cuda:0")
    want = {k: ref.learner.sets[k].cpu().numpy() for k in ("online", "target", "m", "v")}
    ctx = mp.get_context("spawn")
    with ctx.Manager() as man:
        out = man.dict()
        port = _free_port()
        procs = [ctx.Process(target=_train_worker, args=(r, 2, port, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
            assert p.exitcode == 0, p.exitcode
        res = dict(out)
    for r in range(2):
        for k, v in want.items():
            assert np.array_equal(res[r][k].view(np.uint32), v.view(np.uint32)), (r, k)
