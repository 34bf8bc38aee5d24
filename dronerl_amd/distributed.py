"""Multi-GPU env sharding and the eval-statistics all-reduce.

Reference: train_jax.py:196-212 shards the env-state pytree along one 'envs'
mesh axis (NamedSharding(mesh, P('envs', ...))) and requires
num_envs % devices == 0 (train_jax.py:401-402); eval_jax (train_jax.py:270-319)
runs `num_evals` seeded single-env episodes sequentially and reports
mean +- stdev of the per-episode mean reward of drone 0 (agent) and drone 1
(random).

Here: one process per GPU (torchrun), a contiguous block of envs per rank with
env_offset = rank * (num_envs / world) so seeds follow the global env index
and a sharded run is bit-identical to an unsharded one.  The env step has no
data exchange; the only collective is the all-reduce (sum) of the eval table
[num_evals, 2] (float64, <= a few KB: latency-bound, RCCL over xGMI via the
torch.distributed "nccl" backend, or gloo on CPU).
"""
from __future__ import annotations

import os
import statistics
from dataclasses import dataclass
from typing import Callable, Optional

import torch


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    env_offset: int
    num_envs: int


def shard_envs(num_envs: int, rank: int, world: int) -> Shard:
    """Contiguous env block of `rank` (train_jax.py:401-402 divisibility rule)."""
    if num_envs <= 0:
        raise ValueError('Number of envs need to be at least 1')
    if world > 1 and num_envs % world != 0:
        raise ValueError(f'The number of envs (={num_envs}) needs to be divisible by the number of devices '
                         f'(={world})')
    per = num_envs // world
    return Shard(rank, world, rank * per, per)


def shard_episodes(num_evals: int, rank: int, world: int) -> range:
    """Eval episodes of `rank`: contiguous, sizes differ by at most one."""
    lo = num_evals * rank // world
    hi = num_evals * (rank + 1) // world
    return range(lo, hi)


def init_from_env(backend: Optional[str] = None):
    """Initialise torch.distributed from torchrun's environment.

    Returns (rank, world, local_rank).  backend None: "nccl" (RCCL on ROCm)
    when a GPU is present, else "gloo".  MASTER_ADDR defaults to 127.0.0.1.
    """
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def allreduce_sum(t: torch.Tensor) -> torch.Tensor:
    """In-place sum over ranks (no-op without an initialised process group).
    A device tensor under gloo is reduced through a host copy."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if t.device.type != "cpu" and dist.get_backend() == "gloo":
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def max_over_ranks(v: float, device=None) -> float:
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return v
    t = torch.tensor([v], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


EpisodeRunner = Callable[[range], torch.Tensor]
"""episodes -> float64 [len(episodes), 2]: per-episode mean reward of drone 0 and drone 1."""


def evaluate_sharded(runner: EpisodeRunner, num_evals: int, rank: int = 0, world: int = 1,
                     device=None):
    """eval_jax (train_jax.py:270-319) with the episodes sharded over ranks.

    Each rank runs its episodes (as one batch of envs), writes them into its
    rows of a zero [num_evals, 2] table, and the table is all-reduced (sum).
    Returns ((mean, std) agent, (mean, std) random) like eval_jax, plus the table.
    """
    eps = shard_episodes(num_evals, rank, world)
    table = torch.zeros((num_evals, 2), dtype=torch.float64, device=device)
    if len(eps):
        table[eps.start:eps.stop] = runner(eps).to(table.device, torch.float64)
    allreduce_sum(table)
    t = table.cpu().tolist()
    a = [r[0] for r in t]
    b = [r[1] for r in t]
    std = (lambda v: statistics.stdev(v) if len(v) > 1 else 0.0)
    return (statistics.mean(a), std(a)), (statistics.mean(b), std(b)), table


def gpu_episode_runner(params, num_steps: int, eval_seed: int, policy: Optional[Callable] = None,
                       action_seed: int = 0, device=None) -> EpisodeRunner:
    """Episodes on the GPU env: env i seeded random.seed(eval_seed + i); every
    drone acts uniformly at random (synthetic stream) except drone 0, which
    follows `policy(obs[E, W*W*6]) -> int32 [E]` when given (the greedy DQN of
    eval_jax)."""

    def run(eps: range) -> torch.Tensor:
        from .env import BatchedDeliveryDrones
        env = BatchedDeliveryDrones(params, len(eps), device=device, env_offset=eps.start)
        env.reset(seed=eval_seed)
        sums = torch.zeros((len(eps), 2), dtype=torch.float64, device=env.device)
        obs = env.get_obs(1) if policy is not None else None
        for t in range(num_steps):
            a = env.synth_actions(seed=action_seed, step=t)
            if policy is not None:
                a[:, 0] = policy(obs.reshape(len(eps), -1)).to(torch.int32)
                r, _, obs = env.step(a, obs_k=1)
            else:
                r, _ = env.step(a)
            sums[:, 0] += r[:, 0].double()
            if params.n_drones > 1:
                sums[:, 1] += r[:, 1].double()
        env.check_errors()
        return sums / num_steps

    return run
