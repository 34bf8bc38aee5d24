"""The train_jax.py driver over the device env and learner.

`train` is train_jax.py:38-115's scan body run step by step on one GPU (or
one env shard): per step, uniform random actions for every drone, the
epsilon-greedy DQN action for drone 0 (drl_qnet_act_synth, the learner's
device epsilon), the env step writing drone 0's next policy code and landing
the drone-0 transitions in the replay ring (drl_step_code_replay:
buffer.add_many), the learner block (drl_dqn_train: sample + train_step when
the buffer can sample, the target update, the epsilon decay, step + 1), and
a reset of every env when step % reset_env_every == 0 (:99-113).
`evaluate` is eval_jax (:270-319): greedy drone 0 against random drones,
episodes sharded over ranks with the eval table all-reduced
(distributed.evaluate_sharded).  The trained agent leaves the device in the
reference's formats through DQNLearner.save (train_jax.py:238-244).

The random streams are the build's (counter hashes), not
jax.random's, so a run reproduces this build's runs, not the reference's.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from .params import EnvParams


@dataclass
class TrainResult:
    env: object
    net: object
    learner: object
    replay: object
    steps: int
    env_steps_per_s: float


def train(params: EnvParams, num_envs: int, num_steps: int, hidden: Sequence[int] = (128, 64), hp=None,
          reset_env_every: int = 100, memory_size: int = 100_000, seed: int = 0, env_offset: int = 0,
          action_seed: int = 2024, act_seed: int = 7, device=None) -> TrainResult:
    """train_jax.py's training loop (see the module docstring).  hp: a
    dqn.DQNHParams (default: train_jax.py's defaults with num_steps, so
    epsilon decays as :133-134 schedules it)."""
    from .dqn import DQNHParams, DQNLearner, QNetwork, ReplayBuffer
    from .env import BatchedDeliveryDrones
    if num_steps < 1 or reset_env_every < 1:
        raise ValueError("num_steps and reset_env_every must be >= 1")
    env = BatchedDeliveryDrones(params, num_envs, device=device, env_offset=env_offset)
    env.reset(seed=seed)
    dev, E, N = env.device, env.num_envs, env.n_drones
    r = params.window_radius
    D = (2 * r + 1) ** 2 * 6
    net = QNetwork(D, tuple(hidden), device=dev, generator=torch.Generator().manual_seed(seed), input="code")
    learner = DQNLearner(net, hp or DQNHParams(num_steps=num_steps), generator=torch.Generator().manual_seed(seed + 1))
    rb = ReplayBuffer(memory_size, D, dev, code_radius=r)
    code = [env.new_code(), env.new_code()]
    env.get_code(out=code[0])
    acts = torch.empty((E, N), dtype=torch.int32, device=dev)
    rew = torch.empty((E, N), dtype=torch.float32, device=dev)
    don = torch.empty((E, N), dtype=torch.uint8, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for t in range(num_steps):
        b, nb = t & 1, (t + 1) & 1
        net.act(code[b], learner.epsilon, seed=act_seed, step=t, env_offset=env.env_offset, actions=acts,
                synth=(action_seed, t))
        env.step(acts, rewards=rew, dones=don, code=code[nb], replay=rb, replay_obs=code[b])
        learner.train(rb)
        if t % reset_env_every == 0:  # train_jax.py:101-113 (step 0 included)
            env.reset(seed=None)
            env.get_code(out=code[nb])
    e1.record()
    torch.cuda.synchronize(dev)
    env.check_errors()
    net.check_errors()
    learner.check_errors()
    dt = e0.elapsed_time(e1) / 1e3
    return TrainResult(env, net, learner, rb, num_steps, E * num_steps / dt)


def greedy_policy(qnet):
    """drone 0's greedy action (dqn.act(..., greedy=True), train_jax.py:286)
    from a QNetwork on f32 observation rows."""

    def policy(obs: torch.Tensor) -> torch.Tensor:
        return qnet.act(obs, 0.0)[:, 0]

    return policy


def evaluate(params: EnvParams, qnet, num_evals: int = 5, num_eval_steps: int = 10_000, eval_seed: int = 0,
             rank: int = 0, world: int = 1, device=None):
    """eval_jax (train_jax.py:270-319): `num_evals` episodes of
    `num_eval_steps` steps, episode i seeded eval_seed + i, drone 0 greedy,
    every other drone uniform random; episodes sharded over ranks and the
    table all-reduced.  Returns ((mean, std) agent, (mean, std) random, table)."""
    from .distributed import evaluate_sharded, gpu_episode_runner
    run = gpu_episode_runner(params, num_eval_steps, eval_seed, policy=greedy_policy(qnet), action_seed=eval_seed,
                             device=device)
    return evaluate_sharded(run, num_evals, rank, world, device=device)
