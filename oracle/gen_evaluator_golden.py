"""ORACLE TOOLING ONLY — evaluator end-to-end fixture.

Runs in the build container only: it imports the reference
(/root/reference/torch_impl, with the stand-ins in oracle/gymshim for gym and
matplotlib) and replays DroneRacerEvaluator._evaluate (drone_evaluator.py:97-204)
for the five submissions of tests/torch_tests/test_drone_evaluator.py:5-11:
6 drones (the 5 baseline nets + the submission as "YOU"), seeds
845, 99, 65, 96, 85, 39, 51, 17, 52, 35, 1000 steps each, every agent acting
greedily on its own 7x7 window (q_values.argmax()).  Rendering and the video
(:171-180, PIL/ffmpeg) are left out: they draw no random numbers.

Writes tests/golden/evaluator_scores.npz:
  scores[s, e, a]   reward sum of agent a (sorted names: YOU, baseline-1..5) in
                    episode e for submission s (float64, the reference's sums)
  actions0[s, t, a] actions of the first 200 steps of episode 0 (debug aid)
The sample nets themselves are copied as data to tests/golden/sample_models/.

Usage:  DEVICE=cpu python oracle/gen_evaluator_golden.py     (~1-2 minutes)
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "gymshim"))
sys.path.insert(0, REF)
os.environ.setdefault("DEVICE", "cpu")

import torch  # noqa: E402
from torch_impl.agents.dqn import BaseDQNFactory  # noqa: E402
from torch_impl.env.env import DeliveryDrones  # noqa: E402
from torch_impl.env.wrappers import WindowedGridView  # noqa: E402

SEEDS = [845, 99, 65, 96, 85, 39, 51, 17, 52, 35]      # drone_evaluator.py:28
STEPS = 1000                                            # drone_evaluator.py:29
BASELINES = {f"baseline-{i}": f"sample_models/dqn-agent-{i}.safetensors" for i in range(1, 6)}
ENV_PARAMS = {  # drone_evaluator.py:112-126
    'charge_reward': -0.1, 'crash_reward': -1, 'delivery_reward': 1, 'charge': 20, 'discharge': 10,
    'drone_density': 0.05, 'dropzones_factor': 2, 'n_drones': 3, 'packets_factor': 3, 'pickup_reward': 0,
    'rgb_render_rescale': 1.0, 'skyscrapers_factor': 3, 'stations_factor': 2}


def set_seed(env, seed):
    # torch_impl/helpers/rl_helpers.py:12-18 (that module imports matplotlib/pandas
    # plotting at import time; its five statements are replayed here verbatim)
    env.reset(seed=seed)
    env.action_space.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    random.seed(seed)


def load(path):
    return BaseDQNFactory.from_checkpoint(os.path.join(REF, path)).create_qnetwork()[0]


def evaluate(submission):
    agents = {name: load(p) for name, p in BASELINES.items()}
    agents["YOU"] = load(submission)
    names = sorted(agents)
    scores = np.zeros((len(SEEDS), len(names)))
    actions0 = np.zeros((200, len(names)), np.int8)
    for e, seed in enumerate(SEEDS):
        params = dict(ENV_PARAMS)
        params["n_drones"] = len(names)
        env = WindowedGridView(DeliveryDrones(params), radius=3)
        set_seed(env, seed)
        state = env.reset()
        for t in range(STEPS):
            acts = {}
            for i, name in enumerate(names):
                with torch.no_grad():
                    q = agents[name]([state[i]])[0]
                acts[i] = q.argmax().item()
            if e == 0 and t < 200:
                actions0[t] = [acts[i] for i in range(len(names))]
            state, rewards, _, _, _ = env.step(acts)
            scores[e] += np.array(list(rewards.values()))
    return scores, actions0


def main():
    subs = [f"sample_models/dqn-agent-{i}.safetensors" for i in range(1, 6)]
    all_scores, all_actions = [], []
    for s in subs:
        sc, a0 = evaluate(s)
        you = sc[:, 0]
        print(f"{s}: score {you.mean():.4f} secondary {you.std():.4f}", flush=True)
        all_scores.append(sc)
        all_actions.append(a0)
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "evaluator_scores.npz"),
                        scores=np.array(all_scores), actions0=np.array(all_actions), seeds=np.array(SEEDS),
                        steps=np.array(STEPS))


if __name__ == "__main__":
    main()
