"""Train the device agent (dronerl_amd.train), save it in the reference's
torch format, reload it with load_qnetwork, and evaluate it greedily
(eval_jax) against the random drones.  One JSON line per run.

  python tools/train_eval.py --grid 9 --drones 4 --envs 4096 --steps 300 1000 3000
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dronerl_amd import EnvParams  # noqa: E402
from dronerl_amd.checkpoint import load_qnetwork, read_checkpoint, to_qnet  # noqa: E402
from dronerl_amd.dqn import DQNHParams  # noqa: E402
from dronerl_amd.train import evaluate, train  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=9)
    ap.add_argument("--drones", type=int, default=4)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, nargs="+", default=[300])
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hidden", type=int, nargs="+", default=[128, 64])
    ap.add_argument("--evals", type=int, default=5)
    ap.add_argument("--eval-steps", type=int, default=2000)
    ap.add_argument("--lr", type=float, default=1e-3)
    args = ap.parse_args()
    p = EnvParams(n_drones=args.drones, grid_size=args.grid)
    for steps in args.steps:
        t0 = time.time()
        hp = DQNHParams(batch=args.batch, num_steps=steps, learning_rate=args.lr)
        res = train(p, args.envs, steps, hidden=args.hidden, hp=hp)
        c = res.learner.counters()
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "agent.safetensors")
            res.learner.save(path, format="torch")
            ref = load_qnetwork(path)
            same = all(torch.equal(w.cpu(), m.weight.detach()) and torch.equal(b.cpu(), m.bias.detach())
                       for (w, b), m in zip(res.learner.params("online"),
                                            [m for m in ref.network.children() if isinstance(m, torch.nn.Linear)]))
            qnet = to_qnet(read_checkpoint(path), device="cuda")
        agent, rnd, _ = evaluate(p, qnet, num_evals=args.evals, num_eval_steps=args.eval_steps)
        print(json.dumps({"grid": args.grid, "drones": args.drones, "envs": args.envs, "steps": steps,
                          "batch": args.batch, "env_steps_per_s": res.env_steps_per_s, "adam_steps": c["count"],
                          "epsilon": c["epsilon"], "loss": c["loss"], "reload_bit_identical": same,
                          "eval_agent": agent, "eval_random": rnd, "wall_s": time.time() - t0}), flush=True)


if __name__ == "__main__":
    main()
