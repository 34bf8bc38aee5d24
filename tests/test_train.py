"""The device-trained agent end to end (train_jax.py:238-256):
dronerl_amd.train.train (the scan body on the device: act, step + replay
add, learner, reset_env_every) -> DQNLearner.save in the reference's three
on-disk forms -> load_qnetwork / read_checkpoint (bit-identical weights) ->
the greedy eval_jax (train.evaluate) of the reloaded net against the random
drones.  The run is deterministic (every kernel is bit-reproducible), so the
learned agent's margin over the random drone is a fixed number, asserted
with room to spare."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_trained_agent_saves_reloads_and_beats_random(tmp_path):
    from dronerl_amd import EnvParams
    from dronerl_amd.checkpoint import load_qnetwork, read_checkpoint, to_qnet
    from dronerl_amd.train import evaluate, train
    p = EnvParams(n_drones=4, grid_size=9)  # train_jax.py's defaults (:338-340)
    res = train(p, 4096, 300)
    c = res.learner.counters()
    assert c["step"] == 300 and c["count"] == 300
    online = [(w.cpu(), b.cpu()) for w, b in res.learner.params("online")]
    for fmt in ("torch", "jax", "torch_agent"):
        path = str(tmp_path / f"agent_{fmt}.safetensors")
        res.learner.save(path, format=fmt)
        ck = read_checkpoint(path)
        assert ck.dense_layers == (128, 64) and tuple(ck.obs_shape) == (7, 7, 6)
        assert ck.metadata.get("checkpoint_format", "torch") == ("torch" if fmt == "torch_agent" else fmt)
        net = load_qnetwork(path)
        lin = [m for m in net.network.children() if isinstance(m, torch.nn.Linear)]
        for (w, b), m in zip(online, lin):
            assert torch.equal(w, m.weight.detach()) and torch.equal(b, m.bias.detach()), fmt
    # the reloaded net on the act kernel == the live net's Q (same parameters, same kernel)
    qnet = to_qnet(read_checkpoint(str(tmp_path / "agent_torch.safetensors")), device="cuda")
    obs = res.env.get_obs(1).reshape(res.env.num_envs, -1)
    q_live = torch.empty((res.env.num_envs, 5), device="cuda")
    q_back = torch.empty_like(q_live)
    from dronerl_amd.dqn import QNetwork
    live = QNetwork(294, (128, 64), precision="f32")
    live.load(*zip(*res.learner.params("online")))
    live.act(obs, 0.0, q_out=q_live)
    qnet.act(obs, 0.0, q_out=q_back)
    assert torch.equal(q_live, q_back)
    agent, rnd, table = evaluate(p, qnet, num_evals=5, num_eval_steps=2000, device="cuda")
    print(f"eval after 300 steps: agent {agent[0]:.4f} +- {agent[1]:.4f}, random {rnd[0]:.4f} +- {rnd[1]:.4f}")
    assert table.shape == (5, 2)
    assert agent[0] > rnd[0] + 0.05, (agent, rnd)  # measured: -0.093 against -0.192


def test_train_main_cli_end_to_end(tmp_path):
    """`python -m dronerl_amd.train` (train_jax.py's options): train, save the
    jax and torch checkpoints under output_dir/jax_run_*, run the final eval."""
    from dronerl_amd.checkpoint import read_checkpoint
    from dronerl_amd.train import main
    m = main(["--num_envs", "512", "--num_steps", "60", "--hidden_layers", "64", "32", "--save_final_checkpoint",
              "--num_evals", "3", "--num_eval_steps", "200", "--output_dir", str(tmp_path)])
    assert m["obs_per_sec"] > 0 and m["num_gpus"] == 1
    for fmt in ("jax", "torch"):
        ck = read_checkpoint(m[f"checkpoint_{fmt}"])
        assert ck.dense_layers == (64, 32) and m[f"checkpoint_{fmt}"].endswith(f"agent_60_steps_{fmt}.safetensors")
    assert -1.0 <= m["eval_reward_mean"] <= 1.0 and -1.0 <= m["random_reward_mean"] <= 1.0
