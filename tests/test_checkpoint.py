"""Safetensors checkpoint interop on the reference's own
sample models (tests/golden/sample_models/, copied data files of
/root/reference/sample_models used by tests/torch_tests/test_drone_evaluator.py).

The rebuilt module is checked against an independent numpy forward of the
reference architectures (dqn.py:44-159): dense = Linear / ReLU chain over the
row-major flattened [7,7,6] window; conv = Conv2d(+ReLU) on [C,H,W], flatten
(C,H,W order), then the dense chain.
"""
import glob
import os

import numpy as np
import pytest
import torch

from dronerl_amd.checkpoint import TorchQNetwork, load_qnetwork, read_checkpoint, save_checkpoint

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MODELS = sorted(glob.glob(os.path.join(GOLD, "sample_models", "*.safetensors")))
PUBLISHED = {1: (-64.98, 6.109), 2: (-81.31, 12.312), 3: (-65.08, 7.777), 4: (-71.88, 13.564), 5: (-68.43, 10.194)}


def np_forward(ck, x):
    """x [B, 7, 7, 6] float32 -> Q [B, 5], float64 accumulation."""
    t = ck.tensors
    x = x.astype(np.float64)
    if ck.network_type == "conv":
        h = np.transpose(x, (0, 3, 1, 2))                      # [B, C, H, W]
        for i, kw in enumerate(ck.conv_layers):
            w, b = t[f"network.conv2d_{i + 1}.weight"].astype(np.float64), t[f"network.conv2d_{i + 1}.bias"]
            p, k = kw.get("padding", 0), kw["kernel_size"]
            hp = np.pad(h, ((0, 0), (0, 0), (p, p), (p, p)))
            H, W = hp.shape[2] - k + 1, hp.shape[3] - k + 1
            out = np.zeros((h.shape[0], w.shape[0], H, W))
            for dy in range(k):
                for dx in range(k):
                    out += np.einsum("bchw,oc->bohw", hp[:, :, dy:dy + H, dx:dx + W], w[:, :, dy, dx])
            h = np.maximum(out + b[None, :, None, None], 0)
        h = h.reshape(h.shape[0], -1)
    else:
        h = x.reshape(x.shape[0], -1)
    n = len(ck.dense_layers) + 1
    for i in range(n):
        h = h @ t[f"network.dense_{i + 1}.weight"].astype(np.float64).T + t[f"network.dense_{i + 1}.bias"]
        if i < n - 1:
            h = np.maximum(h, 0)
    return h


def test_sample_models_present():
    assert len(MODELS) == 5


@pytest.mark.parametrize("path", MODELS)
def test_rebuilt_network_matches_numpy_forward(path):
    ck = read_checkpoint(path)
    net = TorchQNetwork(ck)
    names = [n for n, _ in net.network.named_children()]
    assert names[-1].startswith("dense_") and all(k in net.state_dict() for k in ck.tensors)
    x = np.random.default_rng(0).random((64, 7, 7, 6)).astype(np.float32)
    with torch.no_grad():
        q = net(x).numpy()
    np.testing.assert_allclose(q, np_forward(ck, x), rtol=1e-5, atol=1e-5)
    with torch.no_grad():  # the evaluator's call shape: agent([window])[0]
        q1 = net([x[3]])[0].numpy()
    np.testing.assert_allclose(q1, q[3], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("path", MODELS)
def test_save_load_roundtrip(path, tmp_path):
    ck = read_checkpoint(path)
    net = TorchQNetwork(ck)
    out = str(tmp_path / "rt.safetensors")
    save_checkpoint(out, net, conv_layers=ck.conv_layers, dense_layers=ck.dense_layers)
    ck2 = read_checkpoint(out)
    assert (ck2.network_type, ck2.dense_layers, ck2.conv_layers) == (ck.network_type, ck.dense_layers, ck.conv_layers)
    for k in ck.tensors:
        np.testing.assert_array_equal(ck2.tensors[k], ck.tensors[k])


@pytest.mark.parametrize("path", MODELS)
def test_save_load_roundtrip_metadata_from_modules(path, tmp_path):
    """save_checkpoint(path, net) with no layer metadata: widths, action shape
    and conv layers are read off the network's modules (dqn.py:330-345)."""
    ck = read_checkpoint(path)
    net = TorchQNetwork(ck)
    out = str(tmp_path / "rt.safetensors")
    save_checkpoint(out, net)
    ck2 = read_checkpoint(out)
    assert (ck2.network_type, ck2.dense_layers, ck2.action_shape) == (ck.network_type, ck.dense_layers,
                                                                       ck.action_shape)
    if ck.network_type == "conv":
        norm = lambda cl: tuple({k: d.get(k, 0) for k in ("out_channels", "kernel_size", "stride", "padding")}
                                for d in cl)  # noqa: E731
        assert norm(ck2.conv_layers) == norm(ck.conv_layers)
    net2 = TorchQNetwork(ck2)
    x = np.random.default_rng(1).random((8, 7, 7, 6)).astype(np.float32)
    with torch.no_grad():
        np.testing.assert_array_equal(net2(x).numpy(), net(x).numpy())


def test_save_checkpoint_many_dense_layers(tmp_path):
    """action_shape comes from the last Linear, not the text-sorted weight
    names (dense_10 sorts before dense_2)."""
    ck = read_checkpoint(MODELS[0])
    widths = (8,) * 10
    ck = type(ck)("dense", (7, 7, 6), (5,), widths)
    rng = np.random.default_rng(0)
    sizes = [294, *widths, 5]
    for i in range(len(sizes) - 1):
        ck.tensors[f"network.dense_{i + 1}.weight"] = rng.standard_normal((sizes[i + 1], sizes[i])).astype(np.float32)
        ck.tensors[f"network.dense_{i + 1}.bias"] = np.zeros(sizes[i + 1], np.float32)
    net = TorchQNetwork(ck)
    out = str(tmp_path / "deep.safetensors")
    save_checkpoint(out, net)
    ck2 = read_checkpoint(out)
    assert ck2.action_shape == (5,) and ck2.dense_layers == widths


@pytest.mark.parametrize("path", MODELS)
def test_jax_format_converts_to_torch_layout(path, tmp_path):
    """jax_impl/agents/dqn.py:228-260 naming and kernel layouts."""
    from safetensors.numpy import save_file
    ck = read_checkpoint(path)
    jp = {}
    for k, v in ck.tensors.items():
        _, layer, what = k.split(".")
        name, idx = layer.split("_")
        jl = ("Dense" if name == "dense" else "Conv") + "_" + str(int(idx) - 1)
        if what == "weight":
            v = v.T if name == "dense" else np.transpose(v, (2, 3, 1, 0))
            what = "kernel"
        jp[f"params.{jl}.{what}"] = np.ascontiguousarray(v)
    md = {"network_type": ck.network_type, "obs_shape": "(7, 7, 6)", "action_shape": "(5,)",
          "checkpoint_format": "jax"}
    if ck.network_type == "dense":
        md["dense_layers"] = str(ck.dense_layers)
    else:
        md.update(conv_layers=str(ck.conv_layers), conv_dense_layers=str(ck.dense_layers), dense_layers="(32, 32)")
    p = str(tmp_path / "jax.safetensors")
    save_file(jp, p, metadata=md)
    ck2 = read_checkpoint(p)
    assert ck2.dense_layers == ck.dense_layers
    for k in ck.tensors:
        np.testing.assert_array_equal(ck2.tensors[k], ck.tensors[k])


def test_evaluator_fixture_reproduces_published_scores():
    """tests/golden/evaluator_scores.npz (oracle/gen_evaluator_golden.py, the
    reference evaluator replayed) against test_drone_evaluator.py:5-11."""
    d = np.load(os.path.join(GOLD, "evaluator_scores.npz"))
    s = d["scores"]                     # [submission, episode, agent]; agent 0 = "YOU"
    assert s.shape == (5, 10, 6)
    for i in range(5):
        mean, std = PUBLISHED[i + 1]
        assert np.isclose(s[i, :, 0].mean(), mean, rtol=1e-2) and np.isclose(s[i, :, 0].std(), std, rtol=1e-2)


# ----------------------------------------------------------- saving an agent ---
AGENT = os.path.join(GOLD, "agent_save")


def _meta(path):
    from safetensors import safe_open
    with safe_open(path, framework="numpy") as f:
        return dict(f.metadata() or {}), {k: f.get_tensor(k) for k in f.keys()}


def _fixture_net():
    ck = read_checkpoint(os.path.join(AGENT, "torch_agent.safetensors"))
    n = len(ck.dense_layers) + 1
    return ([ck.tensors[f"network.dense_{i + 1}.weight"] for i in range(n)],
            [ck.tensors[f"network.dense_{i + 1}.bias"] for i in range(n)], ck)


def test_save_torch_agent_matches_reference_save(tmp_path):
    """save_dense(format="torch_agent") of the fixture's weights == the
    reference's own torch DQNAgent.save (torch_impl/agents/dqn.py:330-345;
    oracle/gen_agent_golden.py): the same metadata strings, tensor names,
    shapes and bytes."""
    from dronerl_amd.checkpoint import save_dense
    ws, bs, _ = _fixture_net()
    p = str(tmp_path / "a.safetensors")
    save_dense(p, ws, bs, (7, 7, 6), format="torch_agent")
    md_ref, t_ref = _meta(os.path.join(AGENT, "torch_agent.safetensors"))
    md, t = _meta(p)
    assert md == md_ref
    assert sorted(t) == sorted(t_ref)
    for k in t:
        assert t[k].dtype == t_ref[k].dtype and np.array_equal(t[k], t_ref[k]), k


@pytest.mark.parametrize("fmt", ["torch", "jax", "torch_agent"])
def test_save_formats_read_back(tmp_path, fmt):
    """Each form reads back (read_checkpoint / load_qnetwork, the jax form's
    renames and transposes undone) to the reference net's Q values; the
    "torch" form was also read by the reference's own loader when the fixture
    was made (q_loader == q_ref); the metadata carries jax dqn.py:282-357's
    keys (save / save_as_torch) with train_jax.py's conv_layers default."""
    from dronerl_amd.checkpoint import TRAIN_JAX_CONV_LAYERS, save_dense
    ws, bs, _ = _fixture_net()
    gold = np.load(os.path.join(AGENT, "agent_q.npz"))
    assert np.array_equal(gold["q_loader"], gold["q_ref"]) and np.array_equal(gold["q_loader_agent"], gold["q_ref"])
    p = str(tmp_path / f"{fmt}.safetensors")
    save_dense(p, ws, bs, (7, 7, 6), format=fmt)
    md, t = _meta(p)
    base = {"network_type": "dense", "dense_layers": "(32, 32)", "obs_shape": "(7, 7, 6)", "action_shape": "(5,)"}
    if fmt == "torch_agent":
        assert md == base
    else:
        assert md == dict(base, conv_layers=str(TRAIN_JAX_CONV_LAYERS), conv_dense_layers="()",
                          checkpoint_format=fmt, checkpoint_format_version="0.1")
    if fmt == "jax":
        assert sorted(t) == sorted(f"params.Dense_{i}.{k}" for i in range(3) for k in ("kernel", "bias"))
        assert t["params.Dense_0.kernel"].shape == (294, 32)
    ck = read_checkpoint(p)
    for i in range(3):
        assert np.array_equal(ck.tensors[f"network.dense_{i + 1}.weight"], ws[i])
        assert np.array_equal(ck.tensors[f"network.dense_{i + 1}.bias"], bs[i])
    net = load_qnetwork(p)
    with torch.no_grad():
        q = net(torch.from_numpy(gold["inputs"].reshape(16, 7, 7, 6))).numpy()
    np.testing.assert_array_equal(q, gold["q_ref"])


def test_save_dense_argument_checks(tmp_path):
    from dronerl_amd.checkpoint import save_dense
    ws, bs, _ = _fixture_net()
    p = str(tmp_path / "x.safetensors")
    with pytest.raises(ValueError):
        save_dense(p, ws, bs, (7, 7, 6), format="onnx")
    with pytest.raises(ValueError):
        save_dense(p, ws, bs[:-1], (7, 7, 6))
    with pytest.raises(ValueError):
        save_dense(p, ws, bs, (5, 5, 6))
