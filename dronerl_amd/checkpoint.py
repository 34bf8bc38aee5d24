"""Safetensors Q-network checkpoints.

Reference formats:
* torch (torch_impl/agents/dqn.py:162-277, 330-345): metadata network_type
  "dense" | "conv", obs_shape, action_shape, dense_layers (hidden widths of a
  dense net, or the dense layers after the convolutions of a conv net),
  conv_layers; tensors network.dense_{i}.weight [out][in] / .bias and
  network.conv2d_{i}.weight [out][in][kh][kw] / .bias (i from 1).
* jax (jax_impl/agents/dqn.py:228-357): checkpoint_format "jax", tensors
  params.Dense_{i}.kernel [in][out] / params.Conv_{i}.kernel [kh][kw][in][out]
  (i from 0); conv nets list their dense layers under conv_dense_layers.

Files are read with safetensors' numpy loader (no pickle) and metadata with
ast.literal_eval, as the reference does.  `TorchQNetwork` rebuilds the
reference module (same nn.Sequential names, so state dicts load unchanged)
and its forward: dense nets flatten [B, H, W, C] row-major; conv nets permute
to [B, C, H, W] first (dqn.py:80-81, 153-159).  `to_qnet` moves a dense net
onto the MFMA consumer (dronerl_amd.dqn.QNetwork) when its widths allow;
`save_dense` writes a (device-trained) dense net in the reference's three
on-disk forms (jax save / save_as_torch, torch DQNAgent.save).
"""
from __future__ import annotations

import ast
from dataclasses import dataclass, field
from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn as nn


@dataclass
class Checkpoint:
    network_type: str                       # "dense" | "conv"
    obs_shape: Tuple[int, ...]              # (H, W, C)
    action_shape: Tuple[int, ...]
    dense_layers: Tuple[int, ...]           # hidden dense widths (after the convs for a conv net)
    conv_layers: Tuple[dict, ...] = ()
    tensors: Dict[str, np.ndarray] = field(default_factory=dict)  # torch names and layouts
    metadata: Dict[str, str] = field(default_factory=dict)


def _lit(md, key, default):
    return tuple(ast.literal_eval(md[key])) if key in md else default


def _from_jax_names(params: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """jax_impl/agents/dqn.py:325-350 (save_as_torch) renaming and transposes."""
    out = {}
    for k, v in params.items():
        parts = k.split(".")
        if parts[0] == "params":
            parts[0] = "network"
        name, idx = parts[1].split("_")
        if name == "Dense":
            parts[1] = f"dense_{int(idx) + 1}"
        elif name == "Conv":
            parts[1] = f"conv2d_{int(idx) + 1}"
        else:
            raise ValueError(f"unexpected key {k}")
        if parts[-1] == "kernel":
            v = v.T if name == "Dense" else np.transpose(v, (3, 2, 0, 1))
            parts[-1] = "weight"
        out[".".join(parts)] = np.ascontiguousarray(v)
    return out


def read_checkpoint(path: str) -> Checkpoint:
    from safetensors import safe_open
    with safe_open(path, framework="numpy") as f:
        md = dict(f.metadata() or {})
        tensors = {k: f.get_tensor(k) for k in f.keys()}
    kind = md.get("network_type", "dense")
    if kind not in ("dense", "conv"):
        raise ValueError(f"unknown network type {kind!r}")
    if md.get("checkpoint_format", "torch") == "jax":
        tensors = _from_jax_names(tensors)
        dense = _lit(md, "dense_layers" if kind == "dense" else "conv_dense_layers", ())
    else:
        dense = _lit(md, "dense_layers", ())
    return Checkpoint(kind, _lit(md, "obs_shape", (7, 7, 6)), _lit(md, "action_shape", (5,)), dense,
                      _lit(md, "conv_layers", ()) if kind == "conv" else (), tensors, md)


class TorchQNetwork(nn.Module):
    """torch_impl DenseQNetwork / ConvQNetwork (dqn.py:44-159), rebuilt from a
    Checkpoint: same module names, same forward."""

    def __init__(self, ck: Checkpoint):
        super().__init__()
        self.kind, self.obs_shape = ck.network_type, tuple(ck.obs_shape)
        self.input_size = int(np.prod(self.obs_shape))
        self.network = nn.Sequential()
        outs = tuple(ck.dense_layers) + tuple(ck.action_shape)
        if self.kind == "dense":
            for i, width in enumerate(outs):
                if i > 0:
                    self.network.add_module(f"dense_act_{i}", nn.ReLU())
                self.network.add_module(f"dense_{i + 1}", nn.Linear(self.input_size if i == 0 else outs[i - 1], width))
        else:
            H, W, C = self.obs_shape
            for i, kw in enumerate(ck.conv_layers):
                cin = C if i == 0 else ck.conv_layers[i - 1]["out_channels"]
                self.network.add_module(f"conv2d_{i + 1}", nn.Conv2d(cin, **kw))
                self.network.add_module(f"conv2d_act_{i + 1}", nn.ReLU())
            self.network.add_module("flatten", nn.Flatten())
            with torch.no_grad():
                flat = self.network(torch.ones([1, C, H, W])).shape[1]
            for i, width in enumerate(outs):
                if i > 0:
                    self.network.add_module(f"dense_act_{i}", nn.ReLU())
                self.network.add_module(f"dense_{i + 1}", nn.Linear(flat if i == 0 else outs[i - 1], width))
        self.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in ck.tensors.items()})

    def forward(self, states):
        x = torch.as_tensor(np.array(states) if not torch.is_tensor(states) else states, dtype=torch.float32)
        x = x.to(next(self.parameters()).device)
        if self.kind == "dense":
            return self.network(x.reshape(-1, self.input_size))
        return self.network(x.reshape(-1, *self.obs_shape).permute(0, 3, 1, 2))


def load_qnetwork(path: str) -> TorchQNetwork:
    """BaseDQNFactory.from_checkpoint(path).create_qnetwork()[0] (dqn.py:171-184)."""
    return TorchQNetwork(read_checkpoint(path)).eval()


def _conv_meta(m: nn.Conv2d) -> dict:
    """A Conv2d as the reference's conv_layers entry (dqn.py:336-341); square
    kernels/strides/paddings are written as ints, as the factories take them."""
    one = lambda v: v[0] if isinstance(v, tuple) and len(set(v)) == 1 else v  # noqa: E731
    return {"out_channels": m.out_channels, "kernel_size": one(m.kernel_size), "stride": one(m.stride),
            "padding": one(m.padding)}


def save_checkpoint(path: str, net: TorchQNetwork, conv_layers=None, dense_layers=None):
    """torch-format checkpoint (dqn.py:330-345 metadata keys).  Layer metadata
    not given is read off the network's own Linear / Conv2d modules."""
    from safetensors.numpy import save_file
    sd = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    lin = [m for m in net.network.children() if isinstance(m, nn.Linear)]
    if not lin:
        raise ValueError("network has no Linear layer")
    if dense_layers is None:
        dense_layers = tuple(m.out_features for m in lin[:-1])
    md = {"network_type": net.kind, "obs_shape": str(tuple(net.obs_shape)),
          "action_shape": str((lin[-1].out_features,)), "dense_layers": str(tuple(dense_layers))}
    if net.kind == "conv":
        if conv_layers is None:
            conv_layers = tuple(_conv_meta(m) for m in net.network.children() if isinstance(m, nn.Conv2d))
        md["conv_layers"] = str(tuple(conv_layers))
    save_file(sd, path, metadata=md)


# train_jax.py:366 --conv_layers default (its JSON key order), which save / save_as_torch write for dense nets too
TRAIN_JAX_CONV_LAYERS = ({"kernel_size": 3, "out_channels": 8, "padding": 1, "stride": 1},)
CHECKPOINT_FORMATS = ("torch", "jax", "torch_agent")


def save_dense(path: str, weights, biases, obs_shape, format: str = "torch", conv_layers=TRAIN_JAX_CONV_LAYERS,
               conv_dense_layers=(), checkpoint_format_version: float = 0.1):
    """Write a dense Q-network (weights [out][in] / biases, torch layout, any
    tensors or arrays) as the reference writes a trained agent:

    * "torch": jax_impl/agents/dqn.py:301-357 save_as_torch (what train_jax.py:
      242-244 writes as agent_<n>_steps_torch.safetensors): network.dense_{i}
      .weight [out][in] / .bias (i from 1) and the metadata network_type,
      dense_layers, conv_dense_layers, conv_layers, obs_shape, action_shape,
      checkpoint_format "torch", checkpoint_format_version;
    * "jax": dqn.py:282-299 save (agent_<n>_steps_jax.safetensors):
      params.Dense_{i}.kernel [in][out] / .bias (i from 0), the same
      metadata keys with checkpoint_format "jax";
    * "torch_agent": torch_impl/agents/dqn.py:330-345 DQNAgent.save: the torch
      names and only network_type, dense_layers, obs_shape, action_shape.

    Every string is the reference's str() of the same Python value, so
    ast.literal_eval in either loader reads it back."""
    from safetensors.numpy import save_file
    if format not in CHECKPOINT_FORMATS:
        raise ValueError(f"format must be one of {CHECKPOINT_FORMATS}")
    ws = [np.ascontiguousarray(np.asarray(w.detach().cpu() if torch.is_tensor(w) else w, dtype=np.float32))
          for w in weights]
    bs = [np.ascontiguousarray(np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, dtype=np.float32))
          for b in biases]
    if not ws or len(ws) != len(bs) or any(w.ndim != 2 or b.shape != (w.shape[0],) for w, b in zip(ws, bs)):
        raise ValueError("weights [out][in] and biases [out], one pair per layer")
    if ws[0].shape[1] != int(np.prod(obs_shape)) or any(ws[i + 1].shape[1] != ws[i].shape[0] for i in range(len(ws) - 1)):
        raise ValueError("layer widths do not chain from the observation size")
    hidden = tuple(int(w.shape[0]) for w in ws[:-1])
    md = {"network_type": "dense", "dense_layers": str(hidden), "obs_shape": str(tuple(int(v) for v in obs_shape)),
          "action_shape": str((int(ws[-1].shape[0]),))}
    if format == "torch_agent":
        t = {}
        for i, (w, b) in enumerate(zip(ws, bs)):
            t[f"network.dense_{i + 1}.weight"], t[f"network.dense_{i + 1}.bias"] = w, b
    else:
        md.update({"conv_layers": str(tuple(conv_layers)), "conv_dense_layers": str(tuple(conv_dense_layers)),
                   "checkpoint_format": format, "checkpoint_format_version": str(checkpoint_format_version)})
        t = {}
        for i, (w, b) in enumerate(zip(ws, bs)):
            if format == "jax":
                t[f"params.Dense_{i}.kernel"], t[f"params.Dense_{i}.bias"] = np.ascontiguousarray(w.T), b
            else:
                t[f"network.dense_{i + 1}.weight"], t[f"network.dense_{i + 1}.bias"] = w, b
    save_file(t, path, metadata=md)


def to_qnet(ck: Checkpoint, device=None):
    """A dense checkpoint on the MFMA consumer (dronerl_amd.dqn.QNetwork).
    Needs hidden widths that are multiples of 32 in [32, 128] (1-3 layers)."""
    from .dqn import QNetwork
    if ck.network_type != "dense":
        raise ValueError("only dense networks run on the MFMA consumer")
    if not ck.dense_layers or len(ck.dense_layers) > 3 or any(w % 32 or not 32 <= w <= 128 for w in ck.dense_layers):
        raise ValueError(f"hidden widths {ck.dense_layers} unsupported by drl_qnet (multiples of 32 in [32, 128])")
    n = len(ck.dense_layers) + 1
    net = QNetwork(int(np.prod(ck.obs_shape)), ck.dense_layers, int(ck.action_shape[0]), device=device)
    ws = [torch.from_numpy(np.array(ck.tensors[f"network.dense_{i + 1}.weight"])) for i in range(n)]
    bs = [torch.from_numpy(np.array(ck.tensors[f"network.dense_{i + 1}.bias"])) for i in range(n)]
    net.load(ws, bs)
    return net
