"""On-device DQN consumer of the observation.

Reference: jax_impl/agents/dqn.py DenseQNetwork (:47-63) and DQNAgent.act
(:132-146), train_jax.py:42-64 (drone 0 of every env follows the agent; the
transition of drone 0 goes to the replay buffer), jax_impl/buffers.py:18-93.

`QNetwork` holds fp32 parameters (torch nn.Linear layout [out][in]; a flax
Dense kernel is the transpose) and packs them for the MFMA kernel
(drl_qnet_pack) whenever they change; `act` runs the forward + epsilon-greedy
choice for every env in one launch (drl_qnet_act; f32 numerics by default,
bf16 operands as an opt-in).  `ReplayBuffer.add_many` is drl_replay_add; `sample` is plain
torch indexing (64 rows).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import torch

from ._native import DRL_ERR_QNET_RANGE, DroneRLError, DrlParams, DrlState, lib

NUM_ACTIONS = 5  # common/constants.py Action


DRL_QNET_BF16, DRL_QNET_F32 = 0, 1  # include/dronerl.h
PRECISIONS = {"bf16": DRL_QNET_BF16, "f32": DRL_QNET_F32}
DRL_QNET_INPUT_OBS, DRL_QNET_INPUT_CODE = 0, 1
INPUTS = {"obs": DRL_QNET_INPUT_OBS, "code": DRL_QNET_INPUT_CODE}


class DrlQnetDesc(ctypes.Structure):
    _fields_ = [("in_features", ctypes.c_int32), ("n_hidden", ctypes.c_int32),
                ("hidden", ctypes.c_int32 * 3), ("n_actions", ctypes.c_int32), ("precision", ctypes.c_int32),
                ("input", ctypes.c_int32)]


class DrlReplay(ctypes.Structure):
    _fields_ = [("capacity", ctypes.c_int64), ("obs_floats", ctypes.c_int32), ("obs", ctypes.c_void_p),
                ("next_obs", ctypes.c_void_p), ("actions", ctypes.c_void_p), ("rewards", ctypes.c_void_p),
                ("dones", ctypes.c_void_p)]


class DrlReplayBatch(ctypes.Structure):
    _fields_ = [("cursor", ctypes.c_int64), ("n", ctypes.c_int64), ("obs", ctypes.c_void_p),
                ("obs_stride", ctypes.c_int64), ("next_obs", ctypes.c_void_p), ("next_obs_stride", ctypes.c_int64),
                ("actions", ctypes.c_void_p), ("action_stride", ctypes.c_int64), ("rewards", ctypes.c_void_p),
                ("reward_stride", ctypes.c_int64), ("dones", ctypes.c_void_p), ("done_stride", ctypes.c_int64)]


class DrlDqnHParams(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("target_update_interval", ctypes.c_int32),
                ("epsilon_decay_every", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("gamma", ctypes.c_double), ("learning_rate", ctypes.c_double), ("beta1", ctypes.c_double),
                ("beta2", ctypes.c_double), ("adam_eps", ctypes.c_double), ("tau", ctypes.c_double),
                ("epsilon_decay", ctypes.c_double), ("epsilon_end", ctypes.c_double), ("sample_seed", ctypes.c_uint64)]


class DrlDqnLayout(ctypes.Structure):
    _fields_ = [("n_params", ctypes.c_int64), ("weight_off", ctypes.c_int64 * 4), ("bias_off", ctypes.c_int64 * 4),
                ("online_off", ctypes.c_int64), ("target_off", ctypes.c_int64), ("m_off", ctypes.c_int64),
                ("v_off", ctypes.c_int64), ("counters_off", ctypes.c_int64), ("scratch_off", ctypes.c_int64),
                ("bytes", ctypes.c_int64), ("grad_workgroups", ctypes.c_int32), ("grad_lds_bytes", ctypes.c_int32)]


_vp = ctypes.c_void_p


def _bind(L):
    if getattr(L, "_qnet_ready", False):
        return L
    i32, i64, u64, f32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
    D = ctypes.POINTER(DrlQnetDesc)
    sig = {
        "drl_qnet_packed_bytes": [D, ctypes.POINTER(i64)],
        "drl_qnet_pack": [D, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp, _vp],
        "drl_qnet_act": [D, _vp, _vp, i64, i64, f32, u64, u64, i64, _vp, i64, _vp, _vp, _vp],
        "drl_qnet_act_synth": [D, _vp, _vp, i64, i64, f32, u64, u64, i64, _vp, i32, u64, u64, _vp, _vp, _vp],
        "drl_qnet_act_code": [D, _vp, _vp, i64, f32, u64, u64, i64, _vp, i64, i32, u64, u64, _vp, _vp, _vp],
        "drl_replay_add": [ctypes.POINTER(DrlReplay), i64, i64, _vp, i64, _vp, i64, _vp, i64, _vp, i64, _vp, i64, _vp],
        "drl_qnet_act_eps": [D, _vp, _vp, i64, i64, _vp, u64, u64, i64, _vp, i64, i32, u64, u64, _vp, _vp, _vp],
        "drl_step_code_replay": [ctypes.POINTER(DrlParams), ctypes.POINTER(DrlState), _vp, _vp, _vp, _vp, _vp,
                                 ctypes.POINTER(DrlReplay), i64, _vp, ctypes.c_uint32, _vp],
        "drl_step_code_replay_synth": [ctypes.POINTER(DrlParams), ctypes.POINTER(DrlState), _vp, _vp, _vp, _vp, _vp,
                                       ctypes.POINTER(DrlReplay), i64, u64, u64, i64, _vp, ctypes.c_uint32, _vp],
        "drl_dqn_layout_query": [D, i32, ctypes.POINTER(DrlDqnLayout)],
        "drl_dqn_init": [D, i32, _vp, f32, _vp],
        "drl_dqn_train": [D, ctypes.POINTER(DrlDqnHParams), _vp, _vp, ctypes.POINTER(DrlReplay), i64, _vp],
        "drl_dqn_train_fresh": [D, ctypes.POINTER(DrlDqnHParams), _vp, _vp, ctypes.POINTER(DrlReplay), i64,
                                ctypes.POINTER(DrlReplayBatch), _vp],
        "drl_dqn_sample_rows": [D, ctypes.POINTER(DrlDqnHParams), _vp, i64, _vp, _vp],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = ctypes.c_int
    L._qnet_ready = True
    return L


def _check(L, rc):
    if rc:
        raise DroneRLError(L.drl_last_error().decode())


def _on(t, device, dtype, name):
    """The kernels read and write raw device pointers: no conversion, no copies."""
    if not isinstance(t, torch.Tensor) or t.device != torch.device(device) or t.dtype != dtype:
        raise ValueError(f"{name} must be a {dtype} tensor on {device}")


def _stream(device):
    return _vp(torch.cuda.current_stream(device).cuda_stream)


class QNetwork:
    """Dense Q-network: in_features -> hidden... (ReLU) -> n_actions.

    precision "f32" (the default): the reference's f32 nets (jax
    dqn.py:47-63, torch dqn.py:44-82): split fp16 hi/lo operands, three MFMAs
    per product tile, Q to f32 rounding (include/dronerl.h DRL_QNET_F32).
    "bf16" (opt-in, narrower than the reference): bf16 MFMA operands, f32
    accumulation (Q to ~1e-2 relative; near-ties may pick another action).

    input "obs": `act` reads the f32 observation rows.  "code" (f32 only, a
    5x5, 7x7 or 9x9 window): `act` reads drone 0's policy code, which
    ``BatchedDeliveryDrones.step(..., code=...)`` writes next to the
    observation (128 B per env at radius 3 instead of 1,176 B of f32); the
    parameters and Q values are the same (drl_qnet_act_code)."""

    def __init__(self, in_features: int, hidden: Sequence[int] = (32, 32), n_actions: int = NUM_ACTIONS,
                 device=None, generator: Optional[torch.Generator] = None, precision: str = "f32",
                 input: str = "obs"):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        if input not in INPUTS:
            raise ValueError(f"input must be one of {sorted(INPUTS)}")
        self.precision = precision
        self.input = input
        self.code_bytes = 0
        if input == "code":
            w = round((in_features / 6) ** 0.5)
            if precision != "f32" or w not in (5, 7, 9) or w * w * 6 != in_features:
                raise ValueError("input='code' needs precision='f32' and in_features = W*W*6 with W in 5, 7, 9")
            self.code_bytes = int(lib().drl_policy_code_bytes((w - 1) // 2))
        self.L = _bind(lib())
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.in_features, self.hidden, self.n_actions = in_features, tuple(hidden), n_actions
        sizes = [in_features, *self.hidden, n_actions]
        self.weights, self.biases = [], []
        for i in range(len(sizes) - 1):
            # he_normal for the hidden layers (dqn.py:53), flax Dense's lecun_normal for the output
            w = flax_kernel_init((sizes[i + 1], sizes[i]), 2.0 if i < len(sizes) - 2 else 1.0, generator)
            self.weights.append(w.to(self.device))
            self.biases.append(torch.zeros(sizes[i + 1], device=self.device))
        self.desc = DrlQnetDesc(in_features, len(self.hidden), (ctypes.c_int32 * 3)(*self.hidden, *[0] * (3 - len(self.hidden))),
                                n_actions, PRECISIONS[precision], INPUTS[input])
        nb = ctypes.c_int64()
        _check(self.L, self.L.drl_qnet_packed_bytes(ctypes.byref(self.desc), ctypes.byref(nb)))
        self.packed = torch.empty(nb.value // 4, dtype=torch.int32, device=self.device)  # 16-B aligned
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)  # DRL_ERR_QNET_RANGE (f32 operand range)
        self.pack()

    def load(self, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor]):
        """Set parameters (torch layout [out][in]) and re-pack.  Nothing
        changes if they are refused."""
        if len(weights) != len(self.weights) or len(biases) != len(self.biases):
            raise ValueError("layer count mismatch")
        for i, (w, b) in enumerate(zip(weights, biases)):
            if tuple(w.shape) != tuple(self.weights[i].shape) or tuple(b.shape) != tuple(self.biases[i].shape):
                raise ValueError(f"layer {i}: shape {tuple(w.shape)} != {tuple(self.weights[i].shape)}")
        ws = [w.detach().to(self.device, torch.float32) for w in weights]
        bs = [b.detach().to(self.device, torch.float32) for b in biases]
        self._validate(ws, bs)
        for i, (w, b) in enumerate(zip(ws, bs)):
            # (in place: a DQNLearner's net holds views of its agent block)
            self.weights[i].copy_(w)
            self.biases[i].copy_(b)
        self.pack()

    def _validate(self, weights, biases):
        for t in (*weights, *biases):
            if not bool(torch.isfinite(t).all()):
                raise ValueError("weights and biases must be finite")
        if self.precision == "f32":  # fp16 hi/lo split range (include/dronerl.h DRL_QNET_F32)
            # the weights are split into fp16 pieces, and so is a code net's
            # layer-0 bias (packed as a weight); every other bias stays f32
            split = list(weights) + ([biases[0]] if self.input == "code" else [])
            for t in split:
                if float(t.abs().max()) >= 65504.0:
                    raise ValueError("f32 precision needs |w| < 65504 (and |b| < 65504 for a code net's layer 0)")

    def pack(self):
        self._validate(self.weights, self.biases)
        n = len(self.weights)
        wp = (_vp * n)(*[w.data_ptr() for w in self.weights])
        bp = (_vp * n)(*[b.data_ptr() for b in self.biases])
        _check(self.L, self.L.drl_qnet_pack(ctypes.byref(self.desc), wp, bp, _vp(self.packed.data_ptr()),
                                            _stream(self.device)))

    def reference_q(self, obs: torch.Tensor, bf16_operands: bool = False) -> torch.Tensor:
        """Plain torch forward (checker for tests); bf16_operands rounds the
        weights, inputs and hidden activations to bf16 as the MFMA path does."""
        r = (lambda t: t.to(torch.bfloat16).to(torch.float32)) if bf16_operands else (lambda t: t)
        x = r(obs.reshape(obs.shape[0], -1).to(torch.float32))
        for i, (w, b) in enumerate(zip(self.weights, self.biases)):
            x = x @ r(w).t() + b
            if i < len(self.weights) - 1:
                x = r(torch.relu(x))
        return x

    def act(self, obs: torch.Tensor, epsilon, seed: int = 0, step: int = 0, env_offset: int = 0,
            actions: Optional[torch.Tensor] = None, q_out: Optional[torch.Tensor] = None,
            synth: Optional[Tuple[int, int]] = None) -> torch.Tensor:
        """Epsilon-greedy action for each row of obs [E, ..., in_features]
        (input "code": the policy code, uint8 [E, code_bytes]).
        `actions` may be an [E, n_drones] int32 tensor: column 0 is written (the
        other drones keep their actions, train_jax.py:47-49).  synth=(seed,
        step): the other columns get BatchedDeliveryDrones.synth_actions(seed,
        step)'s values in the same launch (drl_qnet_act_synth).  epsilon: a
        float, or a float32 device tensor of one element read by the kernel
        (DQNLearner.epsilon: the learner's decaying schedule; drl_qnet_act_eps)."""
        E = obs.shape[0]
        if self.input == "code":
            _on(obs, self.device, torch.uint8, "code")
            if tuple(obs.shape) != (E, self.code_bytes) or not obs.is_contiguous():
                raise ValueError(f"code must be a contiguous uint8 [E, {self.code_bytes}] tensor")
        else:
            _on(obs, self.device, torch.float32, "obs")
        flat = obs.reshape(E, -1)
        if self.input == "obs" and (flat.shape[1] < self.in_features or flat.stride(1) != 1):
            raise ValueError("obs must hold at least in_features contiguous float32 values per env")
        if actions is None:
            actions = torch.empty((E, 1), dtype=torch.int32, device=self.device)
        _on(actions, self.device, torch.int32, "actions")
        if actions.shape[0] != E or actions.dim() > 2 or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous int32 [E] or [E, n] tensor")
        if q_out is not None:
            _on(q_out, self.device, torch.float32, "q_out")
            if tuple(q_out.shape) != (E, self.n_actions) or not q_out.is_contiguous():
                raise ValueError(f"q_out must be a contiguous float32 [{E}, {self.n_actions}] tensor")
        stride_a = actions.shape[1] if actions.dim() == 2 else 1
        if isinstance(epsilon, torch.Tensor):
            _on(epsilon, self.device, torch.float32, "epsilon")
            if epsilon.numel() != 1:
                raise ValueError("a device epsilon must be one float32 element")
            sn, ss, st = (stride_a, synth[0] & (2**64 - 1), synth[1]) if synth is not None else (0, 0, 0)
            x = obs if self.input == "code" else flat
            _check(self.L, self.L.drl_qnet_act_eps(
                ctypes.byref(self.desc), _vp(self.packed.data_ptr()), _vp(x.data_ptr()), E,
                0 if self.input == "code" else flat.stride(0), _vp(epsilon.data_ptr()), seed & (2**64 - 1), step,
                env_offset, _vp(actions.data_ptr()), stride_a, sn, ss, st,
                None if q_out is None else _vp(q_out.data_ptr()), _vp(self.err.data_ptr()), _stream(self.device)))
            return actions
        if self.input == "code":
            sn, ss, st = (stride_a, synth[0] & (2**64 - 1), synth[1]) if synth is not None else (0, 0, 0)
            _check(self.L, self.L.drl_qnet_act_code(
                ctypes.byref(self.desc), _vp(self.packed.data_ptr()), _vp(obs.data_ptr()), E, float(epsilon),
                seed & (2**64 - 1), step, env_offset, _vp(actions.data_ptr()), stride_a, sn, ss, st,
                None if q_out is None else _vp(q_out.data_ptr()), _vp(self.err.data_ptr()), _stream(self.device)))
            return actions
        if synth is not None:
            _check(self.L, self.L.drl_qnet_act_synth(
                ctypes.byref(self.desc), _vp(self.packed.data_ptr()), _vp(flat.data_ptr()), E, flat.stride(0),
                float(epsilon), seed & (2**64 - 1), step, env_offset, _vp(actions.data_ptr()), stride_a,
                synth[0] & (2**64 - 1), synth[1], None if q_out is None else _vp(q_out.data_ptr()),
                _vp(self.err.data_ptr()), _stream(self.device)))
            return actions
        _check(self.L, self.L.drl_qnet_act(ctypes.byref(self.desc), _vp(self.packed.data_ptr()), _vp(flat.data_ptr()),
                                           E, flat.stride(0), float(epsilon), seed & (2**64 - 1), step, env_offset,
                                           _vp(actions.data_ptr()), stride_a,
                                           None if q_out is None else _vp(q_out.data_ptr()), _vp(self.err.data_ptr()),
                                           _stream(self.device)))
        return actions

    def check_errors(self):
        """Synchronise and raise if an f32 act met an operand outside fp16's
        split range (|input or hidden activation| >= 65520, or NaN): its Q
        values and greedy actions are then not valid (DRL_ERR_QNET_RANGE)."""
        e = int(self.err.item())
        if e:
            self.err.zero_()
            if e & DRL_ERR_QNET_RANGE:
                raise DroneRLError("f32 act: an input or hidden activation is outside the fp16 split range "
                                   "(|v| >= 65520 or NaN); Q values are not valid")
            raise DroneRLError(f"qnet error bits {e:#x}")


def decode_policy_code(code: torch.Tensor, window_radius: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Policy-code rows uint8 [n, code_bytes] -> drone 0's observation f32
    [n, W*W*6], bit for bit what drl_obs writes (drl_code_decode)."""
    L = lib()
    W = 2 * window_radius + 1
    n = code.shape[0]
    _on(code, code.device, torch.uint8, "code")
    if code.dim() != 2 or code.shape[1] != L.drl_policy_code_bytes(window_radius) or not code.is_contiguous():
        raise ValueError("code must be a contiguous uint8 [n, policy_code_bytes] tensor")
    if out is None:
        out = torch.empty((n, W * W * 6), dtype=torch.float32, device=code.device)
    _on(out, code.device, torch.float32, "out")
    if out.numel() != n * W * W * 6 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous float32 tensor of {n * W * W * 6} values")
    _check(L, L.drl_code_decode(window_radius, _vp(code.data_ptr()), n, _vp(out.data_ptr()), _stream(code.device)))
    return out


@dataclass
class ReplayBuffer:
    """jax_impl/buffers.py ReplayBuffer on device tensors (drone-0 transitions).

    code_radius > 0: the rows hold drone 0's policy code (uint8 [capacity,
    code_bytes], 128 B at radius 3 instead of 1,176 B of f32) -- add_many
    takes code rows (BatchedDeliveryDrones.step(..., code=...)) -- and sample
    decodes the drawn rows to the f32 observation (decode_policy_code), so the
    learner sees exactly the observations the reference buffer would hold."""
    capacity: int
    obs_floats: int
    device: torch.device
    code_radius: int = 0

    def __post_init__(self):
        self.L = _bind(lib())
        d = torch.device(self.device)
        if self.code_radius:
            W = 2 * self.code_radius + 1
            if self.obs_floats != W * W * 6:
                raise ValueError(f"obs_floats must be {W * W * 6} for a code_radius {self.code_radius} buffer")
            self.code_bytes = int(self.L.drl_policy_code_bytes(self.code_radius))
            if self.code_bytes <= 0:
                raise ValueError("bad code_radius")
            self.obs = torch.zeros((self.capacity, self.code_bytes), dtype=torch.uint8, device=d)
            self.next_obs = torch.zeros((self.capacity, self.code_bytes), dtype=torch.uint8, device=d)
            row_words = self.code_bytes // 4
        else:
            self.obs = torch.zeros((self.capacity, self.obs_floats), device=d)
            self.next_obs = torch.zeros((self.capacity, self.obs_floats), device=d)
            row_words = self.obs_floats
        self.actions = torch.zeros(self.capacity, dtype=torch.int32, device=d)
        self.rewards = torch.zeros(self.capacity, device=d)
        self.dones = torch.zeros(self.capacity, dtype=torch.uint8, device=d)
        self.cursor = 0          # current_idx
        self.size = 0            # current_size
        self._c = DrlReplay(self.capacity, row_words, self.obs.data_ptr(), self.next_obs.data_ptr(),
                            self.actions.data_ptr(), self.rewards.data_ptr(), self.dones.data_ptr())

    def add_many(self, obs: torch.Tensor, actions: torch.Tensor, rewards: torch.Tensor, next_obs: torch.Tensor,
                 dones: torch.Tensor):
        """buffers.py:57-80.  obs/next_obs [E, >= obs_floats] f32 rows (a code
        buffer: uint8 [E, code_bytes] policy-code rows); actions i32, rewards
        f32, dones u8 as [E] or [E, n_drones] (column 0 taken).  Returns the
        batch's description (DQNLearner.train(fresh=...): a learner step that
        may run while this add is still in flight)."""
        E = obs.shape[0]
        dev = self.obs.device
        odt = torch.uint8 if self.code_radius else torch.float32
        for t, dt, name in ((obs, odt, "obs"), (next_obs, odt, "next_obs"),
                            (actions, torch.int32, "actions"), (rewards, torch.float32, "rewards"),
                            (dones, torch.uint8, "dones")):
            _on(t, dev, dt, name)
            if t.shape[0] != E or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous [{E}, ...] tensor")
            if name in ("actions", "rewards", "dones") and t.dim() > 2:
                raise ValueError(f"{name} must be [E] or [E, n_drones]")
        o, no = obs.reshape(E, -1), next_obs.reshape(E, -1)
        if self.code_radius:
            if o.shape[1] != self.code_bytes or no.shape[1] != self.code_bytes:
                raise ValueError(f"code rows must hold code_bytes={self.code_bytes} bytes")
            o, no = o.view(torch.float32), no.view(torch.float32)  # copied bit for bit
        elif o.shape[1] < self.obs_floats or no.shape[1] < self.obs_floats:
            raise ValueError(f"obs rows must hold at least obs_floats={self.obs_floats} values")
        col = lambda t: t.shape[1] if t.dim() == 2 else 1  # noqa: E731
        _check(self.L, self.L.drl_replay_add(ctypes.byref(self._c), self.cursor, E, _vp(o.data_ptr()), o.stride(0),
                                             _vp(no.data_ptr()), no.stride(0), _vp(actions.data_ptr()), col(actions),
                                             _vp(rewards.data_ptr()), col(rewards), _vp(dones.data_ptr()), col(dones),
                                             _stream(self.obs.device)))
        batch = DrlReplayBatch(self.cursor, E, o.data_ptr(), o.stride(0), no.data_ptr(), no.stride(0),
                               actions.data_ptr(), col(actions), rewards.data_ptr(), col(rewards), dones.data_ptr(),
                               col(dones))
        self.cursor = (self.cursor + E) % self.capacity
        self.size = min(self.size + E, self.capacity)
        return batch

    def _add_from_step(self, env, actions: torch.Tensor, rewards: torch.Tensor, dones: torch.Tensor,
                       code_prev: torch.Tensor, code: torch.Tensor, flags: int, synth=None):
        """BatchedDeliveryDrones.step(..., code=code, replay=self, replay_obs=code_prev): the step and the
        add_many(code_prev, actions, rewards, code, dones) of its drone-0 transitions in one launch
        (drl_step_code_replay; train_jax.py:55-62's env.step + buffer.add_many pair).  The ring ends up
        bit-identical to step + add_many.  synth=(seed, step): drone indices >= 1 act as
        env.synth_actions(seed, step) would write them, drawn in the step (drl_step_code_replay_synth;
        only actions[:, 0] is read).  Returns the batch's description (as add_many)."""
        E, N = env.num_envs, env.n_drones
        if not self.code_radius or self.code_radius != env.params.window_radius:
            raise ValueError("replay= needs a code buffer of the env's window radius (ReplayBuffer(code_radius=...))")
        _on(code_prev, self.obs.device, torch.uint8, "replay_obs")
        if tuple(code_prev.shape) != (E, self.code_bytes) or not code_prev.is_contiguous():
            raise ValueError(f"replay_obs must be a contiguous [{E}, {self.code_bytes}] uint8 tensor")
        if code_prev.data_ptr() == code.data_ptr():
            raise ValueError("replay_obs must be another buffer than code (the rows the act read)")
        s = env.state.c()
        if synth is None:
            _check(self.L, self.L.drl_step_code_replay(
                ctypes.byref(env._cp), ctypes.byref(s), _vp(actions.data_ptr()), _vp(rewards.data_ptr()),
                _vp(dones.data_ptr()), _vp(code.data_ptr()), _vp(code_prev.data_ptr()), ctypes.byref(self._c),
                self.cursor, _vp(env.err.data_ptr()), flags, _stream(self.obs.device)))
        else:
            seed, step = synth
            _check(self.L, self.L.drl_step_code_replay_synth(
                ctypes.byref(env._cp), ctypes.byref(s), _vp(actions.data_ptr()), _vp(rewards.data_ptr()),
                _vp(dones.data_ptr()), _vp(code.data_ptr()), _vp(code_prev.data_ptr()), ctypes.byref(self._c),
                self.cursor, int(seed), int(step), int(env.env_offset), _vp(env.err.data_ptr()), flags,
                _stream(self.obs.device)))
        w = self.code_bytes // 4
        batch = DrlReplayBatch(self.cursor, E, code_prev.data_ptr(), w, code.data_ptr(), w, actions.data_ptr(), N,
                               rewards.data_ptr(), N, dones.data_ptr(), N)
        self.cursor = (self.cursor + E) % self.capacity
        self.size = min(self.size + E, self.capacity)
        self.last_batch = batch
        return batch

    def can_sample(self, batch: int = 64) -> bool:
        return self.size >= batch

    def sample(self, batch: int = 64, generator: Optional[torch.Generator] = None) -> dict:
        """buffers.py:82-93: uniform indices in [0, size)."""
        idx = torch.randint(0, self.size, (batch,), device=self.obs.device, generator=generator)
        obs, next_obs = self.obs[idx], self.next_obs[idx]
        if self.code_radius:
            obs = decode_policy_code(obs, self.code_radius)
            next_obs = decode_policy_code(next_obs, self.code_radius)
        return dict(obs=obs, actions=self.actions[idx], rewards=self.rewards[idx],
                    next_obs=next_obs, dones=self.dones[idx])


def flax_kernel_init(shape, scale: float, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """flax's variance_scaling(scale, "fan_in", "truncated_normal") for a torch-layout [out][in] weight:
    he_normal (scale 2, the hidden layers, jax dqn.py:54) and Dense's default lecun_normal (scale 1, the output
    layer, :56) -- a normal truncated at +-2 standard deviations, its deviation divided by .87962566103423978
    (the truncated unit normal's) so the variance is scale / fan_in."""
    std = (scale / shape[1]) ** 0.5 / .87962566103423978
    return torch.nn.init.trunc_normal_(torch.empty(shape), 0.0, std, -2.0 * std, 2.0 * std, generator=generator)


@dataclass
class DQNHParams:
    """The learner's hyperparameters: jax_impl/agents/dqn.py DQNAgentParams
    (:20-33) with train_jax.py's defaults (:349-360) and optax.adam's
    (b1 0.9, b2 0.999, eps 1e-8).  `epsilon_decay` None: train_jax.py:133-134's
    value for `num_steps` (half the way to epsilon_end after 20 % of them)."""
    batch: int = 8
    gamma: float = 0.9
    learning_rate: float = 1e-3
    beta1: float = 0.9
    beta2: float = 0.999
    adam_eps: float = 1e-8
    tau: float = 1.0
    target_update_interval: int = 10
    epsilon_start: float = 1.0
    epsilon_decay: Optional[float] = None
    epsilon_end: float = 0.01
    epsilon_decay_every: int = 5
    num_steps: int = 1000
    sample_seed: int = 0

    def decay(self) -> float:
        if self.epsilon_decay is not None:
            return self.epsilon_decay
        return (1 - 0.5 * (1 - self.epsilon_end / self.epsilon_start)) ** (1 / (0.2 * self.num_steps))

    def c(self) -> DrlDqnHParams:
        return DrlDqnHParams(self.batch, self.target_update_interval, self.epsilon_decay_every, 0, self.gamma,
                             self.learning_rate, self.beta1, self.beta2, self.adam_eps, self.tau, self.decay(),
                             self.epsilon_end, self.sample_seed & (2**64 - 1))


class DQNLearner:
    """jax_impl/agents/dqn.py DQNAgent's training state on the device: the
    online net (`net`, whose weights become views of the agent block), a target
    net, Adam's moments and the counters (step, Adam count, epsilon) -- one
    agent block (include/dronerl.h drl_dqn_layout).  `train(rb)` is the
    learner block of one train_jax.py scan step (:68-98): sample + train_step
    when the buffer can sample, the target update every
    target_update_interval steps, the epsilon decay every epsilon_decay_every
    steps, step + 1 -- all on the device (drl_dqn_train), the packed net the
    act reads refreshed in the same call.  `epsilon` is a device scalar to
    pass to QNetwork.act.

    target: the target net's initial (weights, biases) (torch layout); the
    reference initialises it from its own key (dqn.py:119-121), so by default
    it is a fresh init from `generator` with the reference's initialisers
    (flax_kernel_init; zero biases)."""

    def __init__(self, net: QNetwork, hp: Optional[DQNHParams] = None, target=None,
                 generator: Optional[torch.Generator] = None):
        self.net, self.hp = net, hp or DQNHParams()
        self.L = net.L
        lay = DrlDqnLayout()
        _check(self.L, self.L.drl_dqn_layout_query(ctypes.byref(net.desc), self.hp.batch, ctypes.byref(lay)))
        self.layout = lay
        dev = net.device
        self.block = torch.zeros(lay.bytes, dtype=torch.uint8, device=dev)
        n = lay.n_params

        def fset(off):
            return self.block[off:off + 4 * n].view(torch.float32)

        self.sets = {k: fset(getattr(lay, k + "_off")) for k in ("online", "target", "m", "v")}
        ctr = self.block[lay.counters_off:lay.counters_off + 64]
        self._ctr_f = ctr.view(torch.float32)
        self._ctr_i = ctr.view(torch.int32)
        self.epsilon = self._ctr_f[2:3]  # drl_dqn_counters.epsilon
        shapes = [(w.shape, b.shape) for w, b in zip(net.weights, net.biases)]
        if target is None:
            g = generator if generator is not None else torch.Generator().manual_seed(1)
            tw = [flax_kernel_init(ws, 2.0 if l < len(shapes) - 1 else 1.0, g) for l, (ws, _) in enumerate(shapes)]
            target = (tw, [torch.zeros(bs) for _, bs in shapes])
        for l, (ws, bs) in enumerate(shapes):
            self.params("online")[l][0].copy_(net.weights[l])
            self.params("online")[l][1].copy_(net.biases[l])
            self.params("target")[l][0].copy_(target[0][l].to(dev, torch.float32))
            self.params("target")[l][1].copy_(target[1][l].to(dev, torch.float32))
        online = self.params("online")
        net.weights = [w for w, _ in online]  # the net now reads the live parameters
        net.biases = [b for _, b in online]
        net.pack()
        _check(self.L, self.L.drl_dqn_init(ctypes.byref(net.desc), self.hp.batch, _vp(self.block.data_ptr()),
                                           float(self.hp.epsilon_start), _stream(dev)))
        self._hp = self.hp.c()

    def params(self, which: str):
        """[(W [out][in], b [out])] views of one parameter set ("online",
        "target", "m", "v")."""
        s, lay = self.sets[which], self.layout
        out = []
        for l, (w, b) in enumerate(zip(self.net.weights, self.net.biases)):
            wo, bo = lay.weight_off[l], lay.bias_off[l]
            out.append((s[wo:wo + w.numel()].view(w.shape), s[bo:bo + b.numel()]))
        return out

    def train(self, rb: "ReplayBuffer", fresh: Optional[DrlReplayBatch] = None):
        """One learner block (train_jax.py:68-98) on the replay's current
        contents (rb.size transitions).  fresh: the value of the
        rb.add_many call that filled the latest rows; their transitions are
        then read from that call's buffers, so the add may still be running
        on another stream (drl_dqn_train_fresh)."""
        if rb.obs.device != self.block.device:
            raise ValueError("the replay buffer must be on the learner's device")
        if fresh is not None:
            _check(self.L, self.L.drl_dqn_train_fresh(ctypes.byref(self.net.desc), ctypes.byref(self._hp),
                                                      _vp(self.block.data_ptr()), _vp(self.net.packed.data_ptr()),
                                                      ctypes.byref(rb._c), rb.size, ctypes.byref(fresh),
                                                      _stream(self.block.device)))
            return
        _check(self.L, self.L.drl_dqn_train(ctypes.byref(self.net.desc), ctypes.byref(self._hp),
                                            _vp(self.block.data_ptr()), _vp(self.net.packed.data_ptr()),
                                            ctypes.byref(rb._c), rb.size, _stream(self.block.device)))

    def sample_slots(self, size: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The replay slots (int64 [batch], in [0, size)) the next train()
        draws (drl_dqn_sample_rows: its counter hash at the step the device
        counters will hold; stream-ordered, no sync)."""
        if out is None:
            out = torch.empty(self.hp.batch, dtype=torch.int64, device=self.block.device)
        _on(out, self.block.device, torch.int64, "out")
        if out.numel() != self.hp.batch or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous int64 [{self.hp.batch}] tensor")
        _check(self.L, self.L.drl_dqn_sample_rows(ctypes.byref(self.net.desc), ctypes.byref(self._hp),
                                                  _vp(self.block.data_ptr()), int(size), _vp(out.data_ptr()),
                                                  _stream(self.block.device)))
        return out

    def check_errors(self):
        """Synchronise; raise if a learner launch gave up waiting for one of
        its hand-offs (a hardware-scheduling fault, never expected).  From
        that launch on every drl_dqn_train returns without touching the
        block (the learner is frozen, not silently corrupted) until
        restart()."""
        if int(self._ctr_i[13].item()):
            raise DroneRLError("drl_dqn_train: a workgroup timed out waiting for another workgroup's hand-off; "
                               "the learner refuses to train until restart()")

    def save(self, path: str, format: str = "torch", **kw):
        """The online net as train_jax.py:238-244 saves the trained agent
        (dronerl_amd.checkpoint.save_dense): format "torch" (jax dqn.py
        save_as_torch), "jax" (dqn.py save) or "torch_agent" (torch_impl
        DQNAgent.save).  Synchronises (a host copy of the parameters)."""
        from .checkpoint import save_dense
        W = round((self.net.in_features / 6) ** 0.5)
        if W * W * 6 != self.net.in_features:
            raise ValueError("the net's input is not a W x W x 6 window")
        ws, bs = zip(*self.params("online"))
        save_dense(path, ws, bs, (W, W, 6), format=format, **kw)

    def restart(self, epsilon: Optional[float] = None):
        """drl_dqn_init on the current parameters: Adam's moments and the
        counters from zero (step 0, epsilon `epsilon` or hp.epsilon_start),
        the scratch zeroed, a timeout flag cleared.  The online and target
        parameters are kept."""
        eps = self.hp.epsilon_start if epsilon is None else float(epsilon)
        _check(self.L, self.L.drl_dqn_init(ctypes.byref(self.net.desc), self.hp.batch, _vp(self.block.data_ptr()),
                                           eps, _stream(self.block.device)))

    def counters(self) -> dict:
        """Host copy of the device counters (synchronises)."""
        f, i = self._ctr_f.cpu(), self._ctr_i.cpu()
        d = self.block[self.layout.counters_off + 16:self.layout.counters_off + 32].view(torch.float64).cpu()
        return {"step": int(i[0]), "count": int(i[1]), "epsilon": float(f[2]), "loss": float(f[3]),
                "beta1_pow": float(d[0]), "beta2_pow": float(d[1])}
