"""Batched DroneRL environment on MI355X (the hot path).

API shape follows jax_impl's vmapped env (jax_impl/env/env.py: reset :89-135,
step :137-250, get_obs :274-309; callers train_jax.py:52-56,186-193) with a
leading env axis on PyTorch-ROCm tensors; semantics are torch_impl's
(env.py:68-233, wrappers.py:10-73), bit-exact, each env carrying its own
CPython-compatible MT19937 stream seeded like ``random.seed(seed + env)``.

PyTorch is plumbing here (device memory and the current stream); every
computation runs in libdronerl.so's HIP kernels.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import torch

from ._native import (DRL_ERR_BAD_ACTION, DRL_ERR_BAD_STATE, DRL_ERR_NO_FREE_CELL, DRL_MT_WORDS, DRL_STEP_OBS_STREAM,
                      DRL_STEP_REFILL, DroneRLError, DrlState, check, lib)
from .params import EnvParams


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def unpack_ground(packed: torch.Tensor, side: int) -> torch.Tensor:
    """Packed ground rows [E, ground_stride] -> object codes uint8 [E, side, side]."""
    E = packed.shape[0]
    cells = torch.stack((packed & 15, packed >> 4), dim=-1).reshape(E, -1)
    return cells[:, :side * side].reshape(E, side, side)


def pack_ground(ground: torch.Tensor, stride: int) -> torch.Tensor:
    """Object codes [E, cells] (uint8, < 16) -> packed rows [E, stride] (zero padding)."""
    E = ground.shape[0]
    g = ground.reshape(E, -1)
    if g.numel() and int(g.max()) > 15:
        raise ValueError("ground codes must be < 16")
    full = torch.zeros((E, 2 * stride), dtype=torch.uint8, device=g.device)
    full[:, :g.shape[1]] = g
    return full[:, 0::2] | (full[:, 1::2] << 4)


@dataclass
class DroneEnvState:
    """Device state of E envs (structure of arrays, env-major; include/dronerl.h).

    ground : uint8 [E, ground_stride]  object codes, row-major, two cells per byte (cell k in the
                                       low nibble of byte k // 2 when k is even, the high one when
                                       odd; include/dronerl.h ABI 8): decode() / set_state() convert
    drones : int32 [E, n_drones]       packed u32 records in dict order O
    mt     : int32 [E, 1776]           two MT19937 blocks + the respawn-candidate ring
    mt_index: int32 [E]                CPython's MT index (bits 0-9), the block holding the
                                       stream (bit 10), ring head / count (bits 11-19 / 20-29)
    (the stream's CPython getstate() words: BatchedDeliveryDrones.mt_words())
    """
    ground: torch.Tensor
    drones: torch.Tensor
    mt: torch.Tensor
    mt_index: torch.Tensor

    @property
    def num_envs(self) -> int:
        return self.ground.shape[0]

    def c(self) -> DrlState:
        return DrlState(self.ground.data_ptr(), self.drones.data_ptr(), self.mt.data_ptr(), self.mt_index.data_ptr(),
                        self.num_envs)

    def clone(self) -> "DroneEnvState":
        return DroneEnvState(self.ground.clone(), self.drones.clone(), self.mt.clone(), self.mt_index.clone())

    def narrow(self, start: int, length: int) -> "DroneEnvState":
        """A view of envs [start, start+length) (used for sharding and subsets)."""
        return DroneEnvState(self.ground.narrow(0, start, length), self.drones.narrow(0, start, length),
                             self.mt.narrow(0, start, length), self.mt_index.narrow(0, start, length))


class BatchedDeliveryDrones:
    """E independent torch_impl DeliveryDrones envs stepped by HIP kernels.

    Global env index g = env_offset + e; env g's stream is seeded as
    ``random.seed(seed + g)`` by ``reset(seed)``, so a sharded run is
    bit-identical to the unsharded one.
    """

    def __init__(self, params: EnvParams, num_envs: int, device=None, env_offset: int = 0):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise DroneRLError("BatchedDeliveryDrones runs on the GPU only (no CPU fallback)")
        if self.device.index is None:  # "cuda" -> the current device (tensors made on it report their index)
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.params = params
        self.layout = params.layout()  # validates (ValueError like the reference)
        self._cp = params.to_c()
        self.num_envs = int(num_envs)
        self.env_offset = int(env_offset)
        self.n_drones = params.n_drones
        self.side = params.side
        L = self.layout
        E = self.num_envs
        dev = self.device
        self.state = DroneEnvState(
            ground=torch.zeros((E, L.ground_stride), dtype=torch.uint8, device=dev),
            drones=torch.zeros((E, L.drone_stride), dtype=torch.int32, device=dev),
            mt=torch.zeros((E, DRL_MT_WORDS), dtype=torch.int32, device=dev),
            mt_index=torch.full((E,), 624, dtype=torch.int32, device=dev),
        )
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        # steps between drl_refill top-ups of the respawn-candidate rings (0: never;
        # the steps then draw every respawn from the MT stream themselves)
        self.refill_every = int(L.refill_every)
        # step()'s default observation store mode: cached stores at P <= 8
        # (C3: the act kernel that reads the observation next runs 64-66 us per
        # loop step against 71 after streaming stores), streaming stores at
        # P >= 16 (C4: 90 vs 93-94 us per loop step, 34.3 vs 36.6 per bare
        # step; profiles/r02_store_mode/)
        self.default_obs_stream = int(L.step_group_lanes) >= 16
        self._since_refill = 0

    # ------------------------------------------------------------ core API --
    def reset(self, seed: Optional[int] = 0, env_mask: Optional[torch.Tensor] = None) -> DroneEnvState:
        """env.py:68-101 for every env (or where env_mask != 0).

        seed is not None: re-seed env g as random.seed(seed + g) first
        (set_seed, rl_helpers.py:18).  seed None: continue each env's stream.
        """
        if env_mask is not None:
            env_mask = self._check(env_mask, torch.uint8, (self.num_envs,), "env_mask")
        reseed = seed is not None
        seed_base = 0
        if reseed:
            # Env g is seeded random.seed(seed + g) with a one-word (u64) key;
            # outside [0, 2**64) CPython's key differs (abs(), longer keys).
            seed_base = int(seed) + self.env_offset
            if seed_base < 0 or seed_base + self.num_envs > 2**64:
                raise ValueError(f"seed + env index must lie in [0, 2**64) for every env; got seed={seed}, "
                                 f"env_offset={self.env_offset}, num_envs={self.num_envs}")
        s = self.state.c()
        check(lib().drl_reset(ctypes.byref(self._cp), ctypes.byref(s), int(reseed), seed_base, _ptr(env_mask),
                              _stream(self.device)), "drl_reset")  # (ends with a refill)
        self._since_refill = 0
        return self.state

    def refill(self):
        """Top up every env's respawn-candidate ring (drl_refill; step() does it every
        ``refill_every`` steps).  Never changes results, only where the MT draws happen."""
        s = self.state.c()
        check(lib().drl_refill(ctypes.byref(self._cp), ctypes.byref(s), _stream(self.device)), "drl_refill")
        self._since_refill = 0

    def step(self, actions: torch.Tensor, obs_k: int = 0, rewards: Optional[torch.Tensor] = None,
             dones: Optional[torch.Tensor] = None, obs: Optional[torch.Tensor] = None,
             obs_stream: Optional[bool] = None, code: Optional[torch.Tensor] = None, replay=None,
             replay_obs: Optional[torch.Tensor] = None, synth=None):
        """env.py:112-215 for every env.  actions int32 [E, N] by drone index.

        Returns (rewards f32 [E,N], dones bool-as-uint8 [E,N]) and, when
        obs_k > 0, the fused observation f32 [E, obs_k, W, W, 6] of drone
        indices 0..obs_k-1 after the step (train_jax.py:55-56 uses obs_k=1).
        obs_stream: write the observation with streaming stores
        (DRL_STEP_OBS_STREAM) or cached ones; None (default) picks
        ``default_obs_stream`` (streaming at step_group_lanes >= 16).  Results
        are identical either way.
        code: uint8 [E, policy_code_bytes] (``new_code()``): also write drone
        0's policy code after the step (drl_step_code), the input of a
        QNetwork(input="code"); with obs_k = 0 the code alone (no f32
        observation rows are written).
        replay: a ReplayBuffer(code_radius=window_radius) and replay_obs the
        code rows the act read (uint8 [E, policy_code_bytes], another buffer
        than ``code``): the step also lands its drone-0 transitions
        (replay_obs, actions[:, 0], rewards[:, 0], code, dones[:, 0]) in the
        ring, exactly as a following ``replay.add_many`` would, in the same
        launch (drl_step_code_replay; obs_k must be 0).  The batch
        description is left in ``replay.last_batch``.
        synth=(seed, step) (with replay=): drone indices 1..N-1 act as
        ``synth_actions(seed, step)`` would write them, drawn inside the step
        (drl_step_code_replay_synth); only actions[:, 0] is read (the
        agent's), the other columns are neither read nor written.
        """
        E, N = self.num_envs, self.n_drones
        actions = self._check(actions, torch.int32, (E, N), "actions")
        if code is not None:
            self._check_out(code, torch.uint8, (E, self.policy_code_bytes), "code")
        if rewards is None:
            rewards = torch.empty((E, N), dtype=torch.float32, device=self.device)
        if dones is None:
            dones = torch.empty((E, N), dtype=torch.uint8, device=self.device)
        W = self.layout.obs_window
        if obs_k and obs is None:
            obs = torch.empty((E, obs_k, W, W, 6), dtype=torch.float32, device=self.device)
        self._check_out(rewards, torch.float32, (E, N), "rewards")
        self._check_out(dones, torch.uint8, (E, N), "dones")
        if obs_k:
            self._check_out(obs, torch.float32, (E, obs_k, W, W, 6), "obs")
        s = self.state.c()
        if obs_stream is None:
            obs_stream = self.default_obs_stream
        flags = DRL_STEP_OBS_STREAM if obs_stream else 0
        # the refill cadence advances only once the launch is accepted: a call refused by the checks below
        # (or by the library) leaves the env exactly as it was
        since = self._since_refill
        if self.refill_every > 0:
            since += 1
            if since >= self.refill_every:
                since = 0
                flags |= DRL_STEP_REFILL
        if synth is not None and replay is None:
            raise ValueError("synth= needs replay= (drl_step_code_replay_synth)")
        if replay is not None:
            if code is None or obs_k or replay_obs is None:
                raise ValueError("replay= needs code= and replay_obs=, and obs_k=0")
            replay._add_from_step(self, actions, rewards, dones, replay_obs, code, flags, synth=synth)
            self._since_refill = since
            return rewards, dones
        check(lib().drl_step_code(ctypes.byref(self._cp), ctypes.byref(s), _ptr(actions), _ptr(rewards), _ptr(dones),
                                  _ptr(obs) if obs_k else None, int(obs_k), None if code is None else _ptr(code),
                                  _ptr(self.err), flags, _stream(self.device)), "drl_step")
        self._since_refill = since
        if obs_k:
            return rewards, dones, obs
        return rewards, dones

    def rollout(self, actions: torch.Tensor, obs_k: int = 0, every_step: bool = True,
                rewards: Optional[torch.Tensor] = None, dones: Optional[torch.Tensor] = None,
                obs: Optional[torch.Tensor] = None):
        """T steps in one launch (jax run_steps, env.py:252-272, plus per-step
        outputs): actions int32 [T, E, N].  Same results as T step() calls.

        every_step: rewards/dones [T, E, N] and obs [T, E, obs_k, W, W, 6];
        otherwise [E, N] / [E, obs_k, W, W, 6] holding the last step's.
        """
        E, N = self.num_envs, self.n_drones
        if actions.dim() != 3 or actions.shape[1:] != (E, N):
            raise ValueError(f"actions must be [T, {E}, {N}], got {tuple(actions.shape)}")
        T = actions.shape[0]
        actions = self._check(actions, torch.int32, (T, E, N), "actions")
        lead = (T,) if every_step else ()
        if rewards is None:
            rewards = torch.empty(lead + (E, N), dtype=torch.float32, device=self.device)
        if dones is None:
            dones = torch.empty(lead + (E, N), dtype=torch.uint8, device=self.device)
        W = self.layout.obs_window
        if obs_k and obs is None:
            obs = torch.empty(lead + (E, obs_k, W, W, 6), dtype=torch.float32, device=self.device)
        self._check_out(rewards, torch.float32, lead + (E, N), "rewards")
        self._check_out(dones, torch.uint8, lead + (E, N), "dones")
        if obs_k:
            self._check_out(obs, torch.float32, lead + (E, obs_k, W, W, 6), "obs")
        ostride = E * obs_k * W * W * 6 if every_step else 0
        s = self.state.c()
        check(lib().drl_rollout(ctypes.byref(self._cp), ctypes.byref(s), T, _ptr(actions), E * N, _ptr(rewards),
                                _ptr(dones), E * N if every_step else 0, _ptr(obs) if obs_k else None, int(obs_k),
                                ostride, _ptr(self.err), _stream(self.device)), "drl_rollout")  # (ends with a refill)
        self._since_refill = 0
        if obs_k:
            return rewards, dones, obs
        return rewards, dones

    def get_obs(self, k: Optional[int] = None, out: Optional[torch.Tensor] = None,
                code: Optional[torch.Tensor] = None) -> torch.Tensor:
        """WindowedGridView observation of drone indices 0..k-1: f32 [E, k, W, W, 6].
        code: uint8 [E, policy_code_bytes], also filled with drone 0's policy code."""
        k = self.n_drones if k is None else int(k)
        W = self.layout.obs_window
        if out is None:
            out = torch.empty((self.num_envs, k, W, W, 6), dtype=torch.float32, device=self.device)
        if code is not None:
            self._check_out(code, torch.uint8, (self.num_envs, self.policy_code_bytes), "code")
        s = self.state.c()
        check(lib().drl_obs_code(ctypes.byref(self._cp), ctypes.byref(s), k, _ptr(out),
                                 None if code is None else _ptr(code), _stream(self.device)), "drl_obs")
        return out

    def get_code(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Drone index 0's policy code alone, uint8 [E, policy_code_bytes] (drl_obs_code, no f32 rows)."""
        if out is None:
            out = self.new_code()
        self._check_out(out, torch.uint8, (self.num_envs, self.policy_code_bytes), "code")
        s = self.state.c()
        check(lib().drl_obs_code(ctypes.byref(self._cp), ctypes.byref(s), 1, None, _ptr(out), _stream(self.device)),
              "drl_obs")
        return out

    @property
    def policy_code_bytes(self) -> int:
        """Bytes per env of the policy code (drl_policy_code_bytes)."""
        return int(lib().drl_policy_code_bytes(self.params.window_radius))

    def new_code(self) -> torch.Tensor:
        """A policy-code buffer, uint8 [E, policy_code_bytes] (16-B aligned rows)."""
        return torch.empty((self.num_envs, self.policy_code_bytes), dtype=torch.uint8, device=self.device)

    def get_grid(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """GridView observation (wrappers.py:34-43): the base grid f32 [E, side, side, 6]
        that every drone of an env sees."""
        G = self.params.side
        if out is None:
            out = torch.empty((self.num_envs, G, G, 6), dtype=torch.float32, device=self.device)
        s = self.state.c()
        check(lib().drl_grid_obs(ctypes.byref(self._cp), ctypes.byref(s), _ptr(out), _stream(self.device)),
              "drl_grid_obs")
        return out

    def synth_actions(self, seed: int, step: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Uniform synthetic actions (counter hash; identical stream to the oracle's)."""
        if out is None:
            out = torch.empty((self.num_envs, self.n_drones), dtype=torch.int32, device=self.device)
        check(lib().drl_synth_actions(seed, step, self.env_offset, self.num_envs, self.n_drones, _ptr(out),
                                      _stream(self.device)), "drl_synth_actions")
        return out

    # ------------------------------------------------------ state plumbing --
    def decode(self) -> dict:
        """Per-index drone vectors (jax DroneEnvState fields) + dict order + grid."""
        E, N, G = self.num_envs, self.n_drones, self.side
        t = lambda dt: torch.empty((E, N), dtype=dt, device=self.device)
        out = dict(order=t(torch.int32), y=t(torch.int32), x=t(torch.int32), charge=t(torch.int32),
                   carrying=t(torch.uint8))
        s = self.state.c()
        check(lib().drl_decode(ctypes.byref(self._cp), ctypes.byref(s), _ptr(out["order"]), _ptr(out["y"]),
                               _ptr(out["x"]), _ptr(out["charge"]), _ptr(out["carrying"]), _stream(self.device)),
              "drl_decode")
        out["ground"] = unpack_ground(self.state.ground, G)
        out["mt_index"] = self.mt_words_device()[:, 624]
        return out

    def set_state(self, ground, order, y, x, charge, carrying, mt_words=None):
        """Hand-built states (as jax_tests/test_env.py:14-110 builds DroneEnvState)."""
        E, N, G = self.num_envs, self.n_drones, self.side
        dev = self.device
        as_t = lambda a, dt: torch.as_tensor(a, dtype=dt).to(dev).reshape(E, -1).contiguous()
        g = as_t(ground, torch.uint8)
        assert g.shape[1] == G * G
        self.state.ground.copy_(pack_ground(g, self.state.ground.shape[1]))
        o, yy, xx, ch = (as_t(v, torch.int32) for v in (order, y, x, charge))
        k = as_t(carrying, torch.uint8)
        if not torch.equal(o.sort(1).values, torch.arange(N, device=dev, dtype=torch.int32).expand(E, N)):
            raise ValueError("order must be a permutation of the drone indices in every env")
        if (yy < 0).any() or (yy >= G).any() or (xx < 0).any() or (xx >= G).any():
            raise ValueError("drone positions outside the grid")
        if (ch < 0).any() or (ch > 100).any():
            raise ValueError("charge must lie in [0, 100]")
        s = self.state.c()
        check(lib().drl_encode(ctypes.byref(self._cp), ctypes.byref(s), _ptr(o), _ptr(yy), _ptr(xx), _ptr(ch),
                               _ptr(k), _stream(dev)), "drl_encode")
        if mt_words is not None:
            self.set_mt_words(mt_words)

    def set_mt_words(self, words625):
        """Load CPython getstate() words (624 state words + index) for every env
        (drl_mt_set: block 0, then a refill of the candidate rings)."""
        w = torch.as_tensor(words625, dtype=torch.int64).reshape(-1, 625)
        w = (w & 0xFFFFFFFF).to(torch.int64)
        if w.shape[0] == 1:
            w = w.expand(self.num_envs, 625)
        if w.shape[0] != self.num_envs:
            raise ValueError(f"need 1 or {self.num_envs} rows of 625 words, got {w.shape[0]}")
        if ((w[:, 624] < 0) | (w[:, 624] > 624)).any():
            raise ValueError("MT index must lie in [0, 624] (CPython setstate)")
        w = torch.where(w >= 2**31, w - 2**32, w).to(torch.int32).to(self.device).contiguous()
        s = self.state.c()
        check(lib().drl_mt_set(ctypes.byref(self._cp), ctypes.byref(s), _ptr(w), _ptr(self.err), _stream(self.device)),
              "drl_mt_set")
        self._since_refill = 0

    def mt_words_device(self) -> torch.Tensor:
        """CPython getstate() words of every env, int32 [E, 625] on the device (drl_mt_get)."""
        out = torch.empty((self.num_envs, 625), dtype=torch.int32, device=self.device)
        s = self.state.c()
        check(lib().drl_mt_get(ctypes.byref(self._cp), ctypes.byref(s), _ptr(out), _stream(self.device)), "drl_mt_get")
        return out

    def mt_words(self):
        """CPython getstate() words (624 state words + index) per env, as int64 on the host."""
        return self.mt_words_device().cpu().to(torch.int64) & 0xFFFFFFFF

    def check_errors(self):
        """Synchronise and raise if a kernel flagged an error since the last check."""
        e = int(self.err.item())
        if e:
            self.err.zero_()
            msgs = []
            if e & DRL_ERR_BAD_ACTION:
                msgs.append("action index out of range (IndexError in the reference)")
            if e & DRL_ERR_NO_FREE_CELL:
                msgs.append("respawn found no free cell")
            if e & DRL_ERR_BAD_STATE:
                msgs.append("MT index outside [0, 624] in a set state (clamped to 624)")
            raise DroneRLError("; ".join(msgs))

    # ------------------------------------------------------------- helpers --
    def _check_out(self, t: torch.Tensor, dtype, shape, name):
        """Output buffers are written in place: no conversion, exact layout."""
        if (not isinstance(t, torch.Tensor) or t.device != self.device or t.dtype != dtype
                or tuple(t.shape) != tuple(shape) or not t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous {dtype} tensor of shape {tuple(shape)} on {self.device}")

    def _check(self, t: torch.Tensor, dtype, shape, name):
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(t)
        if t.device != self.device:
            t = t.to(self.device)
        if t.dtype != dtype:
            t = t.to(dtype)
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
        return t.contiguous()
