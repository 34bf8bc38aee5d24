"""ctypes binding of the library-owned env handles (include/dronerl.h drl_env_*,
SURVEY.md §8 B2/B3) — what a maintainer binds from Python when the library
should own the state.  BatchedDeliveryDrones (env.py) is the tensor-level
façade over the stateless calls; both run the same kernels.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from ._native import DrlLayout, DrlParams, DrlState, DroneRLError, lib
from .params import EnvParams


class DrlStateView(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("ground", "order", "y", "x", "charge", "carry", "mt")]


_vp = ctypes.c_void_p


def _bind(L):
    if getattr(L, "_env_ready", False):
        return L
    i32, i64, u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    sig = {
        "drl_env_create": [ctypes.POINTER(DrlParams), i32, i64, i64, u64, ctypes.POINTER(_vp)],
        "drl_env_destroy": [_vp],
        "drl_env_seed": [_vp, u64],
        "drl_env_reset": [_vp, _vp, _vp],
        "drl_env_step": [_vp, _vp, _vp, _vp, _vp],
        "drl_env_step_obs": [_vp, _vp, _vp, _vp, i32, _vp, _vp],
        "drl_env_obs": [_vp, i32, _vp, _vp],
        "drl_env_get_state": [_vp, ctypes.POINTER(DrlStateView), _vp],
        "drl_env_set_state": [_vp, ctypes.POINTER(DrlStateView), _vp],
        "drl_env_state": [_vp, ctypes.POINTER(DrlState), ctypes.POINTER(DrlParams), ctypes.POINTER(DrlLayout)],
        "drl_env_errors": [_vp, ctypes.POINTER(i32), i32, _vp],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = ctypes.c_int
    L._env_ready = True
    return L


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class DrlEnvHandle:
    """A drl_env handle on one device: `num_envs` envs, global indices
    env_offset + e, first reset seeded random.seed(base_seed + env_offset + e)."""

    def __init__(self, params: EnvParams, num_envs: int, device: int = 0, env_offset: int = 0, base_seed: int = 0):
        self.L = _bind(lib())
        self.params = params
        self.device = torch.device("cuda", device)
        self._cp = params.to_c()
        h = _vp()
        self._check(self.L.drl_env_create(ctypes.byref(self._cp), device, num_envs, env_offset, base_seed,
                                          ctypes.byref(h)))
        self._h = h
        self.num_envs = num_envs
        lay = DrlLayout()
        self._check(self.L.drl_env_state(self._h, None, None, ctypes.byref(lay)))
        self.layout = lay

    def _check(self, rc):
        if rc:
            raise DroneRLError(self.L.drl_last_error().decode())

    def _stream(self):
        return _vp(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "_h", None):
            self._check(self.L.drl_env_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def seed(self, base_seed: int):
        self._check(self.L.drl_env_seed(self._h, base_seed))

    def reset(self, env_mask: Optional[torch.Tensor] = None):
        self._check(self.L.drl_env_reset(self._h, _ptr(env_mask), self._stream()))

    def step(self, actions: torch.Tensor, obs_k: int = 0):
        E, N = self.num_envs, self.params.n_drones
        rewards = torch.empty((E, N), dtype=torch.float32, device=self.device)
        dones = torch.empty((E, N), dtype=torch.uint8, device=self.device)
        if obs_k:
            W = self.layout.obs_window
            obs = torch.empty((E, obs_k, W, W, 6), dtype=torch.float32, device=self.device)
            self._check(self.L.drl_env_step_obs(self._h, _ptr(actions), _ptr(rewards), _ptr(dones), obs_k,
                                                _ptr(obs), self._stream()))
            return rewards, dones, obs
        self._check(self.L.drl_env_step(self._h, _ptr(actions), _ptr(rewards), _ptr(dones), self._stream()))
        return rewards, dones

    def obs(self, k: int = 1) -> torch.Tensor:
        W = self.layout.obs_window
        out = torch.empty((self.num_envs, k, W, W, 6), dtype=torch.float32, device=self.device)
        self._check(self.L.drl_env_obs(self._h, k, _ptr(out), self._stream()))
        return out

    def get_state(self) -> dict:
        E, N, G = self.num_envs, self.params.n_drones, self.params.side
        d = dict(ground=torch.empty((E, G, G), dtype=torch.uint8, device=self.device),
                 order=torch.empty((E, N), dtype=torch.int32, device=self.device),
                 y=torch.empty((E, N), dtype=torch.int32, device=self.device),
                 x=torch.empty((E, N), dtype=torch.int32, device=self.device),
                 charge=torch.empty((E, N), dtype=torch.int32, device=self.device),
                 carry=torch.empty((E, N), dtype=torch.uint8, device=self.device),
                 mt=torch.empty((E, 625), dtype=torch.int32, device=self.device))
        v = DrlStateView(*(d[k].data_ptr() for k in ("ground", "order", "y", "x", "charge", "carry", "mt")))
        self._check(self.L.drl_env_get_state(self._h, ctypes.byref(v), self._stream()))
        return d

    def set_state(self, d: dict):
        keep = [d[k].to(self.device).contiguous() for k in ("ground", "order", "y", "x", "charge", "carry", "mt")]
        v = DrlStateView(*(t.data_ptr() for t in keep))
        self._check(self.L.drl_env_set_state(self._h, ctypes.byref(v), self._stream()))
        torch.cuda.current_stream(self.device).synchronize()  # `keep` may be freed after this

    def errors(self, clear: bool = True) -> int:
        f = ctypes.c_int32(0)
        self._check(self.L.drl_env_errors(self._h, ctypes.byref(f), 1 if clear else 0, self._stream()))
        return f.value
