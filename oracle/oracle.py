"""ORACLE — TEST INFRASTRUCTURE ONLY (not part of the product).

ctypes wrapper around ``oracle/liboracle.so``, the plain-C restatement of the
nyx-ai/droneRL ``torch_impl`` environment (see the header of
``oracle/dronerl_oracle.c`` for the file:line map).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DRL_ORACLE_LIB: another build of the same source (the sanitizer build of `make asan`)
_LIB_PATH = os.environ.get("DRL_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    """Compile liboracle.so from oracle/dronerl_oracle.c (gcc, seconds)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class OrcParams(ctypes.Structure):
    _fields_ = [
        ("side", ctypes.c_int32),
        ("n_drones", ctypes.c_int32),
        ("charge", ctypes.c_int32),
        ("discharge", ctypes.c_int32),
        ("packets_factor", ctypes.c_int32),
        ("dropzones_factor", ctypes.c_int32),
        ("stations_factor", ctypes.c_int32),
        ("skyscrapers_factor", ctypes.c_int32),
        ("pickup_reward", ctypes.c_double),
        ("delivery_reward", ctypes.c_double),
        ("crash_reward", ctypes.c_double),
        ("charge_reward", ctypes.c_double),
    ]


class NoFreeCell(RuntimeError):
    """A respawn found every cell blocked: the reference's
    _find_respawn_position (env.py:226-233) would loop forever."""


def _step_status(st: int):
    if st == -1:
        raise IndexError("list index out of range")
    if st == -2:
        raise NoFreeCell("respawn found no free cell (the reference loops forever)")
    if st:
        raise RuntimeError(f"orc_step failed ({st})")


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "dronerl_oracle.c")
        if not os.environ.get("DRL_ORACLE_LIB") and (not os.path.exists(_LIB_PATH)
                                                     or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i32, i64, u32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
        L.orc_mt_sizeof.restype = ctypes.c_size_t
        L.orc_mt_seed.argtypes = [vp, u64]
        L.orc_mt_genrand.argtypes = [vp]
        L.orc_mt_genrand.restype = u32
        L.orc_getrandbits.argtypes = [vp, ctypes.c_int]
        L.orc_getrandbits.restype = u32
        L.orc_randbelow.argtypes = [vp, u32]
        L.orc_randbelow.restype = u32
        L.orc_shuffle.argtypes = [vp, vp, i32]
        L.orc_sample.argtypes = [vp, vp, i32, i32, vp]
        L.orc_sample.restype = ctypes.c_int
        L.orc_mt_get.argtypes = [vp, vp]
        L.orc_mt_set.argtypes = [vp, vp]
        L.orc_env_create.argtypes = [ctypes.POINTER(OrcParams)]
        L.orc_env_create.restype = vp
        L.orc_env_destroy.argtypes = [vp]
        L.orc_env_rng.argtypes = [vp]
        L.orc_env_rng.restype = vp
        L.orc_reset.argtypes = [vp]
        L.orc_reset.restype = ctypes.c_int
        L.orc_step.argtypes = [vp, vp, vp, vp]
        L.orc_step.restype = ctypes.c_int
        L.orc_obs.argtypes = [vp, i32, i32, vp]
        L.orc_get_state.argtypes = [vp] + [vp] * 7
        L.orc_set_state.argtypes = [vp] + [vp] * 7
        L.orc_synth_action.argtypes = [u64, u64, u64, u32, u32]
        L.orc_synth_action.restype = i32
        L.orc_rollout.argtypes = [ctypes.POINTER(OrcParams), i64, i64, u64, u64, i64, i32, i32, i32] + [vp] * 9
        L.orc_rollout.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class MT:
    """CPython-compatible MT19937 stream (the oracle's copy)."""

    def __init__(self, seed: int | None = None):
        self._buf = ctypes.create_string_buffer(lib().orc_mt_sizeof())
        if seed is not None:
            self.seed(seed)

    @property
    def _p(self):
        return ctypes.cast(self._buf, ctypes.c_void_p)

    def seed(self, s: int):
        lib().orc_mt_seed(self._p, s)

    def genrand(self) -> int:
        return lib().orc_mt_genrand(self._p)

    def getrandbits(self, k: int) -> int:
        return lib().orc_getrandbits(self._p, k)

    def randbelow(self, n: int) -> int:
        return lib().orc_randbelow(self._p, n)

    def randint(self, a: int, b: int) -> int:
        return a + self.randbelow(b - a + 1)

    def shuffle(self, x: list) -> list:
        arr = np.ascontiguousarray(x, dtype=np.int32)
        lib().orc_shuffle(self._p, _ptr(arr), len(arr))
        return arr.tolist()

    def sample(self, pop: list, k: int) -> list:
        arr = np.ascontiguousarray(pop, dtype=np.int32)
        out = np.zeros(max(k, 1), dtype=np.int32)
        if lib().orc_sample(self._p, _ptr(arr), len(arr), k, _ptr(out)):
            raise ValueError("Sample larger than population or is negative")
        return out[:k].tolist()

    def getstate_words(self) -> np.ndarray:
        w = np.zeros(625, dtype=np.uint32)
        lib().orc_mt_get(self._p, _ptr(w))
        return w


@dataclass
class Params:
    side: int
    n_drones: int
    charge: int = 20
    discharge: int = 10
    packets_factor: int = 3
    dropzones_factor: int = 2
    stations_factor: int = 2
    skyscrapers_factor: int = 3
    pickup_reward: float = 0.0
    delivery_reward: float = 1.0
    crash_reward: float = -1.0
    charge_reward: float = -0.1

    def c(self) -> OrcParams:
        return OrcParams(self.side, self.n_drones, self.charge, self.discharge, self.packets_factor,
                         self.dropzones_factor, self.stations_factor, self.skyscrapers_factor,
                         float(self.pickup_reward), float(self.delivery_reward), float(self.crash_reward),
                         float(self.charge_reward))


class OracleEnv:
    """One torch_impl-semantics env (CPU restatement)."""

    def __init__(self, p: Params):
        self.p = p
        self._cp = p.c()
        self._e = lib().orc_env_create(ctypes.byref(self._cp))
        if not self._e:
            raise ValueError("bad params")
        self.rng = MT()
        self.rng._buf = None  # the env owns its own stream; access through helpers below

    def __del__(self):
        try:
            lib().orc_env_destroy(self._e)
        except Exception:
            pass

    def seed(self, s: int):
        lib().orc_mt_seed(lib().orc_env_rng(self._e), s)

    def set_mt_words(self, w625):
        w = np.ascontiguousarray(w625, dtype=np.uint32)
        lib().orc_mt_set(lib().orc_env_rng(self._e), _ptr(w))

    def reset(self):
        if lib().orc_reset(self._e):
            raise ValueError("Not enough positions to spawn objects")

    def step(self, actions):
        N = self.p.n_drones
        a = np.ascontiguousarray(actions, dtype=np.int32)
        assert a.shape == (N,)
        r = np.zeros(N, dtype=np.float64)
        d = np.zeros(N, dtype=np.uint8)
        _step_status(lib().orc_step(self._e, _ptr(a), _ptr(r), _ptr(d)))
        return r, d.astype(bool)

    def obs(self, radius: int = 3, k: int | None = None) -> np.ndarray:
        k = self.p.n_drones if k is None else k
        W = 2 * radius + 1
        out = np.zeros((k, W, W, 6), dtype=np.float32)
        lib().orc_obs(self._e, radius, k, _ptr(out))
        return out

    def state(self) -> dict:
        G, N = self.p.side, self.p.n_drones
        ground = np.zeros((G, G), dtype=np.uint8)
        order = np.zeros(N, dtype=np.int32)
        y = np.zeros(N, dtype=np.int32)
        x = np.zeros(N, dtype=np.int32)
        ch = np.zeros(N, dtype=np.int32)
        pk = np.zeros(N, dtype=np.uint8)
        mt = np.zeros(625, dtype=np.uint32)
        lib().orc_get_state(self._e, _ptr(ground), _ptr(order), _ptr(y), _ptr(x), _ptr(ch), _ptr(pk), _ptr(mt))
        return dict(ground=ground, order=order, y=y, x=x, charge=ch, packet=pk.astype(bool), mt=mt)

    def set_state(self, ground, order, y, x, charge, packet, mt=None):
        c = lambda a, t: np.ascontiguousarray(a, dtype=t)
        g = c(ground, np.uint8)
        o, yy, xx, ch = c(order, np.int32), c(y, np.int32), c(x, np.int32), c(charge, np.int32)
        pk = c(packet, np.uint8)
        m = None if mt is None else c(mt, np.uint32)
        lib().orc_set_state(self._e, _ptr(g), _ptr(o), _ptr(yy), _ptr(xx), _ptr(ch), _ptr(pk), _ptr(m))


def synth_action(seed: int, step: int, env: int, n_drones: int, drone: int) -> int:
    return lib().orc_synth_action(seed, step, env, n_drones, drone)


def synth_actions(seed: int, step: int, env_ids, n_drones: int) -> np.ndarray:
    env_ids = np.asarray(env_ids)
    out = np.zeros((len(env_ids), n_drones), dtype=np.int32)
    L = lib()
    for i, e in enumerate(env_ids):
        for d in range(n_drones):
            out[i, d] = L.orc_synth_action(seed, step, int(e), n_drones, d)
    return out


def rollout(p: Params, E: int, steps: int, seed0: int = 0, action_seed: int = 0, env_offset: int = 0,
            nthreads: int = 1, want_state: bool = True, obs_k: int = 0, radius: int = 3):
    """E independent envs, env e seeded random.seed(seed0 + env_offset + e),
    `steps` synthetic-action steps.  Returns a dict of final states + sums."""
    G, N = p.side, p.n_drones
    cp = p.c()
    out = dict(reward_sum=np.zeros(E, dtype=np.float64), done_sum=np.zeros(E, dtype=np.int64))
    if want_state:
        out.update(ground=np.zeros((E, G, G), dtype=np.uint8), order=np.zeros((E, N), dtype=np.int32),
                   y=np.zeros((E, N), dtype=np.int32), x=np.zeros((E, N), dtype=np.int32),
                   charge=np.zeros((E, N), dtype=np.int32), packet=np.zeros((E, N), dtype=np.uint8),
                   mt=np.zeros((E, 625), dtype=np.uint32))
    g = lambda k: _ptr(out.get(k))
    st = lib().orc_rollout(ctypes.byref(cp), E, env_offset, seed0, action_seed, steps, nthreads, obs_k, radius,
                           g("ground"), g("order"), g("y"), g("x"), g("charge"), g("packet"), g("mt"),
                           g("reward_sum"), g("done_sum"))
    if st:
        raise ValueError("rollout failed (reset could not place objects)")
    if want_state:
        out["packet"] = out["packet"].astype(bool)
    return out


class OracleMulti:
    """E oracle envs stepped together (C loop, optional threads)."""

    def __init__(self, p: Params, E: int):
        L = lib()
        if not hasattr(L, "_multi_ready"):
            vp = ctypes.c_void_p
            L.orc_multi_create.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int64]
            L.orc_multi_create.restype = vp
            L.orc_multi_destroy.argtypes = [vp]
            L.orc_multi_reset.argtypes = [vp, vp]
            L.orc_multi_reset.restype = ctypes.c_int
            L.orc_multi_step.argtypes = [vp, vp, vp, vp, ctypes.c_int32]
            L.orc_multi_step.restype = ctypes.c_int
            L.orc_multi_get_state.argtypes = [vp] * 8
            L.orc_multi_set_state.argtypes = [vp] * 8
            L.orc_multi_obs.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp]
            L._multi_ready = True
        self.p, self.E = p, E
        self._cp = p.c()
        self._m = L.orc_multi_create(ctypes.byref(self._cp), E)

    def __del__(self):
        try:
            lib().orc_multi_destroy(self._m)
        except Exception:
            pass

    def reset(self, seeds=None):
        s = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint64)
        if lib().orc_multi_reset(self._m, _ptr(s)):
            raise ValueError("Not enough positions to spawn objects")

    def step(self, actions, nthreads: int = 8):
        N = self.p.n_drones
        a = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.E, N)
        r = np.zeros((self.E, N), dtype=np.float64)
        d = np.zeros((self.E, N), dtype=np.uint8)
        _step_status(lib().orc_multi_step(self._m, _ptr(a), _ptr(r), _ptr(d), nthreads))
        return r, d.astype(bool)

    def state(self) -> dict:
        E, G, N = self.E, self.p.side, self.p.n_drones
        out = dict(ground=np.zeros((E, G, G), np.uint8), order=np.zeros((E, N), np.int32),
                   y=np.zeros((E, N), np.int32), x=np.zeros((E, N), np.int32), charge=np.zeros((E, N), np.int32),
                   packet=np.zeros((E, N), np.uint8), mt=np.zeros((E, 625), np.uint32))
        lib().orc_multi_get_state(self._m, *(_ptr(out[k]) for k in
                                             ["ground", "order", "y", "x", "charge", "packet", "mt"]))
        out["packet"] = out["packet"].astype(bool)
        return out

    def set_state(self, ground, order, y, x, charge, packet, mt=None):
        c = lambda a, t: None if a is None else np.ascontiguousarray(a, dtype=t)
        lib().orc_multi_set_state(self._m, _ptr(c(ground, np.uint8)), _ptr(c(order, np.int32)),
                                  _ptr(c(y, np.int32)), _ptr(c(x, np.int32)), _ptr(c(charge, np.int32)),
                                  _ptr(c(packet, np.uint8)), _ptr(c(mt, np.uint32)))

    def obs(self, radius: int = 3, k: int | None = None) -> np.ndarray:
        k = self.p.n_drones if k is None else k
        W = 2 * radius + 1
        out = np.zeros((self.E, k, W, W, 6), dtype=np.float32)
        lib().orc_multi_obs(self._m, radius, k, _ptr(out))
        return out
