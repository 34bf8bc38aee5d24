"""ctypes binding of libdronerl.so (include/dronerl.h).

There is no CPU fallback: if the HIP library is missing or fails to load,
every entry point raises.  Build it with ``python -m dronerl_amd.build``
(``__graft_entry__.build()`` does this too).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DRL_LIB: an alternative build of the same library (tools/variants.py A/B runs)
LIB_PATH = os.environ.get("DRL_LIB") or os.path.join(_HERE, "libdronerl.so")

DRL_ABI_VERSION = 9  # include/dronerl.h
DRL_MT_WORDS = 1776  # per-env RNG row: two MT blocks + the respawn-candidate ring
DRL_MT_RING = 1248
DRL_MT_RING_END = 1760
DRL_CAND_SLOTS = 512
DRL_MAX_DRONES = 64
DRL_MAX_SIDE = 128
DRL_MAX_RADIUS = 8
DRL_ERR_BAD_ACTION = 1
DRL_ERR_NO_FREE_CELL = 2
DRL_ERR_BAD_STATE = 4
DRL_ERR_QNET_RANGE = 8  # drl_qnet_act (f32): an operand outside fp16's split range
DRL_STEP_OBS_STREAM = 1  # drl_step_ex flag: streaming (non-temporal) observation stores
DRL_STEP_REFILL = 2      # drl_step_ex flag: top up the respawn-candidate rings after the step

# Every symbol include/dronerl.h declares (tests check the .so exports them all).
EXPORTS = ["drl_abi_version", "drl_last_error", "drl_side_from_density", "drl_layout_query", "drl_reset",
           "drl_step", "drl_step_ex", "drl_rollout", "drl_refill", "drl_mt_get", "drl_mt_set", "drl_obs", "drl_grid_obs", "drl_decode", "drl_encode", "drl_synth_actions",
           # the policy code (drone 0's window, one u16 per cell) for drl_qnet_act_code
           "drl_policy_code_bytes", "drl_step_code", "drl_obs_code", "drl_code_decode",
           # library-owned env handles
           "drl_env_create", "drl_env_destroy", "drl_env_seed", "drl_env_reset", "drl_env_step",
           "drl_env_step_obs", "drl_env_obs", "drl_env_grid_obs", "drl_env_get_state", "drl_env_set_state", "drl_env_state",
           "drl_env_errors",
           # DQN consumer
           "drl_qnet_packed_bytes", "drl_qnet_pack", "drl_qnet_act", "drl_qnet_act_synth", "drl_qnet_act_code",
           "drl_replay_add", "drl_qnet_act_eps", "drl_step_code_replay",
           "drl_step_code_replay_synth",
           # DQN learner (train_step / update_target / update_epsilon / sample)
           "drl_dqn_layout_query", "drl_dqn_init", "drl_dqn_train", "drl_dqn_train_fresh", "drl_dqn_sample_rows",
           # measurement helper (the measured copy-kernel peak)
           "drl_hbm_probe"]


class DrlParams(ctypes.Structure):
    _fields_ = [
        ("side", ctypes.c_int32),
        ("n_drones", ctypes.c_int32),
        ("charge", ctypes.c_int32),
        ("discharge", ctypes.c_int32),
        ("packets_factor", ctypes.c_int32),
        ("dropzones_factor", ctypes.c_int32),
        ("stations_factor", ctypes.c_int32),
        ("skyscrapers_factor", ctypes.c_int32),
        ("window_radius", ctypes.c_int32),
        ("pickup_reward", ctypes.c_float),
        ("delivery_reward", ctypes.c_float),
        ("crash_reward", ctypes.c_float),
        ("charge_reward", ctypes.c_float),
    ]


class DrlLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in [
        "side", "n_drones", "cells", "ground_stride", "drone_stride", "mt_stride", "obs_window", "obs_floats",
        "step_group_lanes", "step_lds_bytes", "cand_slots", "refill_every"]]


class DrlState(ctypes.Structure):
    _fields_ = [
        ("ground", ctypes.c_void_p),
        ("drones", ctypes.c_void_p),
        ("mt", ctypes.c_void_p),
        ("mt_index", ctypes.c_void_p),
        ("num_envs", ctypes.c_int64),
    ]


class DroneRLError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libdronerl.so, raising loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DroneRLError(f"{LIB_PATH} is missing: build the HIP extension with `python -m dronerl_amd.build` "
                           "(there is no CPU fallback)")
    if not os.environ.get("DRL_LIB"):
        # the in-tree library must have been built from the sources beside it
        from . import build as _b
        if not _b.up_to_date():
            raise DroneRLError(f"{LIB_PATH} was not built from the current sources (digest mismatch with "
                               f"{_b.HASH}): rebuild with `python -m dronerl_amd.build`")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    P = ctypes.POINTER(DrlParams)
    S = ctypes.POINTER(DrlState)
    L.drl_abi_version.restype = i32
    L.drl_last_error.restype = ctypes.c_char_p
    L.drl_side_from_density.argtypes = [i32, ctypes.c_double]
    L.drl_side_from_density.restype = i32
    L.drl_layout_query.argtypes = [P, ctypes.POINTER(DrlLayout)]
    L.drl_reset.argtypes = [P, S, i32, u64, vp, vp]
    L.drl_step.argtypes = [P, S, vp, vp, vp, vp, i32, vp, vp]
    L.drl_step_ex.argtypes = [P, S, vp, vp, vp, vp, i32, vp, ctypes.c_uint32, vp]
    L.drl_rollout.argtypes = [P, S, i32, vp, i64, vp, vp, i64, vp, i32, i64, vp, vp]
    L.drl_refill.argtypes = [P, S, vp]
    L.drl_mt_get.argtypes = [P, S, vp, vp]
    L.drl_mt_set.argtypes = [P, S, vp, vp, vp]
    L.drl_obs.argtypes = [P, S, i32, vp, vp]
    L.drl_obs_code.argtypes = [P, S, i32, vp, vp, vp]
    L.drl_step_code.argtypes = [P, S, vp, vp, vp, vp, i32, vp, vp, ctypes.c_uint32, vp]
    L.drl_code_decode.argtypes = [i32, vp, i64, vp, vp]
    L.drl_policy_code_bytes.argtypes = [i32]
    L.drl_policy_code_bytes.restype = i32
    L.drl_grid_obs.argtypes = [P, S, vp, vp]
    L.drl_decode.argtypes = [P, S, vp, vp, vp, vp, vp, vp]
    L.drl_encode.argtypes = [P, S, vp, vp, vp, vp, vp, vp]
    L.drl_synth_actions.argtypes = [u64, u64, i64, i64, i32, vp, vp]
    L.drl_hbm_probe.argtypes = [vp, vp, i64, i32, vp]
    for f in ["drl_layout_query", "drl_reset", "drl_step", "drl_step_ex", "drl_rollout", "drl_refill", "drl_mt_get", "drl_mt_set", "drl_obs", "drl_grid_obs", "drl_decode", "drl_encode",
              "drl_synth_actions", "drl_obs_code", "drl_step_code", "drl_code_decode", "drl_hbm_probe"]:
        getattr(L, f).restype = ctypes.c_int
    if L.drl_abi_version() != DRL_ABI_VERSION:
        raise DroneRLError("libdronerl.so ABI version mismatch; rebuild it")
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        raise DroneRLError(f"{what} failed ({rc}): {lib().drl_last_error().decode()}")


def check_value(rc: int):
    """Parameter errors surface as ValueError, like the reference's spawn checks."""
    if rc != 0:
        raise ValueError(lib().drl_last_error().decode())
