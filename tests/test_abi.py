"""CPU-side checks of the C ABI and host logic (no GPU compute)."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

from dronerl_amd import EnvParams, side_from_density
from dronerl_amd._native import EXPORTS, LIB_PATH, DrlLayout, lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dronerl.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:const\s+)?\w+\*?\s+\*?(drl_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    lib()
    fns = header_functions()
    assert fns == sorted(EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\s(drl_\w+)$", out, re.M))
    missing = [f for f in fns if f not in exported]
    assert not missing, missing
    assert lib().drl_abi_version() == 9


def test_library_is_gfx950_code_object():
    out = subprocess.run(["strings", LIB_PATH], capture_output=True, text=True, check=True)
    assert "amdgcn-amd-amdhsa--gfx950" in out.stdout


def test_no_oracle_in_product():
    """The product package never references the oracle."""
    pkg = os.path.join(REPO, "dronerl_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                txt = open(os.path.join(root, f)).read()
                assert not re.search(r"(import\s+oracle|from\s+oracle|liboracle|orc_\w+\()", txt), f


@pytest.mark.parametrize("n,density,side", [(4, 4 / 64, 8), (8, 8 / 256, 16), (16, 16 / 1024, 32),
                                            (32, 32 / 4096, 64), (1, 0.05, 5), (2, 0.05, 7), (6, 0.05, 11),
                                            (8, 0.05, 13), (3, 0.05, 8)])
def test_side_from_density_matches_reference_formula(n, density, side):
    assert side_from_density(n, density) == side
    assert lib().drl_side_from_density(n, density) == side


def test_layout_and_validation():
    L = EnvParams(n_drones=8, grid_size=16).layout()
    assert (L.cells, L.ground_stride, L.drone_stride, L.mt_stride, L.obs_window, L.obs_floats) == \
        (256, 128, 8, 1776, 7, 294)  # ground: two cells per byte (ABI 8)
    assert L.step_group_lanes == 8
    assert (L.cand_slots, L.refill_every) == (512, 48)  # 0.62 of a block's mean use, capped at 48 (round 4)
    L = EnvParams(n_drones=32, grid_size=64).layout()
    assert L.step_group_lanes in (32, 64) and L.step_lds_bytes <= 160 * 1024
    # 0.62 of a block's worth of candidates (156 pairs at power-of-two sides) at ~1.53 + 0.06 N per step
    assert L.refill_every == 28
    L = EnvParams(n_drones=1, grid_size=5).layout()
    assert L.ground_stride == 16  # 25 cells -> 13 bytes -> 16
    with pytest.raises(ValueError, match="Not enough positions"):
        EnvParams(n_drones=8, grid_size=8).layout()  # 80 objects on 64 cells
    with pytest.raises(ValueError):
        EnvParams(n_drones=65, grid_size=64).layout()
    with pytest.raises(ValueError):
        EnvParams(n_drones=4, grid_size=8, window_radius=0).layout()
    with pytest.raises(ValueError):
        EnvParams(n_drones=4, grid_size=8, discharge=-1).layout()


def test_null_and_empty_calls_fail_cleanly():
    from dronerl_amd._native import DrlState
    p = EnvParams(n_drones=8, grid_size=16).to_c()
    s = DrlState(None, None, None, None, 0)
    assert lib().drl_step(ctypes.byref(p), ctypes.byref(s), None, None, None, None, 0, None, None) == 0
    s = DrlState(None, None, None, None, 10)
    assert lib().drl_step(ctypes.byref(p), ctypes.byref(s), None, None, None, None, 0, None, None) != 0
    assert b"NULL" in lib().drl_last_error()


def test_from_torch_config():
    p = EnvParams.from_torch_config({'n_drones': 6})
    assert p.side == 11 and p.charge_reward == -0.1
    assert isinstance(DrlLayout(), ctypes.Structure)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device path")
def test_env_handle_without_device_fails_cleanly():
    from dronerl_amd._native import DroneRLError
    from dronerl_amd.handle import DrlEnvHandle
    from dronerl_amd.params import EnvParams
    with pytest.raises(DroneRLError, match="device"):
        DrlEnvHandle(EnvParams(n_drones=4, grid_size=8), 4)


@pytest.mark.parametrize("field,value", [("charge", 7.5), ("discharge", 2.5), ("packets_factor", 1.5),
                                         ("skyscrapers_factor", 0.5)])
def test_fractional_integer_params_rejected(field, value):
    """The C ABI does charge / factor arithmetic on integers: a fraction is an
    error, not a silent truncation (env.py:79-82 uses Python numbers)."""
    p = EnvParams(n_drones=4, grid_size=8).replace(**{field: value})
    with pytest.raises(ValueError, match="integer"):
        p.to_c()
    EnvParams(n_drones=4, grid_size=8).replace(**{field: float(int(value) + 1)}).to_c()  # integral floats are fine


def test_replay_add_rejects_short_rows():
    """drl_replay_add validates before any device work (no GPU needed)."""
    from dronerl_amd.dqn import DrlReplay, _bind
    L = _bind(lib())
    r = DrlReplay(16, 294, 8, 8, 8, 8, 8)
    vp = ctypes.c_void_p
    args = lambda stride: (ctypes.byref(r), 0, 4, vp(8), stride, vp(8), 294, vp(8), 1, vp(8), 1, vp(8), 1, None)  # noqa
    assert L.drl_replay_add(*args(292)) != 0
    assert b"obs_floats" in L.drl_last_error()
    r0 = DrlReplay(16, 294, 8, 8, 8, 8, 8)
    assert L.drl_replay_add(ctypes.byref(r0), 0, 4, vp(8), 294, vp(8), 294, vp(8), 0, vp(8), 1, vp(8), 1, None) != 0
    assert b"strides" in L.drl_last_error()


def test_step_code_replay_validates_before_device_work():
    """drl_step_code_replay (the step + add_many of its drone-0 transitions)
    checks its ring and buffers before any device work (no GPU needed)."""
    from dronerl_amd._native import DrlState
    from dronerl_amd.dqn import DrlReplay, _bind
    L = _bind(lib())
    vp = ctypes.c_void_p
    p = EnvParams(n_drones=8, grid_size=16).to_c()  # radius 3: 128-B code rows = 32 words
    s = DrlState(vp(64), vp(64), vp(64), vp(64), 10)
    good = DrlReplay(100, 32, 64, 64, 64, 64, 64)

    def call(r, code=vp(1024), prev=vp(2048), cursor=0):
        return L.drl_step_code_replay(ctypes.byref(p), ctypes.byref(s), vp(64), vp(64), vp(64), code, prev,
                                      None if r is None else ctypes.byref(r), cursor, None, 0, None)
    assert call(good, prev=None) != 0 and b"code_prev" in L.drl_last_error()
    assert call(good, prev=vp(1024)) != 0 and b"another buffer" in L.drl_last_error()
    assert call(good, prev=vp(2056)) != 0 and b"16-byte" in L.drl_last_error()
    assert call(None) != 0 and b"replay is NULL" in L.drl_last_error()
    assert call(DrlReplay(100, 32, 64, 64, 64, 64, None)) != 0 and b"NULL" in L.drl_last_error()
    assert call(DrlReplay(100, 32, 72, 64, 64, 64, 64)) != 0 and b"aligned" in L.drl_last_error()
    assert call(good, cursor=-1) != 0 and b"cursor" in L.drl_last_error()
    assert call(DrlReplay(100, 294, 64, 64, 64, 64, 64)) != 0 and b"obs_floats" in L.drl_last_error()

    # drl_step_code_replay_synth (drone indices >= 1 drawn in the step): the same checks, and env_offset >= 0
    def call_synth(r, prev=vp(2048), env_offset=0):
        return L.drl_step_code_replay_synth(ctypes.byref(p), ctypes.byref(s), vp(64), vp(64), vp(64), vp(1024), prev,
                                            None if r is None else ctypes.byref(r), 0, 3, 4, env_offset, None, 0, None)
    assert call_synth(good, env_offset=-1) != 0 and b"env_offset" in L.drl_last_error()
    assert call_synth(good, prev=vp(1024)) != 0 and b"another buffer" in L.drl_last_error()
    assert call_synth(None) != 0 and b"replay is NULL" in L.drl_last_error()


@pytest.mark.parametrize("val,ok", [("0", False), ("-3", False), ("x", False), ("", False), ("7", True)])
def test_refill_cadence_override_must_be_positive(monkeypatch, val, ok):
    """DRL_REFILL_EVERY=0 used to mean "after every step" in C but
    "never" for the Python env's refill_every; non-positive or non-numeric
    overrides are now refused."""
    monkeypatch.setenv("DRL_REFILL_EVERY", val)
    p = EnvParams(n_drones=8, grid_size=16)
    if ok:
        assert p.layout().refill_every == 7
    else:
        with pytest.raises(ValueError, match="DRL_REFILL_EVERY"):
            p.layout()


def test_ground_pack_roundtrip():
    """The packed-nibble ground (ABI 8) round-trips through env.py's host-side
    conversions for odd and even cell counts."""
    from dronerl_amd.env import pack_ground, unpack_ground
    g = torch.Generator().manual_seed(0)
    for side in (5, 8, 13, 16, 64):
        E = 7
        ground = torch.randint(0, 6, (E, side * side), dtype=torch.uint8, generator=g)
        stride = ((side * side + 1) // 2 + 15) // 16 * 16
        packed = pack_ground(ground, stride)
        assert packed.shape == (E, stride)
        assert torch.equal(packed[:, 0], ground[:, 0] | (ground[:, 1] << 4))
        assert torch.equal(unpack_ground(packed, side).reshape(E, -1), ground)
        assert not packed[:, (side * side + 1) // 2:].any()  # zero padding
    with pytest.raises(ValueError):
        pack_ground(torch.full((1, 4), 16, dtype=torch.uint8), 16)


# Every __global__ kernel of the product library and the -m gpu test that
# launches it (no shipped kernel without a GPU test).  A new
# kernel must be listed here with its test; a listed test must exist.
KERNEL_TESTS = {
    "drl_step_kernel": "test_gpu_parity.py::test_rollout_matches_oracle",
    "drl_rollout_kernel": "test_gpu_parity.py::test_rollout_equals_steps",
    "drl_obs_kernel": "test_gpu_parity.py::test_obs_variants",
    "drl_grid_obs_kernel": "test_gpu_parity.py::test_grid_obs_vs_oracle_state_and_compat_gridview",
    "drl_reset_wave_kernel": "test_gpu_parity.py::test_reset_matches_oracle",  # every WPB instance: RESET_KERNELS
    "drl_reset_kernel": "test_gpu_parity.py::test_reset_matches_oracle",       # the "lane" variant
    "drl_refill_list_kernel": "test_gpu_parity.py::test_candidate_ring_cadence_matches_oracle",
    "drl_refill_kernel": "test_gpu_parity.py::test_candidate_ring_cadence_matches_oracle",  # refill_kernel "wave"
    "drl_mt_get_kernel": "test_gpu_parity.py::test_candidate_ring_holds_the_streams_randint_pairs",
    "drl_mt_set_kernel": "test_gpu_parity.py::test_reference_trajectory_on_gpu",
    "drl_decode_kernel": "test_gpu_parity.py::test_reset_matches_oracle",
    "drl_encode_kernel": "test_gpu_validation.py::test_full_grid_respawn_raises_no_free_cell",
    "drl_ground_pack_kernel": "test_gpu_validation.py::test_handle_set_state_flags_bad_ground_code",
    "drl_ground_unpack_kernel": "test_gpu_validation.py::test_handle_set_state_clamps_and_flags_bad_mt_index",
    "drl_synth_actions_kernel": "test_dqn.py::test_qnet_act_synth_equals_synth_then_act",
    "drl_code_decode_kernel": "test_policy_code.py::test_code_decode_and_get_code",
    "drl_hbm_probe_kernel": "test_gpu_validation.py::test_hbm_probe_copies_and_reads",
    "drl_qnet_pack_kernel": "test_dqn.py::test_qnet_load_repacks",
    "drl_qnet_act_kernel": "test_dqn.py::test_qnet_greedy_matches_torch_reference",   # bf16
    "drl_qnet_act_f32_kernel": "test_dqn.py::test_qnet_f32_matches_fp32_forward",
    "drl_qnet_act_code_kernel": "test_policy_code.py::test_qnet_act_code_matches_f32_forward",   # other nets
    "drl_qnet_act_code2_kernel": "test_policy_code.py::test_qnet_act_code_matches_f32_forward",  # kernel="code2"
    "drl_qnet_act_code4_kernel": "test_policy_code.py::test_qnet_act_code_matches_f32_forward",  # benchmark net
    "drl_replay_add16_kernel": "test_policy_code.py::test_code_replay_buffer_samples_decode_to_obs_buffer",
    "drl_replay_add_kernel": "test_dqn.py::test_replay_add_many_matches_sequential_add",
    "drl_replay_add_rows_kernel": "test_dqn.py::test_replay_add_two_float_rows",
    "drl_dqn_train_kernel": "test_dqn_learner.py::test_learner_matches_oracle_bit_exact",
    "drl_dqn_init_kernel": "test_dqn_learner.py::test_learner_matches_oracle_bit_exact",
    "drl_dqn_sample_kernel": "test_dqn_learner.py::test_sample_slots_are_the_learners_draws",
}


def test_every_kernel_has_a_gpu_test():
    import glob
    import re
    csrc = os.path.join(REPO, "dronerl_amd", "csrc")
    found = set()
    for f in glob.glob(os.path.join(csrc, "*.hip")):
        src = open(f).read()
        for m in re.finditer(r"__global__", src):
            k = re.search(r"\b(drl_[a-z0-9_]+_kernel)\s*\(", src[m.end():m.end() + 300])
            if k:
                found.add(k.group(1))
    assert found == set(KERNEL_TESTS), (sorted(found - set(KERNEL_TESTS)), sorted(set(KERNEL_TESTS) - found))
    for kern, ref in KERNEL_TESTS.items():
        fname, test = ref.split("::")
        text = open(os.path.join(REPO, "tests", fname)).read()
        assert re.search(rf"^def {test}\(", text, re.M), (kern, ref)
        assert "gpu" in text, ref
