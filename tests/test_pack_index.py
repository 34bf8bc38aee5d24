"""The learner's parameter -> packed-element map (drl::qnet_pack_elem, used by
drl_dqn_update_kernel to refresh the act kernels' image) is the exact inverse
of drl_qnet_pack's element -> parameter map (drl::qnet_pack_slot), for code
and observation nets: host code from dronerl_internal.h, compiled here."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_pack_index_round_trip(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    exe = str(tmp_path / "pack_index_check")
    subprocess.run([hipcc, "-O1", "-std=c++17", "-I", os.path.join(os.path.dirname(HERE), "include"), "-o", exe,
                    os.path.join(HERE, "native", "pack_index_check.cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout
