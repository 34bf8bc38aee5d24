"""Build libdronerl.so (hand-written HIP for gfx950) in-tree with hipcc.

python -m dronerl_amd.build   (or dronerl_amd.build.build())
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdronerl.so")
SOURCES = [os.path.join(CSRC, "dronerl_kernels.hip"), os.path.join(CSRC, "dronerl_api.cpp"),
           os.path.join(CSRC, "dronerl_env.cpp"), os.path.join(CSRC, "dronerl_qnet.hip"),
           os.path.join(CSRC, "dronerl_qnet_api.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, "dronerl_internal.h"), os.path.join(REPO, "include", "dronerl.h")]
ARCH = os.environ.get("DRL_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in [os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"]:
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-I", os.path.join(REPO, "include"), "-o", LIB + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
