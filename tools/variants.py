#!/usr/bin/env python3
"""Build libdronerl variants with tuning macros (diagnostic; never the product).

python tools/variants.py d1:-DDRL_DRAWS_P8=1 d2:-DDRL_DRAWS_P8=2
writes tools/var_<name>.so; time them with tools/ab.py --lib tools/var_<name>.so.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from dronerl_amd import build as b  # noqa: E402


def build_one(spec):
    name, _, flags = spec.partition(":")
    out = os.path.join(REPO, "tools", f"var_{name}.so")
    cmd = [b.hipcc(), f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-I",
           os.path.join(REPO, "include"), "-o", out] + [f for f in flags.split(",") if f] + b.SOURCES
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(build_one, sys.argv[1:]):
            print(o)
