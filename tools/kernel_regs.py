#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of a HIP source (hipcc
-Rpass-analysis=kernel-resource-usage, device-only compile for gfx950).

    python tools/kernel_regs.py dronerl_amd/csrc/dronerl_qnet.hip [-k REGEX] [-D NAME=VAL ...]
"""
import argparse
import re
import subprocess
import sys

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("-k", default="", help="regex on the demangled kernel name")
ap.add_argument("-D", action="append", default=[])
a = ap.parse_args()
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", "include", "-c",
       "--offload-device-only", a.src, "-o", "/tmp/_kregs.o", "-Rpass-analysis=kernel-resource-usage"]
cmd += [f"-D{d}" for d in a.D]
r = subprocess.run(cmd, capture_output=True, text=True)
if r.returncode:
    print(r.stderr[-3000:])
    sys.exit(1)
rows, cur = [], None
for ln in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", ln)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
names = {}
if rows:
    dm = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True)
    names = dict(zip([r["name"] for r in rows], dm.stdout.splitlines()))
keys = ["VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "SGPRs Spill", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]",
        "ScratchSize [bytes/lane]"]
print(f"{'V':>4} {'A':>4} {'S':>4} {'Vsp':>4} {'Ssp':>4} {'occ':>3} {'LDS':>6} {'scr':>5}  kernel")
for row in rows:
    n = names.get(row["name"], row["name"])
    if a.k and not re.search(a.k, n):
        continue
    v = [row.get(k, "-") for k in keys]
    print(f"{v[0]:>4} {v[1]:>4} {v[2]:>4} {v[3]:>4} {v[4]:>4} {v[5]:>3} {v[6]:>6} {v[7]:>5}  {n[:110]}")
