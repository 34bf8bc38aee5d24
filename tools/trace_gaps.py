#!/usr/bin/env python3
"""Per-kernel mean durations and the idle gaps between consecutive kernels
from a rocprofv3 --kernel-trace csv (last N dispatches)."""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 600
rows = rows[-last:]
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:60]
    dur[name].append(e - s)
    if prev_end is not None:
        gap[name].append(s - prev_end)
    prev_end = e
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print(f"{len(rows)} dispatches over {span/1e3:.1f} us")
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    d, g = dur[k], gap.get(k, [0])
    print(f"{k:60s} n={len(d):4d} mean {sum(d)/len(d)/1e3:8.2f} us  total {sum(d)/1e3:9.1f} us  "
          f"gap-before mean {sum(g)/len(g)/1e3:6.2f} us")
