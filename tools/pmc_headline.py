#!/usr/bin/env python3
"""Summarise a `tools/gpu.sh profile` run (rocprofv3 kernel trace + one --pmc
pass per counter group) for one kernel: average launch from the trace, the
counters per launch, HBM traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB; the x2
calibrated in profiles/r02_fetch_calib/) and the read roofline of SURVEY.md
section 8 D3 (R bytes per env-step).

python tools/pmc_headline.py gpurun_out/prof_TAG --kernel 'drl_step_kernel<8, drl::Geo<16, 8, 3, 1>, false, false, false>' \
    --envs 65536 --read-bytes 296 --out profiles/r06_final_c3
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--envs", type=int, required=True)
    ap.add_argument("--read-bytes", type=float, required=True, help="algorithmic read bytes per env-step (R)")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(os.path.join(args.prof, "trace", "run_kernel_stats.csv"))))
    k = [r for r in rows if args.kernel in r["Name"]]
    if len(k) != 1:
        raise SystemExit(f"{len(k)} kernels match {args.kernel!r}")
    avg_ns = float(k[0]["AverageNs"])
    per = defaultdict(list)  # counter -> per-launch values
    for f in sorted(glob.glob(os.path.join(args.prof, "pmc*", "run_counter_collection.csv"))):
        launches = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            if args.kernel not in r["Kernel_Name"]:
                continue
            launches[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for d in launches.values():
            for c, v in d.items():
                per[c].append(v)
    cpl = {c: sum(v) / len(v) for c, v in per.items()}
    waves = cpl.get("SQ_WAVES", 0.0)
    traffic = (2 * cpl["FETCH_SIZE"] + cpl["WRITE_SIZE"]) * 1024.0
    E = args.envs
    out = {
        "config": args.config,
        "kernel": k[0]["Name"],
        "avg_launch_ns_rocprof": avg_ns,
        "launches_traced": int(k[0]["Calls"]),
        "counters_per_launch": cpl,
        "traffic_bytes_per_launch": traffic,
        "traffic_bytes_per_env_step": traffic / E,
        "read_bytes_per_env_step": 2 * cpl["FETCH_SIZE"] * 1024.0 / E,
        "write_bytes_per_env_step": cpl["WRITE_SIZE"] * 1024.0 / E,
        "achieved_read_GBs": E * args.read_bytes / avg_ns,
        "frac_of_8TBs": E * args.read_bytes / avg_ns / 8000.0,
        "measured_traffic_TBs": traffic / avg_ns / 1e3,
        "note": "FETCH_SIZE and WRITE_SIZE in KiB per launch (rocprofv3 --pmc, one pass each), traffic = "
                "2*FETCH + WRITE (the x2 calibrated in profiles/r02_fetch_calib/); algorithmic read R = "
                f"{args.read_bytes:g} B per env-step (SURVEY.md section 8 D3); tools/pmc_headline.py",
    }
    os.makedirs(args.out, exist_ok=True)
    json.dump(out, open(os.path.join(args.out, "pmc_summary.json"), "w"), indent=1)
    with open(os.path.join(args.out, "pmc_summary.txt"), "w") as f:
        for c in sorted(cpl):
            f.write(f"{c:<28} {cpl[c]:>16.1f}   per-wave {cpl[c] / waves if waves else 0:>12.1f}\n")
    print(json.dumps({k2: v for k2, v in out.items() if k2 != "counters_per_launch"}, indent=1))


if __name__ == "__main__":
    main()
