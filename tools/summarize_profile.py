#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof) into profiles/.

Writes profiles/<tag>/kernel_stats.csv (rocprofv3 --kernel-trace --stats of
the bench command), profiles/<tag>/pmc_summary.json, and
profiles/pmc_<cfg>.json, which bench.py reads for `roofline.traffic`.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).  The x2 is
the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the
bytes of wide (16-B/lane) reads, and the bulk of this kernel's reads is the
16-B LDS-DMA ground staging.  WRITE_SIZE is exact for 16-B streaming stores.
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_wave(src: str):
    """Mean counter values per dispatch, and per wave (SQ_WAVES), over every
    pass under src/pmc*/ (tools/gpu.sh pmc)."""
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(src, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    w = m.get("SQ_WAVES", 1.0)
    for k in sorted(m):
        print(f"{k:24s} {m[k]:16.1f}   per-wave {m[k] / w:10.1f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-wave", default="", help="print per-wave PMC means of a tools/gpu.sh pmc directory")
    ap.add_argument("--src", default=os.path.join(REPO, "gpurun_out", "prof"))
    ap.add_argument("--tag", default="")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--kernel", default="drl_step_kernel")
    args = ap.parse_args()
    if args.per_wave:
        return per_wave(args.per_wave)
    out = os.path.join(REPO, "profiles", args.tag)
    os.makedirs(out, exist_ok=True)
    ks = os.path.join(args.src, "trace", "run_kernel_stats.csv")
    stats = {}
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(out, "kernel_stats.csv"))
        for r in csv.DictReader(open(ks)):
            if args.kernel in r["Name"]:
                stats = {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                         "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(args.src, "pmc*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if args.kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    pmc = {k: sum(v) / len(v) for k, v in agg.items()}
    summary = {"config": args.config, "envs": args.envs, "kernel_trace": stats, "pmc_mean_per_launch": pmc}
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        hbm = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024
        summary["hbm_bytes_per_launch"] = hbm
        summary["hbm_bytes_per_env_step"] = hbm / args.envs
        summary["read_bytes_per_env_step"] = 2 * pmc["FETCH_SIZE"] * 1024 / args.envs
        summary["write_bytes_per_env_step"] = pmc["WRITE_SIZE"] * 1024 / args.envs
        if stats:
            summary["hbm_gbs_at_trace_avg"] = hbm / stats["avg_ns"]
        summary["note"] = ("2*FETCH_SIZE+WRITE_SIZE in bytes (gfx950 FETCH_SIZE halving corrected, "
                           "MI355X_MICROARCH.md §HBM); PMC passes are separate runs of the same bench command")
        with open(os.path.join(REPO, "profiles", f"pmc_{args.config}.json"), "w") as f:
            json.dump(summary, f, indent=1)
    with open(os.path.join(out, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
