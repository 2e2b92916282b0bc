#!/usr/bin/env python3
"""Aggregate rocprofv3 per-dispatch counter CSVs into per-kernel means (for
runs with tens of thousands of dispatches, whose raw CSVs are too large to
keep).  usage: pmc_agg.py OUT_DIR [WORKLOAD_KEY] -> OUT_DIR/agg.json

HBM bytes per launch = 2 x FETCH_SIZE (gfx950 reports half the bytes of
16-B-per-lane reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, in KiB units;
the coherent kernels mix 8-/16-B accesses, so the figure is an estimate of
the order of magnitude (calibration: tools/calib)."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].strip()


def main():
    d = sys.argv[1]
    res = {"kernels": collections.defaultdict(dict)}
    if len(sys.argv) > 2:
        res["workload_key"] = sys.argv[2]
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            res["kernels"][short(r["Name"])].update(
                {"launches": int(r["Calls"]), "mean_us": float(r["AverageNs"]) / 1e3,
                 "total_ms": float(r["TotalDurationNs"]) / 1e6, "pct": float(r["Percentage"])})
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, 0]))
        for r in csv.DictReader(open(f)):
            a = acc[short(r["Kernel_Name"])][r["Counter_Name"]]
            a[0] += float(r["Counter_Value"])
            a[1] += 1
        for k, c in acc.items():
            pm = res["kernels"][k].setdefault("pmc_per_launch", {})
            for n, (s, cnt) in c.items():
                pm[n] = s / cnt
    for k, v in res["kernels"].items():
        pm = v.get("pmc_per_launch", {})
        if "TCC_HIT_sum" in pm:
            h, m = pm["TCC_HIT_sum"], pm.get("TCC_MISS_sum", 0)
            v["l2_hit_rate"] = h / (h + m) if h + m else None
        if "FETCH_SIZE" in pm:
            v["fetch_bytes_per_launch_x2"] = pm["FETCH_SIZE"] * 1024 * 2   # MI355X_MICROARCH.md §HBM (16-B loads)
        if "WRITE_SIZE" in pm:
            v["write_bytes_per_launch"] = pm["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
            v["hbm_bytes"] = v["fetch_bytes_per_launch_x2"] + v["write_bytes_per_launch"]
    json.dump(res, open(os.path.join(d, "agg.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
