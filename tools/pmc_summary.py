#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of tools/gpu_prof.sh + tools/gpu_pmc.sh into
one JSON (per kernel: launches, mean duration, HBM bytes per launch).

FETCH_SIZE / WRITE_SIZE are kilobytes (TCC_EA0_RDREQ/WRREQ based).  On gfx950
FETCH_SIZE reports half the bytes of 16-B-per-lane loads
(MI355X_MICROARCH.md §HBM), which is the load width of every kernel on the
path (dwordx4 record blocks, dwordx4 slot loads); it is doubled here.

usage: pmc_summary.py STATS_CSV PMC_DIR OUT_JSON [label [tiles per_tile]]
"""
import csv
import collections
import json
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].strip()


def main():
    stats_csv, pmc_dir, out = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    kern = {}
    for r in csv.DictReader(open(stats_csv)):
        kern[short(r["Name"])] = {"launches": int(r["Calls"]), "mean_ms": float(r["AverageNs"]) / 1e6,
                                  "total_pct": float(r["Percentage"])}
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("fetch", "write", "sq", "sq2"):
        try:
            rows = list(csv.DictReader(open("%s/%s/run_counter_collection.csv" % (pmc_dir, p))))
        except OSError:
            continue
        for r in rows:
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in pmc.items():
        d = kern.setdefault(k, {})
        per = {n: sum(v) / len(v) for n, v in c.items()}
        d["pmc_per_launch"] = per
        if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
            d["hbm_read_bytes"] = per["FETCH_SIZE"] * 1024 * 2
            d["hbm_write_bytes"] = per["WRITE_SIZE"] * 1024
            d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
    res = {"label": label, "fetch_size_correction": 2.0, "kernels": kern}
    if len(sys.argv) > 6:
        res["workload"] = {"tiles": int(sys.argv[5]), "per_tile": int(sys.argv[6])}
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
