#!/usr/bin/env python3
"""Per-kernel summary of tools/r03_pmc.sh's rocprofv3 passes -> OUT/summary.json.

HBM bytes per launch = FETCH_SIZE x 1024 x f_read + WRITE_SIZE x 1024 x f_write
(MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB from the L2's
memory-side request counters; gfx950 reports 1/2 of the bytes of wide 16-B
reads; other widths are uncalibrated -> calibrated here).  The coherent
kernels load 8-B words scattered over 64-B records and queue images and store
scattered 4- / 8-B words, so f_read is the calibration of 8-B loads (read8)
and f_write that of scattered 4-B stores (scatter4) from tools/calib/calib_traffic
in the same session; both are reported with the figure.
usage: r03_pmc_agg.py OUT_DIR WORKLOAD_KEY"""
import collections
import csv
import glob
import json
import os
import sys

CALIB = {"k_read<unsigned int>": "read4", "k_read<unsigned long>": "read8", "k_read16": "read16",
         "k_scatter4": "scatter4", "k_write16": "write16"}


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].strip()


def rows(d, pattern):
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        yield from csv.DictReader(open(f))


def main():
    d, key = sys.argv[1], sys.argv[2]
    res = {"workload_key": key, "kernels": collections.defaultdict(dict), "calibration": {}}
    for r in rows(os.path.join(d, "trace"), "*kernel_stats.csv"):
        res["kernels"][short(r["Name"])].update({"launches": int(r["Calls"]), "mean_us": float(r["AverageNs"]) / 1e3,
                                                 "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                                 "pct": float(r["Percentage"])})
    for p in ("fetch", "write", "sq"):
        acc = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, 0]))
        for r in rows(os.path.join(d, p), "*counter_collection.csv"):
            a = acc[short(r["Kernel_Name"])][r["Counter_Name"]]
            a[0] += float(r["Counter_Value"])
            a[1] += 1
        for k, c in acc.items():
            pm = res["kernels"][k].setdefault("pmc_per_launch", {})
            for n, (s, cnt) in c.items():
                pm[n] = s / cnt
    for p, ctr in (("calib_fetch", "FETCH_SIZE"), ("calib_write", "WRITE_SIZE")):
        try:
            nbytes = json.load(open(os.path.join(d, p + ".json")))["bytes_per_kernel"]
        except (OSError, ValueError, KeyError):
            continue
        acc = collections.defaultdict(float)
        for r in rows(os.path.join(d, p), "*counter_collection.csv"):
            k = short(r["Kernel_Name"])
            if k in CALIB and r["Counter_Name"] == ctr:
                acc[CALIB[k]] += float(r["Counter_Value"])
        for k, v in acc.items():
            if v > 0:
                res["calibration"][k] = nbytes / (v * 1024)
    cal = res["calibration"]
    fr, fw = cal.get("read8"), cal.get("scatter4")
    for k, v in res["kernels"].items():
        pm = v.get("pmc_per_launch", {})
        if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm and fr and fw:
            v["traffic_factors"] = {"read": fr, "write": fw, "source": "calib_traffic read8 / scatter4"}
            v["hbm_read_bytes"] = pm["FETCH_SIZE"] * 1024 * fr
            v["hbm_write_bytes"] = pm["WRITE_SIZE"] * 1024 * fw
            v["hbm_bytes"] = v["hbm_read_bytes"] + v["hbm_write_bytes"]
        if "SQ_WAVE_CYCLES" in pm and "SQ_WAIT_ANY" in pm and pm["SQ_WAVE_CYCLES"]:
            v["wait_fraction"] = pm["SQ_WAIT_ANY"] / pm["SQ_WAVE_CYCLES"]
    res["kernels"] = {k: v for k, v in res["kernels"].items() if k not in CALIB}
    json.dump(res, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(json.dumps({k: {x: v.get(x) for x in ("launches", "mean_us", "hbm_bytes", "wait_fraction")}
                      for k, v in res["kernels"].items() if v.get("launches", 0) > 100}, indent=1))


if __name__ == "__main__":
    main()
