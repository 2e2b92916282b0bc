#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of tools/gpu_prof.sh + tools/gpu_pmc.sh into
one JSON (per kernel: launches, mean duration, HBM bytes per launch).

FETCH_SIZE / WRITE_SIZE are kilobytes (TCC_EA0_RDREQ/WRREQ based).  On gfx950
FETCH_SIZE reports half the bytes of 16-B-per-lane loads (MI355X_MICROARCH.md
§HBM); other widths are uncalibrated there, so tools/calib/calib_traffic moves
known byte counts with the access widths of k_cache_stream (8-B + 4-B loads,
scattered 4-B stores) and the 16-B widths of the sharded kernels, and the
factors measured in that run (PMC_DIR/calib_fetch, PMC_DIR/calib_write) scale
each kernel's counters.  Without a calibration run, 2.0 / 1.0 (the guide's
16-B figures) are used.

usage: pmc_summary.py STATS_CSV PMC_DIR OUT_JSON [label [tiles per_tile]]
"""
import csv
import collections
import json
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].strip()


CALIB_KERNELS = {"k_read<unsigned int>": "read4", "k_read<unsigned long>": "read8", "k_read16": "read16",
                 "k_scatter4": "scatter4", "k_write16": "write16"}


def calibration(pmc_dir):
    """Byte / counter ratios per access pattern from the calib_traffic passes."""
    f = {}
    for p, ctr in (("calib_fetch", "FETCH_SIZE"), ("calib_write", "WRITE_SIZE")):
        try:
            rows = list(csv.DictReader(open("%s/%s/run_counter_collection.csv" % (pmc_dir, p))))
            nbytes = json.load(open("%s/%s.json" % (pmc_dir, p)))["bytes_per_kernel"]
        except (OSError, ValueError, KeyError):
            continue
        acc = collections.defaultdict(float)
        for r in rows:
            k = short(r["Kernel_Name"])
            if k in CALIB_KERNELS and r["Counter_Name"] == ctr:
                acc[CALIB_KERNELS[k]] += float(r["Counter_Value"])
        for k, v in acc.items():
            if v > 0:
                f[k] = nbytes / (v * 1024)
    return f


def factors(kernel, cal):
    """(read, write) byte factors of a kernel's FETCH_SIZE / WRITE_SIZE."""
    if kernel.startswith("k_cache_stream"):
        # 8-B address + 4-B metadata loads (bytes 2:1), scattered 4-B result stores
        if "read8" in cal and "read4" in cal and "scatter4" in cal:
            return 12.0 / (8.0 / cal["read8"] + 4.0 / cal["read4"]), cal["scatter4"]
    elif "read16" in cal and "write16" in cal:
        return cal["read16"], cal["write16"]
    return 2.0, 1.0


def main():
    stats_csv, pmc_dir, out = sys.argv[1:4]
    cal = calibration(pmc_dir)
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    kern = {}
    for r in csv.DictReader(open(stats_csv)):
        kern[short(r["Name"])] = {"launches": int(r["Calls"]), "mean_ms": float(r["AverageNs"]) / 1e6,
                                  "total_pct": float(r["Percentage"])}
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("fetch", "write", "l2", "sq", "sq2"):
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
            fr, fw = factors(k, cal)
            d["traffic_factors"] = {"read": fr, "write": fw}
            d["hbm_read_bytes"] = per["FETCH_SIZE"] * 1024 * fr
            d["hbm_write_bytes"] = per["WRITE_SIZE"] * 1024 * fw
            d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
    res = {"label": label, "calibration": cal, "kernels": {k: v for k, v in kern.items()
                                                            if k not in CALIB_KERNELS}}
    if len(sys.argv) > 6:
        res["workload"] = {"tiles": int(sys.argv[5]), "per_tile": int(sys.argv[6])}
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
