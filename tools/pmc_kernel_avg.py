#!/usr/bin/env python3
"""Per-kernel average of every PMC counter in a rocprofv3 counter_collection
CSV (streams the file; prints one JSON line per kernel with at least
MIN_LAUNCHES launches, default 10).  usage: pmc_kernel_avg.py CSV [MIN_LAUNCHES]"""
import collections
import csv
import json
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"][:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    lim = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    for k, v in agg.items():
        n = len(disp[k])
        if n >= lim:
            print(json.dumps({"kernel": k, "launches": n, "per_launch": {c: round(x / n, 1) for c, x in sorted(v.items())}}))


if __name__ == "__main__":
    main()
