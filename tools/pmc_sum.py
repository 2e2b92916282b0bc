#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc counter_collection.csv (kernels whose
name contains the filter), printed as JSON; the raw CSV can then be deleted.
usage: pmc_sum.py dir [filter]"""
import collections
import csv
import glob
import json
import sys

flt = sys.argv[2] if len(sys.argv) > 2 else "k_c_"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if flt not in k:
            continue
        k = k.split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
print(json.dumps({k: {"dispatches": len(disp[k]), **{c: x / len(disp[k]) for c, x in v.items()}} for k, v in agg.items()},
                 indent=1))
