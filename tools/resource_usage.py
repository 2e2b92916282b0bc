#!/usr/bin/env python3
"""Kernel resource usage of the product build: every unit compiled with
-Rpass-analysis=kernel-resource-usage (SGPRs, VGPRs, spills, scratch, LDS,
occupancy), as a markdown table.  usage: resource_usage.py [unit ...]"""
import concurrent.futures as cf
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "graphite_amd", "csrc")
UNITS = ["gg_cache", "gg_core", "gg_coh_step", "gg_coh_step_fast", "gg_coh_step_mosi", "gg_coh_step_shl2",
         "gg_coh_persist", "gg_coh_persist_lc", "gg_coh_walk"]
FIELDS = ["TotalSGPRs", "VGPRs", "SGPRs Spill", "VGPRs Spill", "ScratchSize [bytes/lane]", "LDS Size [bytes/block]",
          "Occupancy [waves/SIMD]"]


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return [re.sub(r"\(.*$", "", n.replace("(anonymous namespace)::", "")) for n in out]


def unit(u):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
           "-fno-fast-math", "-w", "-I../../include", "-Rpass-analysis=kernel-resource-usage", "-c", u + ".hip",
           "-o", "/tmp/ru_%s.o" % u]
    cache = "/tmp/ru_%s.txt" % u
    if os.environ.get("RU_REUSE") and os.path.exists(cache):
        err = open(cache).read()
    else:
        err = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr
        open(cache, "w").write(err)
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    names = demangle([r["name"] for r in rows])
    return [(u, n, r) for n, r in zip(names, rows)]


def main():
    units = sys.argv[1:] or UNITS
    with cf.ThreadPoolExecutor(6) as ex:
        res = list(ex.map(unit, units))
    print("| unit | kernel | SGPRs | VGPRs | SGPRs Spill | VGPRs Spill | ScratchSize B/lane | LDS Size B | Occupancy |")
    print("|---|---|---|---|---|---|---|---|---|")
    for rows in res:
        for u, n, r in rows:
            print("| %s | `%s` | %s |" % (u, n, " | ".join(r.get(f, "?") for f in FIELDS)))


if __name__ == "__main__":
    main()
