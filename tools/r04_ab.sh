#!/bin/bash
# A/B of library variants (variants/<name>/libgraphite_gpu.so) on the
# headline workload: 2 runs each (the first warms up), wall time printed.
# usage: VARIANTS="a b c" tools/r04_ab.sh   Diagnostics only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04/ab
for v in $VARIANTS; do
  GG_LIB=variants/$v/libgraphite_gpu.so timeout -k 10 120 python -u tools/coh_bench.py 1024 256 8 256 --hbh --warm --no-oracle \
    > gpurun_out/r04/ab/$v.txt 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/r04/ab/$v.txt; exit 1; }
  echo "$v: $(grep '^gpu' gpurun_out/r04/ab/$v.txt)"
done
