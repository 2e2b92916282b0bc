#!/bin/bash
# A/B of library variants on the headline (tools/coh_bench.py, warm run, no
# oracle), REPS alternations: VARIANTS="base variants/x/libgraphite_gpu.so ..."
# (base = the tree's build).  BENCH_ARGS overrides the workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06/ab}
mkdir -p $OUT
for rep in $(seq ${REPS:-3}); do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then lib=""; else lib=$v; fi
    GG_LIB=$lib timeout -k 10 300 python -u tools/coh_bench.py ${BENCH_ARGS:-1024 256 8 256 --hbh} --warm --no-oracle > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
    echo "$v: $(grep gpu $OUT/ab.log)"
  done
done
