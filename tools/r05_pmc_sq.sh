#!/bin/bash
# Round-5: SQ / SQC counter passes of the headline's kernels (one --pmc run per pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05/${TAG:-sq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS SQ_INSTS_SALU SQ_INSTS_VALU SQ_IFETCH" \
            "SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/coh_bench.py 1024 256 8 256 --hbh --no-oracle > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
for i in 1 2; do python3 $GRAFT_REPO_ROOT/tools/pmc_kernel_avg.py $OUT/p$i/run_counter_collection.csv; done
