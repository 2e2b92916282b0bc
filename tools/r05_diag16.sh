#!/bin/bash
# Diagnostics trace of the 16-tile persistent path (k_c_persist, hop counter)
set -e
export GG_LIB=variants/diag/libgraphite_gpu.so
OUT=${OUT:-gpurun_out/r05/diag16}
mkdir -p $OUT
GG_COH_TRACE=3000 GG_COH_TRACE_OUT=/tmp/tr16 timeout -k 10 300 python -u tools/coh_bench.py 16 20000 1 64 --no-oracle --warm > $OUT/diag_trace.log 2>&1
python tools/coh_trace.py /tmp/tr16 500 > $OUT/diag_trace_summary.json
timeout -k 10 300 python -u tools/coh_bench.py 16 20000 1 64 --no-oracle --warm > $OUT/plain.log 2>&1
echo done
