#!/bin/bash
# Round-5 diagnostics of the headline step (GPU box): the diagnostics build's
# per-launch trace of the critical tile (tools/coh_trace.py) and the phase
# profile.  Trace dumps stay in /tmp on the box; only the summaries return.
set -e
export GG_LIB=variants/diag/libgraphite_gpu.so
OUT=${OUT:-gpurun_out/r05}
mkdir -p $OUT
GG_COH_TRACE=1200 GG_COH_TRACE_OUT=/tmp/tr timeout -k 10 300 python -u tools/coh_bench.py 1024 256 8 256 --hbh --no-oracle --warm > $OUT/diag_trace.log 2>&1
python tools/coh_trace.py /tmp/tr 200 > $OUT/diag_trace_summary.json
GG_COH_PROFILE=1 timeout -k 10 300 python -u tools/coh_bench.py 1024 256 8 256 --hbh --no-oracle > $OUT/diag_prof.log 2>&1
echo done
