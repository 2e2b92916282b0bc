#!/bin/bash
# configs[0] step diagnostics (GPU box): persistent vs per-step launches on a
# prefix of the FFT trace, then the diagnostics build's per-launch trace of the
# critical tile (tools/coh_trace.py); dumps stay in /tmp on the box.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/r05/fftdiag}
mkdir -p $OUT
timeout -k 10 300 python -u tools/fft_diag.py 20000 > $OUT/persist.log 2>&1
GG_COH_NO_PERSIST=1 timeout -k 10 300 python -u tools/fft_diag.py 20000 > $OUT/steps.log 2>&1
GG_LIB=variants/diag/libgraphite_gpu.so GG_COH_NO_PERSIST=1 GG_COH_TRACE=1500 GG_COH_TRACE_OUT=/tmp/ftr timeout -k 10 300 python -u tools/fft_diag.py 20000 > $OUT/diag.log 2>&1
python tools/coh_trace.py /tmp/ftr 100 > $OUT/trace_summary.json
cat $OUT/persist.log $OUT/steps.log $OUT/diag.log | grep fft
