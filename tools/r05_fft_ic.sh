#!/bin/bash
# configs[0] instructions per simulated access: one SQ
# PMC pass over the persistent FFT prefix run (tools/fft_diag.py, the first
# 20 000 records of each of the 16 tiles), instruction counts per kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05/fftic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY -d $OUT/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fft_diag.py 20000 > $OUT/run.log 2>&1
rc=$?
tail -2 $OUT/run.log
exit $rc
