set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r05/wait}
COUNTERS=${COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $COUNTERS -d /tmp/pmcw -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/coh_bench.py 1024 256 8 256 --hbh --no-oracle > $GRAFT_REPO_ROOT/$OUT/p1.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/pmc_sum.py /tmp/pmcw > $GRAFT_REPO_ROOT/$OUT/summary.json
tail -2 $GRAFT_REPO_ROOT/$OUT/p1.log
