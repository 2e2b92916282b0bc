#!/bin/bash
# instruction mix / issue-wait / icache counters of one command (default: the
# configs[0] FFT coherent run, tools/fft_prof.py), each pass a run of its own
# Output: gpurun_out/pmc/${PMC_NAME:-mix}/summary*.json (tools/pmc_agg.py)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc/${PMC_NAME:-mix}"
mkdir -p "$OUT"
CMD=${PMC_CMD:-"$GRAFT_REPO_ROOT/tools/fft_prof.py 14 1"}
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 $CMD > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc pass $name rc=$rc"
  return $rc
}
pass mix SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH &&
pass mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVES &&
pass ic SQC_ICACHE_HITS SQC_ICACHE_MISSES
rc=$?
python3 "$GRAFT_REPO_ROOT/tools/pmc_agg.py" "$OUT" ${PMC_KEY:-} || exit 1
find "$OUT" -name "*counter_collection.csv" -delete
find "$OUT" -name "*kernel_trace.csv" -delete
exit $rc
