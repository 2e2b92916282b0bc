#!/bin/bash
# instruction-fetch / instruction-mix counters of the headline coherent run
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc/${PMC_NAME:-ic}"
mkdir -p "$OUT"
ARGS=${PMC_ARGS:-1024 256 8 256 --hbh --no-oracle --no-timing}
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/tools/coh_bench.py" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc pass $name rc=$rc"
  return $rc
}
pass ic SQC_ICACHE_HITS SQC_ICACHE_MISSES &&
pass mix SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH
rc=$?
python3 "$GRAFT_REPO_ROOT/tools/pmc_agg.py" "$OUT" || exit 1
find "$OUT" -name "*counter_collection.csv" -delete
exit $rc
