#!/bin/bash
# rocprofv3 of the bench headline workload (coherent, 1024 tiles x PER hotspot,
# MSI + emesh_hop_by_hop, 8 logical shards) through tools/coh_bench.py:
# one kernel-trace --stats pass, then counter passes of their own (FETCH_SIZE
# and WRITE_SIZE apart, MI355X_MICROARCH.md §rocprofv3 PMC slots).
# Output: gpurun_out/pmc/${PMC_NAME:-coh}/<pass>/run_*.csv
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc/${PMC_NAME:-coh}"
mkdir -p "$OUT"
ARGS=${PMC_ARGS:-1024 256 8 256 --hbh --no-oracle --no-timing}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/coh_bench.py" $ARGS > "$OUT/trace.log" 2>&1 || exit $?
echo "trace rc=0"
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/tools/coh_bench.py" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc pass $name rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass l2 TCC_HIT_sum TCC_MISS_sum &&
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS
rc=$?
python3 "$GRAFT_REPO_ROOT/tools/pmc_agg.py" "$OUT" ${PMC_KEY:-} || exit 1
find "$OUT" -name "*counter_collection.csv" -delete
find "$OUT" -name "*kernel_trace.csv" -delete
exit $rc
