#!/bin/bash
# Round-4 counters of the headline (coh_bench: 1024 tiles x 256 hotspot
# accesses, MSI + emesh_hop_by_hop, 8 logical shards): SQ instruction mix and
# instruction-cache passes (PASSES="sq ic"), per-launch means per kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r04/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {   # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/tools/coh_bench.py" 1024 256 8 256 --hbh --no-oracle --no-timing > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  [ $rc -eq 0 ] || return $rc
  f=$(find "$OUT/$name" -name "*counter_collection.csv" | head -1)
  python3 "$GRAFT_REPO_ROOT/tools/pmc_kernel_avg.py" "$f" > "$OUT/$name.json" && cat "$OUT/$name.json"
  rm -f "$f"
}
for p in ${PASSES:-sq ic}; do
  case $p in
    sq) run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_IFETCH || exit 1 ;;
    ic) run ic SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES || exit 1 ;;
  esac
done
exit 0
