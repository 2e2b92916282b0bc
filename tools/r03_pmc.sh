#!/bin/bash
# Round-3 rocprofv3 counters of the bench headline command (coherent, 1024
# tiles x 256 hotspot accesses, MSI + emesh_hop_by_hop, 8 logical shards; one
# uninstrumented run): a kernel-trace --stats pass, FETCH_SIZE and WRITE_SIZE
# in passes of their own (MI355X_MICROARCH.md §rocprofv3 PMC slots), an SQ
# pass, then the counter calibration of tools/calib/calib_traffic (known byte
# counts at 4 / 8 / 16-B widths: MI355X_MICROARCH.md §HBM "other access widths
# are uncalibrated").  Per-launch means: tools/r03_pmc_agg.py.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/${ROUND:-r03}/pmc"
mkdir -p "$OUT"
ARGS="--sections '' --steps 1 --warmup 0 --no-cpu-baseline --no-verify --no-kernel-profile ${PMC_ARGS:-}"
cd /tmp && export TMPDIR=/tmp
run() {   # name, rocprofv3 options...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --sections "" --steps 1 --warmup 0 --no-cpu-baseline --no-verify \
    --no-kernel-profile ${PMC_ARGS:-} > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run trace --kernel-trace --stats &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
run sq --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD || exit 1
CAL="$GRAFT_REPO_ROOT/tools/calib/calib_traffic"
for c in FETCH_SIZE:calib_fetch WRITE_SIZE:calib_write; do
  timeout -k 10 120 rocprofv3 --pmc ${c%%:*} -d "$OUT/${c##*:}" -o run --output-format csv -- "$CAL" 2048 \
    > "$OUT/${c##*:}.json" 2> "$OUT/${c##*:}.log" || exit 1
  echo "calibration ${c##*:} rc=0"
done
cd "$GRAFT_REPO_ROOT"
python3 tools/r03_pmc_agg.py "$OUT" "coherent_hop_by_hop_1024x256_k8" || exit 1
find "$OUT" -name "*counter_collection.csv" -delete
find "$OUT" -name "*kernel_trace.csv" -delete
exit 0
