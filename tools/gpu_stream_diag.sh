#!/bin/bash
# Streaming-replay diagnostics: hand-off counters (GG_STREAM_DEBUG) and one SQ
# PMC pass of the default bench workload.  Output under gpurun_out/diag/.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/diag"
mkdir -p "$OUT"
ARGS=${DIAG_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline --no-verify --coherent-tiles 0"}
GG_STREAM_DEBUG=1 timeout -k 10 200 python3 bench.py $ARGS > "$OUT/debug.json" 2> "$OUT/debug.err" || exit $?
grep gg_stream "$OUT/debug.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU \
  -d "$OUT/sq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUT/sq.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE \
  -d "$OUT/sq2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUT/sq2.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
for f in $(find "$OUT" -name "*counter_collection.csv"); do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_cache_stream" in r["Kernel_Name"] or "k_cache_replay" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        vg = r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"]
print(sys.argv[1].split("/")[-3], dict(acc), "vgpr/agpr/sgpr/lds", vg)
PY
done
