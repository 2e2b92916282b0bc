#!/bin/bash
# rocprofv3 PMC passes of one bench configuration (counters only: no sys/runtime
# traces).  FETCH_SIZE and WRITE_SIZE need separate passes on gfx950
# (MI355X_MICROARCH.md §rocprofv3 PMC slots); the SQ pass gives the issue/wait
# breakdown of the replay.  Output: gpurun_out/pmc/$PMC_NAME/<pass>/...
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc/${PMC_NAME:-run}"
mkdir -p "$OUT"
ARGS=${PMC_ARGS:---steps 1 --warmup 0 --no-cpu-baseline --no-verify}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/../counters_list.txt" 2>&1 || exit $?
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc pass $name rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU &&
pass sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
rc=$?
[ $rc -ne 0 ] && exit $rc
# counter calibration: known byte counts at the access widths of the path
CAL="$GRAFT_REPO_ROOT/tools/calib/calib_traffic"
for c in FETCH_SIZE:calib_fetch WRITE_SIZE:calib_write; do
  timeout -k 10 120 rocprofv3 --pmc ${c%%:*} -d "$OUT/${c##*:}" -o run --output-format csv -- "$CAL" 2048 \
    > "$OUT/${c##*:}.json" 2> "$OUT/${c##*:}.log" || exit $?
  echo "calibration ${c##*:} rc=0"
done
find "$OUT" -name "*counter_collection*" | head -20
exit 0
