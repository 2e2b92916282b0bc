#!/bin/bash
# Round-6 iocoom profile (bench.py's iocoom section, after the one-run
# headline every bench invocation starts with): a rocprofv3 kernel-trace
# --stats pass, then PMC passes of their own (tools/r06_fetch.sh): FETCH_SIZE,
# the SQ instruction / wait mix, and the per-type active / wait split.  Each
# pass under its own time limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r06/iocoom"
mkdir -p "$OUT"
ARGS="--sections iocoom --steps 1 --warmup 0 --no-cpu-baseline --no-verify --no-kernel-profile"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUT/trace.log" 2>&1 ) || { tail -5 "$OUT/trace.log"; exit 1; }
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/trace" -name "*kernel_trace.csv" -delete
grep -i "iocoom\|Name" "$OUT/kernel_stats.csv" | cut -c1-200
TAG=iocoom MINL=1 BENCH_ARGS="$ARGS" \
  PASSES="fetch:FETCH_SIZE|sq:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY|mix:SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
  bash tools/r06_fetch.sh | grep -i "iocoom" > "$OUT/pmc.txt" || exit 1
cat "$OUT/pmc.txt"
