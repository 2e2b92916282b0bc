#!/bin/bash
# rocprofv3 kernel-trace --stats of the bench headline command (sections off)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/benchprof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --sections "" --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
find "$OUT" -name "*kernel_trace.csv" -delete
exit 0
