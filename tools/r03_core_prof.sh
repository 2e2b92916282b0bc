#!/bin/bash
# rocprofv3 kernel trace of the bench's core_model section (k_core_model on
# 1024 tiles x 2^18 records; the headline runs once before it, shrunk).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r03/core"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --sections core_model --per-tile 16 --steps 1 --warmup 0 --no-cpu-baseline \
  --no-verify --no-kernel-profile > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
find "$OUT" -name "*kernel_trace.csv" -delete
exit 0
