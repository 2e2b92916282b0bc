#!/bin/bash
# NoC sections only (the headline shrunk to 16 accesses per tile): the bench
# line with GG_NOC_PROFILE=1 phase counters on stderr, then a rocprofv3
# kernel trace of an uninstrumented run.  TAG=name
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-noc}
mkdir -p $OUT
ARGS="--sections noc --per-tile 16 --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-profile $NOC_ARGS"
GG_NOC_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err \
  || { tail -30 $OUT/bench.err; exit 1; }
grep "gg_noc" $OUT/bench.err | tail -6
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["noc"]
for k in ("hop_counter", "hop_by_hop", "broadcast_tree"):
    print(k, d[k]["value"], d[k].get("bit_exact_checked"), d[k].get("seconds"))
PY
if [ -n "$PROF" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$GRAFT_REPO_ROOT/$OUT/prof.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err" \
    || { tail -20 "$GRAFT_REPO_ROOT/$OUT/prof.err"; exit 1; }
  cd "$GRAFT_REPO_ROOT"
  f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && head -8 "$f" | cut -c1-160
fi
exit 0
