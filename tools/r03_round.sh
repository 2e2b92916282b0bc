#!/bin/bash
# Round-3 GPU check: selected GPU tests, the bench line (BENCH_ARGS), and a
# rocprofv3 kernel trace of the headline.  Every GPU step under its own time
# limit; the first failure ends the script.
#   TESTS="tests/test_gpu_coherent.py ..."  (empty: none)   TAG=name
#   BENCH=1 / PROF=1                                         BENCH_ARGS=...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-run}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread $TESTK \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_LIMIT:-600} python -u bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -30 $OUT/bench.err; exit 1; }
  python - "$OUT/bench.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms/step", d["ms_per_step"], "exact", d["bit_exact_checked"])
print("roofline", {k: d["roofline"].get(k) for k in ("kernel", "achieved", "frac", "kernel_avg_us", "launch_accesses")})
print("cpu", d.get("cpu_baseline", {}).get("value"), d.get("cpu_baseline", {}).get("cores"))
for k, v in d.items():
    if isinstance(v, dict) and ("value" in v or "error" in v) and k not in ("roofline", "cpu_baseline"):
        print(k, v.get("value"), v.get("bit_exact_checked"), v.get("error"))
EOF
fi
if [ -n "$PROF" ]; then
  cd /tmp
  timeout -k 10 ${PROF_LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --sections "" --no-cpu-baseline --no-verify --no-kernel-profile --steps 3 --warmup 1 $PROF_ARGS \
    > "$GRAFT_REPO_ROOT/$OUT/prof.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err" || { tail -20 "$GRAFT_REPO_ROOT/$OUT/prof.err"; exit 1; }
  cd "$GRAFT_REPO_ROOT"
  f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && head -8 "$f"
fi
exit 0
