#!/bin/bash
# Round-5 GPU check: selected GPU tests, then bench.py with a chosen section
# list (SECTIONS) and no CPU leg; the JSON line into $OUT/bench.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r05/sect}
TESTS=${TESTS:-tests/test_gpu_coherent.py}
SECTIONS=${SECTIONS:-hop_counter,fft}
mkdir -p $OUT
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-profile --sections "$SECTIONS" $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"])
for k, v in d.get("sections", {}).items():
    if isinstance(v, dict): print(k, {a: v[a] for a in ("value", "unit", "ms") if a in v})
PY
