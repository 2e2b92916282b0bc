#!/bin/bash
# Mode P producer A/B: the cache GPU tests on the product build, then bench's
# private sections on each library of LIBS (product first and last).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r05/pm}
mkdir -p $OUT
if [ "${TESTS:-tests/test_gpu_cache.py}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_cache.py} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
i=0
for lib in ${LIBS:-graphite_amd/libgraphite_gpu.so variants/pm0/libgraphite_gpu.so graphite_amd/libgraphite_gpu.so}; do
  i=$((i+1))
  GG_LIB=$lib timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-profile --sections private,private_16way $BENCH_ARGS > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -20 $OUT/bench_$i.err; exit 1; }
  python - $OUT/bench_$i.json $lib <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("private", "private_16way"):
    v = d.get(k, {})
    print(sys.argv[2], k, {a: v.get(a) for a in ("value", "ms", "kernel_ms")}, (v.get("roofline") or {}).get("frac"))
PY
done
