#!/bin/bash
# Mode P A/B: the cache GPU tests, then bench's private sections with the
# 16-bit-tag stream kernel on (GG_STREAM_T16=1) and off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r05/modep}
mkdir -p $OUT
if [ "${TESTS:-tests/test_gpu_cache.py}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_cache.py} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for v in ${VARIANTS:-1 0}; do
  GG_STREAM_T16=$v timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-profile --sections private,private_16way $BENCH_ARGS > $OUT/bench_t16_$v.json 2> $OUT/bench_t16_$v.err || { tail -20 $OUT/bench_t16_$v.err; exit 1; }
  python - $OUT/bench_t16_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("private", "private_16way"):
    v = d.get(k, {})
    print("t16=%s" % sys.argv[2], k, {a: v.get(a) for a in ("value", "ms", "kernel_ms")}, (v.get("roofline") or {}).get("frac"))
PY
done
