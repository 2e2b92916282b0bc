#!/bin/bash
# Round-6 iocoom A/B: the iocoom GPU tests on the tree's build, then bench.py's
# iocoom section alternating the tree's build and VARIANTS (.so paths, set inside the
# gpurun command), 3 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06/abio; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_iocoom.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2 3; do
for v in base ${VARIANTS:-}; do
  if [ $v = base ]; then l=""; else l=$v; fi
  GG_LIB=$l timeout -k 10 300 python -u bench.py --sections iocoom --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-profile > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 - $OUT/b.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
io = d["iocoom"]
print(sys.argv[2], round(io["value"] / 1e6, 1), "M instr/s", round(io["kernel_ms"], 3), "ms", "exact", io["bit_exact_checked"], flush=True)
PY
done; done
