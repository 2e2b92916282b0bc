#!/bin/bash
# Round-5 GPU check after a kernel change: the selected GPU tests, then the
# headline through tools/coh_bench.py (warm run, checked against the oracle).
# Each GPU step under its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r05/check}
TESTS=${TESTS:-tests/test_gpu_coherent.py}
mkdir -p $OUT
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for i in 1 2; do
  timeout -k 10 300 python -u tools/coh_bench.py 1024 256 8 256 --hbh --warm $BENCH_ARGS > $OUT/bench$i.log 2>&1 || { tail $OUT/bench$i.log; exit 1; }
  grep -v amdgpu.ids $OUT/bench$i.log
  BENCH_ARGS="$BENCH_ARGS --no-oracle"
done
exit 0
