#!/bin/bash
# GPU round check: parity tests, then benches.  Each GPU step has its own time
# limit; a crash/timeout stops the script (pytest failures, rc=1, do not).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 900 python -m pytest $TESTS -m gpu -q --timeout 600 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for args in ${BENCH_ARGS:-"--steps 5 --warmup 2"}; do :; done
i=0
while IFS= read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  timeout -k 10 300 python bench.py $args > gpurun_out/bench_$i.json 2> gpurun_out/bench_$i.err; rc=$?
  echo "bench[$args] rc=$rc"; cat gpurun_out/bench_$i.json; tail -3 gpurun_out/bench_$i.err
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<< "${BENCH_LIST:---steps 5 --warmup 2}"
exit 0
