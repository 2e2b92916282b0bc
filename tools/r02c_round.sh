#!/bin/bash
# Round-2 (third session) GPU call: the whole GPU test suite, the default
# bench line, and the rocprofv3 kernel trace of the NoC section (the
# broadcast-tree walk k_tree_win beside the unicast stage kernels).  Every
# GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/$OUT/nocprof" -o noc -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --sections noc --no-cpu-baseline --no-verify \
    > "$GRAFT_REPO_ROOT/$OUT/noc_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/noc_bench.err" )
rc=$?; echo "noc prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find "$OUT/nocprof" -name "*kernel_trace.csv" -delete
exit 0
