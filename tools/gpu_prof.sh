#!/bin/bash
# rocprofv3 kernel-trace summary of one bench configuration (no PMC here).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/${PROF_NAME:-run}" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" ${PROF_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > "$GRAFT_REPO_ROOT/gpurun_out/prof/${PROF_NAME:-run}.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof/${PROF_NAME:-run}.log"
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head
exit $rc
