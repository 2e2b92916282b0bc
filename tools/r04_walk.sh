#!/bin/bash
# Round-4 walker iteration: coherent GPU tests (hop-by-hop), the headline
# timing, and (TRACE=1) the walker event trace.  Each GPU step under its own
# time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04/${TAG:-walk}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-400} python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread $TESTK \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 200 python -u tools/coh_bench.py 1024 256 8 256 --hbh --warm ${ORACLE:---no-oracle} > $OUT/bench.txt 2>&1 || { cat $OUT/bench.txt; exit 1; }
grep -v amdgpu.ids $OUT/bench.txt
if [ -n "$TRACE" ]; then
  # the trace hooks are in the diagnostics build only (tools/build_variant.sh diag -DGG_COH_DIAG=1)
  GG_LIB=variants/diag/libgraphite_gpu.so GG_COH_TRACE=600 GG_COH_TRACE_EV=300 GG_COH_TRACE_OUT=/tmp/ct timeout -k 10 200 python -u tools/coh_bench.py 1024 256 8 256 --hbh --no-oracle --no-timing > $OUT/trace_run.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/coh_trace_ev.py /tmp/ct > $OUT/trace_ev.json && timeout -k 10 200 python tools/coh_trace.py /tmp/ct 200 > $OUT/trace.json || exit 1
  cat $OUT/trace_ev.json; python3 -c "import json;d=json.load(open('$OUT/trace.json'));print(json.dumps({k:d[k] for k in ('per_launch_ns','walk_x','walk_y')}))"
fi
exit 0
