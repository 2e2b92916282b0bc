#!/bin/bash
# Round-6 record: every GPU test, smoke(), the default bench line, then the
# headline's rocprofv3 passes (tools/r03_pmc.sh with ROUND=r06: kernel-trace
# --stats, FETCH_SIZE, WRITE_SIZE, SQ, the byte calibration).  Each GPU step
# under its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06/final}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 1000 python -u bench.py > $OUT/bench_full_sections.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_full_sections.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])
for k, v in d.get('sections', {}).items():
    if isinstance(v, dict): print(k, {a: v[a] for a in ('value', 'unit', 'ms') if a in v})"
[ -n "$SKIP_PMC" ] && exit 0
ROUND=r06 bash tools/r03_pmc.sh || exit 1
exit 0
