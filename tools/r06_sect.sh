#!/bin/bash
# Round-6 quick measurement: the headline bench line plus selected sections
# (SECTIONS, default fft,hop_counter,stress), no CPU baseline.  GG_LIB selects
# a variant library.  One GPU step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06/sect}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --no-cpu-baseline --sections "${SECTIONS-fft,hop_counter,stress}" $BENCH_ARGS \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('headline', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])
for k, v in d.get('sections', {}).items():
    if isinstance(v, dict): print(k, {a: v[a] for a in ('value', 'unit', 'ms') if a in v})"
