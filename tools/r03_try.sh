#!/bin/bash
# round-3 quick GPU check: coherent parity on the shard kernel, then the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_coherent.py -x -v --timeout 120 --timeout-method thread \
  -k "${TESTK:-matches_oracle}" > gpurun_out/r03/t_${TAG:-a}.log 2>&1
rc=$?
tail -5 gpurun_out/r03/t_${TAG:-a}.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --sections "" --no-cpu-baseline --steps 3 --warmup 1 \
  > gpurun_out/r03/b_${TAG:-a}.json 2> gpurun_out/r03/b_${TAG:-a}.err
rc=$?
cat gpurun_out/r03/b_${TAG:-a}.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['bit_exact_checked'], d['coherent'])"
exit $rc
