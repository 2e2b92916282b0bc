#!/bin/bash
# A/B of k_c_persist placements on configs[0] (bench section fft, no checks):
# VARIANTS="base variants/x/libgraphite_gpu.so ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r05/pab}
mkdir -p $OUT
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=""; else lib=$v; fi
  GG_LIB=$lib timeout -k 10 300 python -u bench.py --sections fft --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-profile --no-verify > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); f=d['fft']; print('$v', f['value'], f.get('seconds'))"
done
