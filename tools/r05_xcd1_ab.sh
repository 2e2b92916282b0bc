#!/bin/bash
# configs[0] placement A/B: all persistent tiles on one XCD (GG_XCD1), with and
# without the grid barrier's release fence; the coherent reference fixtures
# (small meshes: the persistent path) on each variant first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r05/xcd1}
mkdir -p $OUT
for v in xcd1 xcd1nr; do
  GG_LIB=variants/$v/libgraphite_gpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_coherent.py -k "fixtures or fft" > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
done
VARIANTS="base variants/xcd1/libgraphite_gpu.so variants/xcd1nr/libgraphite_gpu.so base" OUT=$OUT bash tools/r05_persist_ab.sh
