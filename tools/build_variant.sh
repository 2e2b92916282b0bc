#!/bin/bash
# A/B builds for GPU experiments: variants/<name>/libgraphite_gpu.so with extra
# -D defines on the coherent units (gg_coherent.hip, gg_coh_step.hip,
# gg_coh_persist.hip, gg_coh_walk.hip; the other objects from graphite_amd/csrc/build).
# Load one with GG_LIB=variants/<name>/libgraphite_gpu.so.  Diagnostics only.
set -e
cd "$(dirname "$0")/../graphite_amd/csrc"
name=$1; shift
mkdir -p ../../variants/$name
units="gg_coherent gg_coh_step gg_coh_step_fast gg_coh_step_mosi gg_coh_step_shl2 gg_coh_persist gg_coh_persist_lc gg_coh_walk"
for u in $units; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w -I../../include "$@" \
    -c $u.hip -o ../../variants/$name/$u.o &
done
wait
objs=$(ls build/*.o | grep -v -e gg_coherent.o -e gg_coh_)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs ../../variants/$name/gg_coh*.o -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o ../../variants/$name/libgraphite_gpu.so
echo "variants/$name/libgraphite_gpu.so"
