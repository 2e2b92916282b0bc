#!/bin/bash
# A/B builds of the private-cache unit: variants/<name>/libgraphite_gpu.so with
# extra -D defines on gg_cache.hip (the other objects from graphite_amd/csrc/build).
# Load one with GG_LIB=variants/<name>/libgraphite_gpu.so.  Experiments only.
set -e
cd "$(dirname "$0")/../graphite_amd/csrc"
name=$1; shift
mkdir -p ../../variants/$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w -I../../include "$@" \
  -c gg_cache.hip -o ../../variants/$name/gg_cache.o
objs=$(ls build/*.o | grep -v -e gg_cache.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs ../../variants/$name/gg_cache.o -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o ../../variants/$name/libgraphite_gpu.so
echo "variants/$name/libgraphite_gpu.so"
