#!/bin/bash
# A/B builds for kernel experiments: tools/build_variant.sh NAME "-DMACRO=..."
# -> exp/NAME/libgraphite_gpu.so (load with GG_LIB=exp/NAME/libgraphite_gpu.so)
set -e
cd "$(dirname "$0")/../graphite_amd/csrc"
NAME=$1; DEFS=$2
OUT=../../exp/$NAME; mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w -I../../include"
/opt/rocm/bin/hipcc $FLAGS $DEFS -c gg_cache.hip -o $OUT/gg_cache.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUT/gg_cache.o build/gg_capi.o build/gg_noc.o build/gg_coherent.o -o $OUT/libgraphite_gpu.so
rm -f $OUT/gg_cache.o
echo built $OUT/libgraphite_gpu.so
