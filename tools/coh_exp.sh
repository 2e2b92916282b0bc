#!/bin/bash
# Coherent-section sweep: COH_CASES="tiles:net ..." (bench.py coherent section only, oracle-checked)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/coh
for a in ${COH_CASES:-"256:hop_counter 256:hop_by_hop 1024:hop_counter"}; do t=${a%%:*}; n=${a#*:}
  timeout -k 10 ${COH_TIMEOUT:-300} python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --fft-m 0 --per-tile 4096 --tiles 64 \
    --coherent-tiles $t --coherent-net $n ${COH_ARGS} > gpurun_out/coh/c_${t}_$n.json 2> gpurun_out/coh/c_${t}_$n.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/coh/c_${t}_$n.json'))['coherent']; print('$t $n', round(d['value']/1e6,3),'M/s', round(d['seconds'],3), 's steps', d['steps'], 'exact', d.get('bit_exact_checked'), 'cpu', round(d['cpu_baseline']['value']/1e6,3))"
done
