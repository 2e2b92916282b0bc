# A/B of exp/<variant>/libgraphite_gpu.so builds on the default bench workload
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-base}; do
  GG_LIB=$GRAFT_REPO_ROOT/exp/$v/libgraphite_gpu.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --coherent-tiles 0 --fft-m 0 ${BENCH_ARGS} > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); k=d['roofline']['kernels']
print('$v', round(d['value']/1e9,2), d.get('bit_exact_checked'), {n: round(v['ms'],3) for n,v in k.items()})"
done
