# stream-kernel time vs resident tiles (1 or 2 workgroups per CU) at 2^20 accesses/tile
cd $GRAFT_REPO_ROOT
for t in ${TILES:-256 512 1024}; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --coherent-tiles 0 --fft-m 0 --tiles $t --per-tile 1048576 > gpurun_out/exp_$t.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/exp_$t.json')); k=d['roofline']['kernels']
print($t, round(d['value']/1e9,2), {n: round(v['ms'],3) for n,v in k.items()})"
done
