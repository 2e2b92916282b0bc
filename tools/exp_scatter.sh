cd $GRAFT_REPO_ROOT
for m in 0 1 0 1; do
  GG_SCATTER_MODE=$m timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify > gpurun_out/exp_m$m.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/exp_m$m.json')); k=d['roofline']['kernels']
print('mode $m', d['value']/1e9, {n: round(v['ms'],3) for n,v in k.items()})"
done
