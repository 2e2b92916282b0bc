cd $GRAFT_REPO_ROOT
for t in 512 768 896 960 1024; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --tiles $t --per-tile 1048576 > gpurun_out/exp_$t.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/exp_$t.json')); k=d['roofline']['kernels']
print($t, {n: round(v['ms'],3) for n,v in k.items()})"
done
