#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06/abs; mkdir -p $OUT
for rep in 1 2; do
for v in base variants/ilp2/libgraphite_gpu.so; do
  if [ $v = base ]; then l=""; else l=$v; fi
  GG_LIB=$l timeout -k 10 400 python -u bench.py --sections iocoom,private,noc,hop_counter,stress,fft --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-profile > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 - $OUT/b.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = {"head": round(d["value"] / 1e3, 1)}
for k in ("iocoom", "private", "hop_counter", "stress", "fft"):
    r[k] = round(d[k]["value"] / 1e6, 2)
r["tree"] = round(d["noc"]["broadcast_tree"]["value"] / 1e6, 2); r["hbh"] = round(d["noc"]["hop_by_hop"]["value"] / 1e6, 2)
print(sys.argv[2].split("/")[1] if "/" in sys.argv[2] else "base", r, flush=True)
PY
done; done
