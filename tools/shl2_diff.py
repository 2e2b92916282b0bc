"""GPU vs oracle on a small shared-L2 case (diagnostics): the first records
whose access words differ, per tile.  usage: shl2_diff.py proto T N hot"""
import sys
import numpy as np
from graphite_amd import config as C
from oracle import pyoracle as po
from tests.gpu_util import torch_dev, to_dev, to_np

proto, T, N, hot = (int(x) for x in sys.argv[1:5])
N = N
cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_COUNTER, protocol=proto)
a, m, o = po.gen_trace(T, N, hot_lines=hot)
oc = po.OracleCoherent(cfg)
ref = oc.run(a, m, o)
torch = torch_dev()
from graphite_amd import backend as B
be = B.Backend(cfg)
out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
try:
    be.coherent_run(to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32), o, out)
    print("gpu ok")
except Exception as e:
    print("gpu error:", e)
torch.cuda.synchronize()
g = to_np(out, np.uint64)
for t in range(T):
    s, e = int(o[t]), int(o[t + 1])
    d = np.nonzero(g[s:e] != ref[s:e])[0]
    if len(d):
        i = s + int(d[0])
        print("tile %d first diff rec %d (#%d): gpu %d (lat %d lvl %d) oracle %d (lat %d lvl %d) addr %#x meta %#x" % (
            t, i, i - s, g[i], g[i] >> 2, g[i] & 3, ref[i], ref[i] >> 2, ref[i] & 3, a[i], m[i]))
        for j in range(max(s, i - 3), i + 1):
            print("   rec %d addr %#x meta %#x home %d gpu %d oracle %d" % (j, a[j], m[j], (a[j] >> 6) % T, g[j], ref[j]))
st, cc, ri = be.coherent_stats()
rs = oc.tile_stats()
names = C.TILE_STATS + ["x%d" % i for i in range(len(C.TILE_STATS), 32)]
for k in range(32):
    if not np.array_equal(st[:, k], rs[:, k]):
        print("stat %-22s gpu %s oracle %s" % (names[k], st[:, k], rs[:, k]))
print("cache gpu L2", cc[:, 1].sum(0), "\ncache orc L2", oc.cache_counters()[:, 1].sum(0))
