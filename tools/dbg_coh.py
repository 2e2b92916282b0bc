import sys, time, numpy as np
sys.path.insert(0, '.')
import torch
from graphite_amd import config as C, backend as B, coherent as CO
from oracle import pyoracle as po
T, N, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
a, m, o = po.gen_trace(T, N, hot_lines=32)
cfg = C.default_config(T, num_shards=K)
be = B.Backend(cfg)
addr = torch.from_numpy(a.view(np.int64)).cuda(); meta = torch.from_numpy(m.view(np.int32)).cuda()
eng = B.CoherentEngine(be, addr, meta, o)
q = 0; t0 = time.time(); nq = 0
while True:
    st = eng.quantum(q); nq += 1
    buf, counts = eng.export(); n = int(counts.sum())
    if n: eng.import_(buf)
    if nq % 50 == 0 or time.time() - t0 > 20:
        print("q", q, "quanta", nq, st, "msgs", n, "t=%.1f" % (time.time() - t0), flush=True)
    nxt = CO.next_quantum(q, 1000000, n, st["active_tiles"], st["blocked_tiles"], st["min_next_ps"])
    if nxt is None: break
    q = nxt
    if time.time() - t0 > 60: print("giving up"); break
print("done quanta", nq, "%.2fs" % (time.time() - t0), be.coherent_stats()[2][:6], flush=True)
