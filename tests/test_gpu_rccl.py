"""GPU: the coherent run over an RCCL communicator through the C ABI
(gg_coherent_run_ranks / gg_round_exchange), with the communicator of a
torch.distributed "nccl" (= RCCL) process group (ProcessGroupNCCL._comm_ptr).
A one-GPU box forms a one-rank communicator only (RCCL refuses two ranks on
one device); the exchange logic over several ranks is the same as
graphite_amd.coherent.run, covered by the gloo tests (tests/test_dist_gloo.py).
The run is repeated with one-record peer slots (GG_ROUND_SLOT=1) so that the
sized overflow round of gg_round_exchange runs too."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, %r)
from graphite_amd import config as C, backend as B, coherent as CO
from oracle import pyoracle as po
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d", world_size=1, rank=0)
torch.cuda.set_device(0)
T, N, K = 64, 200, 8
a, m, o = po.gen_trace(T, N, hot_lines=32)
addr = torch.from_numpy(a.view(np.int64)).cuda(); meta = torch.from_numpy(m.view(np.int32)).cuda()
res = []
for mode in ("rccl", "rccl_slot1", "single"):
    # rccl_slot1: one record per peer slot, so nearly every quantum takes the sized overflow round
    os.environ["GG_ROUND_SLOT"] = "1" if mode == "rccl_slot1" else "1024"
    cfg = C.default_config(T, num_shards=K, net_model=C.NET_EMESH_HOP_BY_HOP)
    be = B.Backend(cfg)
    out = torch.zeros(T * N, dtype=torch.int64, device="cuda")
    if mode.startswith("rccl"):
        CO.run_rccl(be, addr, meta, o, out)
    else:
        be.coherent_run(addr, meta, o, out)
    torch.cuda.synchronize()
    st, cc, ri = be.coherent_stats()
    res.append((out.cpu().numpy(), st, cc, be.noc_counters(), ri[:2]))
    be.close()
ok = all(np.array_equal(x, y) for r in res[1:] for x, y in zip(res[0], r))
oc = po.OracleCoherent(C.default_config(T, num_shards=K, net_model=C.NET_EMESH_HOP_BY_HOP))
ref = oc.run(a, m, o)
ok = ok and np.array_equal(res[0][0].view(np.uint64), ref) and np.array_equal(res[0][1], oc.tile_stats())
dist.destroy_process_group()
print("RCCL_RUN_OK" if ok else "RCCL_RUN_MISMATCH")
"""


def test_coherent_run_over_torch_rccl_communicator():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT % (ROOT, port)], capture_output=True, text=True, timeout=240,
                       env=env)
    assert "RCCL_RUN_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
