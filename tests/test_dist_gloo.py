"""The N>1 path with world_size 2 on CPU (gloo): disjoint tile shards per rank,
counter gather and max-reduced timing.  The per-rank compute here is the
oracle (the CPU stand-in for the GPU kernel), so the test covers the
distributed plumbing that bench.py uses, not the kernel."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, T, N, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from graphite_amd import dist as D
    from graphite_amd import config as C
    from oracle import pyoracle as po
    D.init("gloo")
    t0, t1 = D.tile_range(rank, T)
    oc = po.OracleCache(C.default_config(T))
    addr = np.concatenate([po.gen_uniform(t, 0, N, lines_log2=12)[0] for t in range(t0, t1)])
    meta = np.concatenate([po.gen_uniform(t, 0, N, lines_log2=12)[1] for t in range(t0, t1)])
    oc.run(addr, meta, np.arange(T + 1, dtype=np.uint64) * np.uint64(N))
    full = D.gather_tile_counters(oc.counters(), rank, world, "gloo")
    slowest = D.max_over_ranks(1.0 + rank, "gloo")
    D.barrier()
    np.save(os.path.join(outdir, "r%d.npy" % rank), full)
    with open(os.path.join(outdir, "r%d.txt" % rank), "w") as f:
        f.write("%r" % slowest)
    import torch.distributed as dist
    dist.destroy_process_group()


def test_two_rank_tile_sharding(tmp_path):
    world, T, N = 2, 3, 4000
    mp.spawn(_worker, args=(world, _free_port(), T, N, str(tmp_path)), nprocs=world, join=True)
    from graphite_amd import config as C
    from oracle import pyoracle as po
    oc = po.OracleCache(C.default_config(world * T))
    addr = np.concatenate([po.gen_uniform(t, 0, N, lines_log2=12)[0] for t in range(world * T)])
    meta = np.concatenate([po.gen_uniform(t, 0, N, lines_log2=12)[1] for t in range(world * T)])
    oc.run(addr, meta, np.arange(world * T + 1, dtype=np.uint64) * np.uint64(N))
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / ("r%d.npy" % r)), oc.counters())
        assert float(open(tmp_path / ("r%d.txt" % r)).read()) == float(world)


def _coherent_worker(rank, world, port, T, N, K, outdir, protocol=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from graphite_amd import dist as D
    from graphite_amd import config as C
    from graphite_amd import coherent as CO
    from oracle import pyoracle as po
    from tests.coherent_util import OracleEngine
    D.init("gloo")
    k0, k1 = CO.shard_range(rank, world, K)
    cfg = C.default_config(T, num_shards=K, shard_begin=k0, shard_end=k1, protocol=protocol)
    a, m, o = po.gen_trace(T, N, hot_lines=16)
    eng = OracleEngine(cfg, a, m, o)
    CO.run(eng, cfg.quantum_ns * 1000, K, world, rank, "gloo", "cpu")
    st = D.gather_tile_counters(eng.o.tile_stats(), 0, 1, "gloo")      # [T, S], zeros for foreign tiles
    import torch
    import torch.distributed as dist
    tt = torch.from_numpy(st.view(np.int64).copy())
    dist.all_reduce(tt)
    ot = torch.from_numpy(eng.out.view(np.int64).copy())
    dist.all_reduce(ot)
    if rank == 0:
        np.save(os.path.join(outdir, "stats.npy"), tt.numpy().view(np.uint64))
        np.save(os.path.join(outdir, "out.npy"), ot.numpy().view(np.uint64))
    dist.destroy_process_group()


@pytest.mark.parametrize("protocol", [0, 1])
def test_two_rank_coherent_exchange(tmp_path, protocol):
    """Mode C over 2 ranks x 2 logical shards each (gloo all-to-all of the
    cross-shard ShmemMsgs at every quantum boundary) == one process owning all
    4 shards: the schedule depends on the shard count, not the rank count.
    protocol 1: MOSI (INV_FLUSH_COMBINED_REQs carry their single receiver
    across ranks)."""
    world, T, N, K = 2, 16, 1200, 4
    mp.spawn(_coherent_worker, args=(world, _free_port(), T, N, K, str(tmp_path), protocol), nprocs=world, join=True)
    from graphite_amd import config as C
    from oracle import pyoracle as po
    a, m, o = po.gen_trace(T, N, hot_lines=16)
    oc = po.OracleCoherent(C.default_config(T, num_shards=K, protocol=protocol))
    out = oc.run(a, m, o)
    np.testing.assert_array_equal(np.load(tmp_path / "out.npy"), out)
    np.testing.assert_array_equal(np.load(tmp_path / "stats.npy"), oc.tile_stats())
