"""GPU parity of the coherent mode (Mode C) through the C ABI: the HIP path
(graphite_amd/csrc/gg_coherent.hip) against the C oracle
(oracle/gg_coherent.inc) on the same seeded traces — per-access level and
latency, per-tile statistics, L1-D/L2 counters and NoC counters, bit-exact."""
import numpy as np
import pytest

from graphite_amd import config as C
from tests.coherent_util import check_invariants
from tests.gpu_util import torch_dev, to_dev, to_np

pytestmark = pytest.mark.gpu


def _gpu_run(cfg, a, m, o):
    torch = torch_dev()
    from graphite_amd import backend as B
    be = B.Backend(cfg)
    addr, meta = to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32)
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_run(addr, meta, o, out)
    torch.cuda.synchronize()
    st, cc, ri = be.coherent_stats()
    return to_np(out, np.uint64), st, cc, be.noc_counters(), ri


def _oracle_run(cfg, a, m, o):
    from oracle import pyoracle as po
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    return out, oc.tile_stats(), oc.cache_counters(), oc.net_counters(), oc.run_info()


def _compare(cfg, a, m, o):
    g = _gpu_run(cfg, a, m, o)
    r = _oracle_run(cfg, a, m, o)
    for name, x, y in zip(("access words", "tile stats", "cache counters", "noc counters"), g[:4], r[:4]):
        if not np.array_equal(x, y):
            d = np.argwhere(np.asarray(x) != np.asarray(y))
            raise AssertionError("%s differ at %d places, first %s: gpu %s oracle %s"
                                 % (name, len(d), d[0], np.asarray(x)[tuple(d[0])], np.asarray(y)[tuple(d[0])]))
    for k in ("steps", "net_msgs", "self_msgs", "boundary_msgs"):
        i = C.RUN_INFO.index(k)
        assert g[4][i] == r[4][i], (k, g[4][i], r[4][i])
    check_invariants(g[1], g[2], g[0], o, per_tile_expected=int(o[1] - o[0]))
    return g


@pytest.mark.parametrize("T,N,hot,K,net", [
    (16, 3000, 0, 1, C.NET_EMESH_HOP_COUNTER),      # private: no sharing
    (16, 2500, 64, 1, C.NET_EMESH_HOP_COUNTER),     # configs[2]-style hotspot, 16 tiles
    (16, 2000, 8, 1, C.NET_MAGIC),
    (64, 1200, 64, 1, C.NET_EMESH_HOP_COUNTER),
    (64, 1000, 32, 8, C.NET_EMESH_HOP_COUNTER),     # 8 logical shards, quantum-boundary delivery
    (256, 300, 64, 4, C.NET_EMESH_HOP_COUNTER),
    (16, 1500, 8, 1, C.NET_EMESH_HOP_BY_HOP),      # configs[2]: router / link contention
    (64, 700, 64, 1, C.NET_EMESH_HOP_BY_HOP),
    (256, 200, 64, 1, C.NET_EMESH_HOP_BY_HOP),
    # hop-by-hop across logical shards: packets held at a shard's edge router
    # continue in the next quantum (2-D block shards, hop_by_hop.cc:367-433)
    (16, 1200, 8, 2, C.NET_EMESH_HOP_BY_HOP),
    (64, 600, 32, 8, C.NET_EMESH_HOP_BY_HOP),
    (256, 150, 64, 4, C.NET_EMESH_HOP_BY_HOP),
    (256, 150, 64, 8, C.NET_EMESH_HOP_BY_HOP),
    (1024, 48, 256, 8, C.NET_EMESH_HOP_BY_HOP),     # configs[3]: 1024 tiles x 8 shards (reduced per-tile length)
    (1024, 64, 256, 8, C.NET_EMESH_HOP_COUNTER),
])
def test_coherent_matches_oracle(T, N, hot, K, net):
    from oracle import pyoracle as po
    cfg = C.default_config(T, num_shards=K, net_model=net)
    a, m, o = po.gen_trace(T, N, hot_lines=hot)
    _compare(cfg, a, m, o)


@pytest.mark.parametrize("T,N,hot,K,net", [(16, 1500, 8, 1, C.NET_EMESH_HOP_BY_HOP),
                                            (64, 600, 32, 8, C.NET_EMESH_HOP_BY_HOP),
                                            (64, 1000, 32, 8, C.NET_EMESH_HOP_COUNTER)])
@pytest.mark.parametrize("env", ["GG_COH_NO_PERSIST", "GG_COH_NO_LDS_CACHE"])
def test_coherent_small_mesh_launch_path(T, N, hot, K, net, env, monkeypatch):
    """Small meshes run the loop in persistent launches (k_c_persist, grid
    barriers; closed-form networks keep the cache state in LDS);
    GG_COH_NO_PERSIST=1 forces the per-step launches, GG_COH_NO_LDS_CACHE=1
    the persistent kernel on the HBM cache arrays: all bit-exact."""
    from oracle import pyoracle as po
    monkeypatch.setenv(env, "1")
    cfg = C.default_config(T, num_shards=K, net_model=net)
    a, m, o = po.gen_trace(T, N, hot_lines=hot)
    _compare(cfg, a, m, o)


@pytest.mark.parametrize("T,N,hot,K", [(256, 300, 64, 8), (256, 300, 64, 1)])
@pytest.mark.parametrize("env", ["GG_COH_WALK_SWEEP", "GG_COH_WALK_WIDE"])
def test_coherent_walker_variants(T, N, hot, K, env, monkeypatch):
    """The hop-by-hop walkers' three forms give the same run: the pipeline
    (one wave per router position) with its per-lane candidate packets (the
    default), the pipeline scanning every packet (GG_COH_WALK_WIDE=1, the
    path of runs with more than 128 packets in a step) and the one-wave
    position sweep (GG_COH_WALK_SWEEP=1, runs longer than 16 routers)."""
    from oracle import pyoracle as po
    monkeypatch.setenv(env, "1")
    cfg = C.default_config(T, num_shards=K, net_model=C.NET_EMESH_HOP_BY_HOP)
    a, m, o = po.gen_trace(T, N, hot_lines=hot)
    _compare(cfg, a, m, o)


@pytest.mark.parametrize("a1,p1,a2,p2,hot,each", [
    (4, C.POLICY_LRU, 8, C.POLICY_LRU, 16, 1),     # the touch-at-a-time path (> 16 ways)
    (2, C.POLICY_LRU, 16, C.POLICY_LRU, 16, 0),    # 2-way L1: rows loaded byte by byte
    (2, C.POLICY_LRU, 16, C.POLICY_LRU, 16, 1),
    (4, C.POLICY_ROUND_ROBIN, 16, C.POLICY_LRU, 16, 0),
    (4, C.POLICY_LRU, 8, C.POLICY_ROUND_ROBIN, 16, 0),
    (8, C.POLICY_LRU, 16, C.POLICY_LRU, 0, 0),
])
def test_coherent_cache_geometries(a1, p1, a2, p2, hot, each, monkeypatch):
    """L1-D / L2 associativity and policy variants through the L1 hit runs
    (closed-form LRU rows up to 16 ways; GG_COH_TOUCH_EACH=1 forces the
    one-touch-at-a-time path that > 16-way caches take)."""
    from oracle import pyoracle as po
    if each:
        monkeypatch.setenv("GG_COH_TOUCH_EACH", "1")
    cfg = C.default_config(16, l1d_assoc=a1, l1d_policy=p1, l2_assoc=a2, l2_policy=p2)
    a, m, o = po.gen_trace(16, 2500, hot_lines=hot)
    _compare(cfg, a, m, o)


def test_coherent_directory_replacements():
    """A small directory: DirectoryCache replacement, NULLIFY, back-invalidations."""
    from oracle import pyoracle as po
    cfg = C.default_config(16, dir_total_entries=64, dir_assoc=4)
    a, m, o = po.gen_trace(16, 1500, hot_lines=32)
    g = _compare(cfg, a, m, o)
    assert g[1][:, C.TILE_STATS.index("dir_back_invalidations")].sum() > 0


def test_coherent_ragged_and_empty_tiles():
    from oracle import pyoracle as po
    T = 16
    parts = [po.gen_hotspot(t, 0, [0, 7, 1500, 31][t % 4], hot_lines=16) for t in range(T)]
    a = np.concatenate([p[0] for p in parts])
    m = np.concatenate([p[1] for p in parts])
    o = np.zeros(T + 1, np.uint64)
    o[1:] = np.cumsum([len(p[0]) for p in parts])
    cfg = C.default_config(T)
    g = _gpu_run(cfg, a, m, o)
    r = _oracle_run(cfg, a, m, o)
    np.testing.assert_array_equal(g[0], r[0])
    np.testing.assert_array_equal(g[1], r[1])


def test_coherent_two_contexts_exchange():
    """Two contexts on one GPU, each owning half of 4 logical shards, exchanging
    the cross-shard messages at every quantum boundary == one context owning all."""
    torch = torch_dev()
    from graphite_amd import backend as B
    from graphite_amd import coherent as CO
    from oracle import pyoracle as po
    T, N, K = 64, 800, 4
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    addr, meta = to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32)
    outs, engines, bes = [], [], []
    for r in range(2):
        k0, k1 = CO.shard_range(r, 2, K)
        be = B.Backend(C.default_config(T, num_shards=K, shard_begin=k0, shard_end=k1))
        out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
        engines.append(B.CoherentEngine(be, addr, meta, o, out))
        outs.append(out); bes.append(be)
    CO.run_local(engines, 1000 * 1000, K)
    torch.cuda.synchronize()
    got = to_np(outs[0], np.uint64) + to_np(outs[1], np.uint64)
    st = sum(be.coherent_stats()[0] for be in bes)
    ref = _oracle_run(C.default_config(T, num_shards=K), a, m, o)
    np.testing.assert_array_equal(got, ref[0])
    np.testing.assert_array_equal(st, ref[1])


def test_gpu_hotspot_generator_matches_oracle():
    torch = torch_dev()
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    T, N = 8, 5000
    addr = torch.empty(T * N, dtype=torch.int64, device="cuda")
    meta = torch.empty(T * N, dtype=torch.int32, device="cuda")
    B.gen_hotspot_trace(addr, meta, 3, T, N, first=11, hot_lines=64)
    a = np.concatenate([po.gen_hotspot(t, 11, N, hot_lines=64)[0] for t in range(3, 3 + T)])
    m = np.concatenate([po.gen_hotspot(t, 11, N, hot_lines=64)[1] for t in range(3, 3 + T)])
    np.testing.assert_array_equal(to_np(addr, np.uint64), a)
    np.testing.assert_array_equal(to_np(meta, np.uint32), m)


def test_gpu_stress_generator_matches_oracle():
    """configs[4] stress generator: device (gg_gen_stress_trace) == oracle (oracle_gen_stress)."""
    torch = torch_dev()
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    T0, T, N, TT = 1000, 24, 3000, 4096
    addr = torch.empty(T * N, dtype=torch.int64, device="cuda")
    meta = torch.empty(T * N, dtype=torch.int32, device="cuda")
    B.gen_stress_trace(addr, meta, T0, T, N, TT, first=7)
    parts = [po.gen_stress(t, 7, N, TT) for t in range(T0, T0 + T)]
    np.testing.assert_array_equal(to_np(addr, np.uint64), np.concatenate([p[0] for p in parts]))
    np.testing.assert_array_equal(to_np(meta, np.uint32), np.concatenate([p[1] for p in parts]))


@pytest.mark.parametrize("T,N,K,net", [
    (4096, 12, 1, C.NET_EMESH_HOP_COUNTER),     # configs[4]: 4096 tiles, 16-way L2 (reduced length)
    (4096, 8, 8, C.NET_EMESH_HOP_COUNTER),
    (1024, 24, 8, C.NET_EMESH_HOP_BY_HOP),      # the stress pool under router contention, 8 shards
])
def test_coherent_stress_matches_oracle(T, N, K, net):
    """configs[4] coherent stress workload (50/50 R/W,
    30 % of accesses to a 4096-line pool shared by ~64-tile groups), 16-way
    L2: bit-exact against the oracle."""
    from oracle import pyoracle as po
    cfg = C.default_config(T, l2_assoc=16, num_shards=K, net_model=net)
    a, m, o = po.gen_stress_trace(T, N)
    _compare(cfg, a, m, o)


@pytest.mark.parametrize("net", [C.NET_EMESH_HOP_BY_HOP, C.NET_EMESH_HOP_COUNTER])
def test_coherent_contexts_split_equals_one_context(net):
    """1 context x 8 logical shards == 2 contexts x 4 shards each (exchanging
    messages and held hop-by-hop packets at every quantum boundary) == 4
    contexts x 2 == 8 contexts x 1, bit for bit: the schedule depends on the
    shard count only."""
    torch = torch_dev()
    from graphite_amd import backend as B
    from graphite_amd import coherent as CO
    from oracle import pyoracle as po
    T, N, K = 64, 500, 8
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    addr, meta = to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32)
    results = []
    for R in (1, 2, 4, 8):
        outs, engines, bes = [], [], []
        for r in range(R):
            k0, k1 = CO.shard_range(r, R, K)
            be = B.Backend(C.default_config(T, num_shards=K, shard_begin=k0, shard_end=k1, net_model=net))
            out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
            engines.append(B.CoherentEngine(be, addr, meta, o, out))
            outs.append(out); bes.append(be)
        CO.run_local(engines, 1000 * 1000, K)
        torch.cuda.synchronize()
        got = sum(to_np(x, np.uint64) for x in outs)
        st = sum(be.coherent_stats()[0] for be in bes)
        nc = sum(be.noc_counters() for be in bes)
        results.append((got, st, nc))
    for g in results[1:]:
        for x, y in zip(results[0], g):
            np.testing.assert_array_equal(x, y)
    ref = _oracle_run(C.default_config(T, num_shards=K, net_model=net), a, m, o)
    np.testing.assert_array_equal(results[0][0], ref[0])
    np.testing.assert_array_equal(results[0][1], ref[1])
    np.testing.assert_array_equal(results[0][2], ref[3])


def test_coherent_hop_by_hop_holds_packets_at_shard_edges():
    """With 8 shards some packets stop at a shard's edge router and resume in
    the next quantum; every message still arrives (sent == received)."""
    from oracle import pyoracle as po
    T, N, K = 256, 100, 8
    cfg = C.default_config(T, num_shards=K, net_model=C.NET_EMESH_HOP_BY_HOP)
    a, m, o = po.gen_trace(T, N, hot_lines=64)
    g = _compare(cfg, a, m, o)
    ri = g[4]
    assert ri[C.RUN_INFO.index("boundary_msgs")] > 0


@pytest.mark.parametrize("name", sorted(__import__("golden_util").coh_manifest()))
def test_coherent_matches_reference_fixtures(name):
    """The HIP path against the fixtures of the reference's own MSI controllers
    (oracle/ref/coh_harness.cc, tests/golden/coh_*)."""
    import golden_util as G
    cfg, a, m, o, exp = G.coh_case(name, G.coh_manifest()[name])
    out, st, cc, nc, ri = _gpu_run(cfg, a, m, o)
    np.testing.assert_array_equal(out, exp["out"])
    np.testing.assert_array_equal(st, exp["stats"])
    np.testing.assert_array_equal(cc, exp["cache"])
    np.testing.assert_array_equal(nc[:, [C.NET_COUNTERS.index(k) for k in G.NET3]], exp["net"])
    assert ri[C.RUN_INFO.index("quanta")] == exp["quanta"]
    assert ri[C.RUN_INFO.index("steps")] == exp["steps"]


def _rank_worker(rank, world, port, T, N, K, outdir):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from graphite_amd import backend as B
    from graphite_amd import coherent as CO
    from oracle import pyoracle as po
    dist.init_process_group("gloo")
    k0, k1 = CO.shard_range(rank, world, K)
    cfg = C.default_config(T, num_shards=K, shard_begin=k0, shard_end=k1)
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    addr = torch.from_numpy(a.view(np.int64)).cuda()
    meta = torch.from_numpy(m.view(np.int32)).cuda()
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be = B.Backend(cfg)
    eng = B.CoherentEngine(be, addr, meta, o, out)
    CO.run(eng, cfg.quantum_ns * 1000, K, world, rank, "gloo", "cpu")
    torch.cuda.synchronize()
    st = be.coherent_stats()[0]
    res = torch.from_numpy(out.cpu().numpy().copy())
    sts = torch.from_numpy(st.view(np.int64).copy())
    dist.all_reduce(res)
    dist.all_reduce(sts)
    if rank == 0:
        np.save(os.path.join(outdir, "out.npy"), res.numpy().view(np.uint64))
        np.save(os.path.join(outdir, "stats.npy"), sts.numpy().view(np.uint64))
    dist.destroy_process_group()


def test_coherent_two_ranks_one_gpu(tmp_path):
    """The multi-rank path with the real GPU engines: 2 processes on cuda:0,
    2 of 4 logical shards each, the cross-shard ShmemMsgs exchanged by
    all_to_all (gloo, staged through the host) at every quantum boundary
    (graphite_amd/coherent.run) == the oracle owning all 4 shards."""
    torch_dev()
    import socket
    import torch.multiprocessing as mp
    from oracle import pyoracle as po
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    T, N, K = 32, 600, 4
    mp.spawn(_rank_worker, args=(2, port, T, N, K, str(tmp_path)), nprocs=2, join=True)
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    ref = _oracle_run(C.default_config(T, num_shards=K), a, m, o)
    np.testing.assert_array_equal(np.load(tmp_path / "out.npy"), ref[0])
    np.testing.assert_array_equal(np.load(tmp_path / "stats.npy"), ref[1])


@pytest.mark.parametrize("qtype,aux,net", [
    (C.QM_HISTORY_LIST, 0, C.NET_EMESH_HOP_COUNTER),
    (C.QM_BASIC, 0, C.NET_EMESH_HOP_COUNTER),
    (C.QM_HISTORY_LIST, 0, C.NET_EMESH_HOP_BY_HOP),       # list in the DRAM queue and the routers
])
def test_coherent_other_queue_models(qtype, aux, net):
    """dram/queue_model/type (and the router queues) = history_list / basic."""
    from oracle import pyoracle as po
    cfg = C.default_config(16, net_model=net, dram_queue_model_type=qtype, queue_model_type=qtype,
                           basic_moving_avg=aux)
    a, m, o = po.gen_trace(16, 1500, hot_lines=16)
    _compare(cfg, a, m, o)


@pytest.mark.parametrize("T,N,quantum,net", [(16, 600, 1000, C.NET_EMESH_HOP_COUNTER),
                                             (16, 400, 20, C.NET_EMESH_HOP_COUNTER),   # accesses straddle barriers
                                             (64, 200, 1000, C.NET_EMESH_HOP_BY_HOP)])
def test_coherent_multiline_accesses(T, N, quantum, net):
    """Multi-line accesses (core.cc:139-266): gg_split_accesses on the GPU
    equals the oracle's split, the coherent run of the line trace is bit-exact,
    and gg_combine_accesses gives the oracle's per-access latency / misses."""
    from oracle import pyoracle as po
    from graphite_amd import backend as B
    from tests.access_util import gen_multiline
    torch = torch_dev()
    addr, size, meta, offs = gen_multiline(T, N)
    la, lm, first, loffs = B.split_accesses(to_dev(torch, addr, torch.int64), to_dev(torch, size, torch.int32),
                                            to_dev(torch, meta, torch.int32), offs)
    ra, rm, rf, rlo = po.split_accesses(addr, size, meta, offs)
    np.testing.assert_array_equal(to_np(la, np.uint64), ra)
    np.testing.assert_array_equal(to_np(lm, np.uint32), rm)
    np.testing.assert_array_equal(to_np(first, np.uint64), rf)
    np.testing.assert_array_equal(loffs, rlo)
    cfg = C.default_config(T, net_model=net, quantum_ns=quantum)
    g = _compare(cfg, ra, rm, rlo)
    lat, miss = B.combine_accesses(to_dev(torch, g[0], torch.int64), first)
    rl, rmiss = po.combine_accesses(g[0], rf)
    np.testing.assert_array_equal(to_np(lat, np.uint64), rl)
    np.testing.assert_array_equal(to_np(miss, np.uint32), rmiss)
