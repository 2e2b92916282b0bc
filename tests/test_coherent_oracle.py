"""CPU tests of the coherent-mode (Mode C) oracle (oracle/gg_coherent.inc):
against the pinned private-mode restatement where the two must agree, the
run invariants, determinism, and the shard semantics."""
import numpy as np
import pytest

from graphite_amd import config as C
from oracle import pyoracle as po
from tests.coherent_util import check_invariants


@pytest.mark.parametrize("T,N,K", [(16, 3000, 1), (16, 2000, 4), (64, 1500, 8)])
def test_private_trace_matches_private_mode(T, N, K):
    """With no sharing and no directory back-invalidation, every L1-D / L2
    counter and every hit level of the coherent run equals the private-mode
    replay (pinned by the reference's own CacheSet code, tests/golden/)."""
    cfg = C.default_config(T, num_shards=K)
    a, m, o = po.gen_trace(T, N, hot_lines=0)
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    st = oc.tile_stats()
    assert st[:, C.TILE_STATS.index("dir_back_invalidations")].sum() == 0
    op = po.OracleCache(cfg)
    res = op.run(a, m, o)
    np.testing.assert_array_equal(oc.cache_counters(), op.counters())
    plvl = np.where(res & C.RES_L1_MISS, np.where(res & C.RES_L2_MISS, 2, 1), 0)
    np.testing.assert_array_equal((out & 3).astype(np.int64), plvl)
    check_invariants(st, oc.cache_counters(), out, o, per_tile_expected=N)


@pytest.mark.parametrize("T,N,hot,net", [(16, 2000, 64, C.NET_EMESH_HOP_COUNTER),
                                         (16, 1500, 8, C.NET_EMESH_HOP_BY_HOP),
                                         (64, 800, 64, C.NET_EMESH_HOP_COUNTER)])
def test_hotspot_invariants_and_determinism(T, N, hot, net):
    cfg = C.default_config(T, net_model=net)
    a, m, o = po.gen_trace(T, N, hot_lines=hot)
    runs = []
    for _ in range(2):
        oc = po.OracleCoherent(cfg)
        out = oc.run(a, m, o)
        runs.append((out, oc.tile_stats(), oc.cache_counters(), oc.net_counters()))
        check_invariants(runs[-1][1], runs[-1][2], out, o, per_tile_expected=N)
    for x, y in zip(*runs):
        np.testing.assert_array_equal(x, y)
    st = runs[0][1]
    # the shared lines generate coherence traffic
    assert st[:, C.TILE_STATS.index("sent_inv_req")].sum() > 0
    assert st[:, C.TILE_STATS.index("sent_flush_req")].sum() + st[:, C.TILE_STATS.index("sent_wb_req")].sum() > 0


def test_shards_defer_cross_shard_messages():
    """More logical shards hold more messages to the boundary; the protocol
    outcome per access stays legal and the invariants hold."""
    T, N = 16, 1500
    a, m, o = po.gen_trace(T, N, hot_lines=16)
    info = {}
    for K in (1, 4):
        oc = po.OracleCoherent(C.default_config(T, num_shards=K))
        out = oc.run(a, m, o)
        check_invariants(oc.tile_stats(), oc.cache_counters(), out, o, per_tile_expected=N)
        info[K] = oc.run_info()
    assert info[1][C.RUN_INFO.index("boundary_msgs")] == 0
    assert info[4][C.RUN_INFO.index("boundary_msgs")] > 0


def test_directory_replacement_nullify():
    """A tiny directory forces DirectoryCache replacements: NULLIFY flows,
    back-invalidations and the extra access of the assert in
    getReplacementCandidates (directory_cache.cc:161)."""
    T, N = 16, 1500
    cfg = C.default_config(T, dir_total_entries=64, dir_assoc=4)
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    st = oc.tile_stats()
    check_invariants(st, oc.cache_counters(), out, o, per_tile_expected=N)
    assert st[:, C.TILE_STATS.index("dir_evictions")].sum() > 0
    assert st[:, C.TILE_STATS.index("dir_back_invalidations")].sum() > 0


@pytest.mark.parametrize("T,K", [(16, 2), (64, 8), (256, 8)])
def test_hop_by_hop_shards_invariants_and_determinism(T, K):
    """emesh_hop_by_hop across logical shards (packets held at the shard edge
    and resumed after the quantum boundary): invariants, determinism, and the
    same network totals as a run with one shard wherever they must agree."""
    N = 300
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    cfg = C.default_config(T, num_shards=K, net_model=C.NET_EMESH_HOP_BY_HOP)
    runs = []
    for _ in range(2):
        oc = po.OracleCoherent(cfg)
        out = oc.run(a, m, o)
        runs.append((out, oc.tile_stats(), oc.cache_counters(), oc.net_counters(), oc.run_info()))
        check_invariants(runs[-1][1], runs[-1][2], out, o, per_tile_expected=N)
    for x, y in zip(*runs):
        np.testing.assert_array_equal(x, y)
    nc = runs[0][3]
    names = C.NET_COUNTERS
    assert nc[:, names.index("packets_sent")].sum() == nc[:, names.index("packets_received")].sum()
    assert runs[0][4][C.RUN_INFO.index("boundary_msgs")] > 0


def test_shard_blocks_keep_routes_inside():
    """Every XY route between two tiles of one 2-D block shard stays in it."""
    for T, K in [(64, 8), (256, 4), (1024, 8), (256, 5)]:
        sm = C.shard_map(T, K)
        w = int(np.sqrt(T))
        for s in range(0, T, 7):
            for d in range(0, T, 5):
                if sm[s] != sm[d]:
                    continue
                x, y = s % w, s // w
                while x != d % w:
                    x += 1 if d % w > x else -1
                    assert sm[y * w + x] == sm[s]
                while y != d // w:
                    y += 1 if d // w > y else -1
                    assert sm[y * w + x] == sm[s]


@pytest.mark.parametrize("T,K,net", [(64, 8, C.NET_EMESH_HOP_BY_HOP), (64, 4, C.NET_EMESH_HOP_COUNTER),
                                     (256, 8, C.NET_EMESH_HOP_BY_HOP)])
def test_parallel_oracle_equals_single_context(T, K, net):
    """The all-core CPU baseline (one oracle context per shard, OpenMP) is the
    same schedule as one context owning every shard: identical outputs."""
    N = 200
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    cfg = C.default_config(T, num_shards=K, net_model=net)
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    got = po.coherent_run_parallel(cfg, a, m, o, threads=4)
    np.testing.assert_array_equal(got[0], out)
    np.testing.assert_array_equal(got[1], oc.tile_stats())
    np.testing.assert_array_equal(got[2], oc.cache_counters())
    np.testing.assert_array_equal(got[3], oc.net_counters())
    ri = oc.run_info()
    for k in ("quanta", "steps", "net_msgs", "self_msgs", "boundary_msgs"):
        assert got[4][C.RUN_INFO.index(k)] == ri[C.RUN_INFO.index(k)], k


@pytest.mark.parametrize("T,K,net,hot", [(64, 8, C.NET_EMESH_HOP_BY_HOP, 32), (64, 1, C.NET_EMESH_HOP_BY_HOP, 32),
                                         (64, 4, C.NET_EMESH_HOP_COUNTER, 32), (256, 8, C.NET_EMESH_HOP_BY_HOP, 64)])
def test_tile_parallel_oracle_equals_serial(T, K, net, hot):
    """The tile-parallel CPU baseline (oracle_coh_set_threads: each step's tiles,
    then the hop-by-hop routing stage by stage - injection per source, X per
    row, Y per column, SELF per destination - on OpenMP threads) produces the
    serial global-event-queue run's outputs bit for bit."""
    N = 200
    a, m, o = po.gen_trace(T, N, hot_lines=hot)
    cfg = C.default_config(T, num_shards=K, net_model=net)
    ref = po.OracleCoherent(cfg)
    out = ref.run(a, m, o)
    par = po.OracleCoherent(cfg, threads=4)
    got = par.run(a, m, o)
    np.testing.assert_array_equal(got, out)
    np.testing.assert_array_equal(par.tile_stats(), ref.tile_stats())
    np.testing.assert_array_equal(par.cache_counters(), ref.cache_counters())
    np.testing.assert_array_equal(par.net_counters(), ref.net_counters())
    np.testing.assert_array_equal(par.run_info(), ref.run_info())
