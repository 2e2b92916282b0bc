"""Miss-type classification (Cache track_miss_types, cache.cc:321-405; the
L1-D takes the L1-I flag, l1_cache_cntlr.cc:69): cold / capacity / sharing
misses from the evicted / invalidated / fetched address sets.  Default off
(carbon_sim.cfg:217,228,239).  The oracle's classification is checked for
its invariants (every miss classified once, nothing else changes); the GPU
coherent path against the oracle bit for bit.  Parity unpinned by the
reference itself: the reference harnesses restate Cache (cache.cc needs
McPAT), so no reference-compiled fixture covers these sets."""
import numpy as np
import pytest

from graphite_amd import config as C

MISSES = C.CACHE_COUNTERS.index("misses")


def _cfg(T, track, **kw):
    return C.default_config(T, l1i_track_miss_types=track, l2_track_miss_types=track, **kw)


@pytest.mark.parametrize("net,K", [(C.NET_EMESH_HOP_COUNTER, 1), (C.NET_EMESH_HOP_BY_HOP, 8)])
def test_oracle_coherent_miss_types(net, K):
    from oracle import pyoracle as po
    T, N = 64, 600
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    runs = []
    for track in (0, 1):
        oc = po.OracleCoherent(_cfg(T, track, num_shards=K, net_model=net))
        runs.append((oc.run(a, m, o), oc.tile_stats(), oc.cache_counters(), oc.miss_types()))
    for x, y in zip(runs[0][:3], runs[1][:3]):
        np.testing.assert_array_equal(x, y)                  # tracking changes nothing else
    assert runs[0][3].sum() == 0
    mt, cc = runs[1][3], runs[1][2]
    np.testing.assert_array_equal(mt.sum(axis=2), cc[:, :, MISSES])   # every miss classified once
    assert mt[:, :, 2].sum() > 0                              # the hot lines make sharing misses
    # a cold miss is the first miss of a line in its cache: at most the lines the tile touched
    for t in range(0, T, 7):
        assert mt[t, 0, 0] <= len(np.unique(a[o[t]:o[t + 1]] >> 6))


def test_oracle_private_miss_types_and_flag_quirk():
    """Mode P: capacity misses once the 2 MB region cycles through the 512 KB
    L2; only the L1-I flag turns the L1-D tracking on."""
    from oracle import pyoracle as po
    T, N = 4, 30000
    A, M = zip(*[po.gen_uniform(t, 0, N, lines_log2=15) for t in range(T)])
    a, m = np.concatenate(A), np.concatenate(M)
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    oc = po.OracleCache(_cfg(T, 1))
    oc.run(a, m, offs)
    mt, cc = oc.miss_types(), oc.counters()
    np.testing.assert_array_equal(mt.sum(axis=2), cc[:, :, MISSES])
    assert mt[:, 1, 1].sum() > 0 and mt[:, 0, 1].sum() > 0
    only_l2 = po.OracleCache(C.default_config(T, l2_track_miss_types=1))
    only_l2.run(a, m, offs)
    assert only_l2.miss_types()[:, 0].sum() == 0 and only_l2.miss_types()[:, 1].sum() == mt[:, 1].sum()


@pytest.mark.gpu
@pytest.mark.parametrize("T,N,net,K,l2a", [(16, 1500, C.NET_EMESH_HOP_COUNTER, 1, 8),
                                           (64, 400, C.NET_EMESH_HOP_BY_HOP, 8, 8),
                                           (256, 150, C.NET_EMESH_HOP_BY_HOP, 8, 16)])
def test_gpu_miss_types_match_oracle(T, N, net, K, l2a):
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev, to_np
    torch = torch_dev()
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    cfg = _cfg(T, 1, num_shards=K, net_model=net, l2_assoc=l2a)
    be = B.Backend(cfg)
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_run(to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32), o, out)
    st, cc, _ = be.coherent_stats()
    oc = po.OracleCoherent(cfg)
    ref = oc.run(a, m, o)
    np.testing.assert_array_equal(to_np(out, np.uint64), ref)
    np.testing.assert_array_equal(cc, oc.cache_counters())
    np.testing.assert_array_equal(be.miss_types(), oc.miss_types())
    text = be.dump_summary()
    assert text.count("    Miss Types:\n") == 2 * T
    c0 = int(be.miss_types()[0, 0, 0])
    assert "      Cold Misses: %d\n" % c0 in text.split("Tile 1 Summary:")[0]


@pytest.mark.gpu
def test_gpu_miss_types_errors():
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev
    torch = torch_dev()
    # Mode P does not track
    be = B.Backend(_cfg(4, 1))
    addr = torch.zeros(64, dtype=torch.int64, device="cuda")
    meta = torch.zeros(64, dtype=torch.int32, device="cuda")
    with pytest.raises(B.GGError):
        be.cache_access_batch(addr, meta, np.array([0, 16, 32, 48, 64], np.uint64))
    # a full address table is a capacity error, not a wrong count
    T, N = 16, 2000
    a, m, o = po.gen_trace(T, N, hot_lines=8)
    be = B.Backend(_cfg(T, 1, miss_track_lines=64))
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    with pytest.raises(B.GGError):
        be.coherent_run(to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32), o, out)
