"""GPU parity of the MOSI protocol (pr_l1_pr_l2_dram_directory_mosi) in the
coherent mode: the HIP path (k_c_step<false, true>, Tile<..., MO = true>)
against the fixtures of the reference's own MOSI controllers
(oracle/ref/coh_harness.cc -DGG_PROTO_MOSI, tests/golden/coh_mosi_*) and against
the oracle's MOSI restatement (oracle/gg_coherent.inc) on other shapes — per
access words, tile statistics, L1-D/L2 and NoC counters and the controllers'
event counters, bit-exact."""
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
    r = (to_np(out, np.uint64), st, cc, be.noc_counters(), ri, be.protocol_stats())
    be.close()
    return r


def _first_diff(name, x, y):
    d = np.argwhere(np.asarray(x) != np.asarray(y))
    return "%s differ at %d places, first %s: gpu %s expected %s" % (
        name, len(d), d[0], np.asarray(x)[tuple(d[0])], np.asarray(y)[tuple(d[0])])


@pytest.mark.parametrize("name", sorted(__import__("golden_util").coh_mosi_manifest()))
def test_mosi_matches_reference_fixtures(name):
    import golden_util as G
    cfg, a, m, o, exp = G.coh_case(name, G.coh_mosi_manifest()[name])
    out, st, cc, nc, ri, ps = _gpu_run(cfg, a, m, o)
    for label, x, y in (("access words", out, exp["out"]), ("tile stats", st, exp["stats"]),
                        ("cache counters", cc, exp["cache"]), ("protocol stats", ps, exp["proto"]),
                        ("noc counters", nc[:, [C.NET_COUNTERS.index(k) for k in G.NET3]], exp["net"])):
        assert np.array_equal(x, y), _first_diff(label, x, y)
    assert ri[C.RUN_INFO.index("quanta")] == exp["quanta"]
    assert ri[C.RUN_INFO.index("steps")] == exp["steps"]


def _compare(cfg, a, m, o):
    from oracle import pyoracle as po
    g = _gpu_run(cfg, a, m, o)
    oc = po.OracleCoherent(cfg)
    r = (oc.run(a, m, o), oc.tile_stats(), oc.cache_counters(), oc.net_counters(), oc.run_info(), oc.proto_stats())
    for label, x, y in zip(("access words", "tile stats", "cache counters", "noc counters"), g[:4], r[:4]):
        assert np.array_equal(x, y), _first_diff(label, x, y)
    assert np.array_equal(g[5], r[5]), _first_diff("protocol stats", g[5], r[5])
    for k in ("steps", "net_msgs", "self_msgs", "boundary_msgs"):
        i = C.RUN_INFO.index(k)
        assert g[4][i] == r[4][i], (k, g[4][i], r[4][i])
    check_invariants(g[1], g[2], g[0], o, per_tile_expected=int(o[1] - o[0]))
    return g


@pytest.mark.parametrize("T,N,hot,K,net", [
    (16, 1500, 8, 1, C.NET_EMESH_HOP_BY_HOP),       # router / link contention
    (16, 1200, 8, 2, C.NET_EMESH_HOP_BY_HOP),       # packets held at a shard edge
    (64, 600, 32, 8, C.NET_EMESH_HOP_BY_HOP),
    (256, 150, 64, 4, C.NET_EMESH_HOP_BY_HOP),
    (64, 1000, 32, 8, C.NET_EMESH_HOP_COUNTER),
    (1024, 48, 256, 8, C.NET_EMESH_HOP_BY_HOP),     # configs[3] shape, reduced length
])
def test_mosi_matches_oracle(T, N, hot, K, net):
    from oracle import pyoracle as po
    cfg = C.default_config(T, num_shards=K, net_model=net, protocol=C.PROTO_MOSI)
    a, m, o = po.gen_trace(T, N, hot_lines=hot)
    g = _compare(cfg, a, m, o)
    P = {k: i for i, k in enumerate(C.PROTO_STATS)}
    assert g[5][:, P["exreq"]].sum() > 0


def test_mosi_directory_replacements_and_evictions():
    """A small directory (NULLIFY of OWNED / SHARED entries, entry RNG reset on
    replacement) and private footprints past the L2 (FLUSH_REP of OWNED lines)."""
    from oracle import pyoracle as po
    cfg = C.default_config(16, dir_total_entries=64, dir_assoc=4, protocol=C.PROTO_MOSI,
                           net_model=C.NET_EMESH_HOP_BY_HOP)
    a, m, o = po.gen_trace(16, 3000, hot_lines=32)
    g = _compare(cfg, a, m, o)
    P = {k: i for i, k in enumerate(C.PROTO_STATS)}
    assert g[5][:, P["nullify_shared"]].sum() > 0


def test_mosi_stress_generator_matches_oracle():
    from oracle import pyoracle as po
    cfg = C.default_config(256, num_shards=8, l2_assoc=16, net_model=C.NET_EMESH_HOP_BY_HOP, protocol=C.PROTO_MOSI)
    a, m, o = po.gen_stress_trace(256, 96)
    _compare(cfg, a, m, o)


def test_mosi_miss_types_follow_the_l1d_flag():
    """MOSI's L1CacheCntlr gives the L1-D its own track flag (…mosi/l1_cache_cntlr.cc:68):
    l1d_track_miss_types turns the L1-D's classification on, the L1-I flag does not."""
    from oracle import pyoracle as po
    T = 16
    a, m, o = po.gen_trace(T, 1500, hot_lines=32)
    for kw, l1_on in ((dict(l1d_track_miss_types=1, l2_track_miss_types=1), True),
                      (dict(l1i_track_miss_types=1), False)):
        cfg = C.default_config(T, protocol=C.PROTO_MOSI, **kw)
        torch = torch_dev()
        from graphite_amd import backend as B
        be = B.Backend(cfg)
        out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
        be.coherent_run(to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32), o, out)
        torch.cuda.synchronize()
        mt = be.miss_types()
        be.close()
        oc = po.OracleCoherent(cfg)
        oc.run(a, m, o)
        assert np.array_equal(mt, oc.miss_types())
        assert (mt[:, 0].sum() > 0) == l1_on


def test_msi_reports_no_protocol_stats():
    from oracle import pyoracle as po
    cfg = C.default_config(16)
    a, m, o = po.gen_trace(16, 300, hot_lines=8)
    assert not _gpu_run(cfg, a, m, o)[5].any()


@pytest.mark.parametrize("W", [2, 4])
@pytest.mark.parametrize("net", [C.NET_EMESH_HOP_BY_HOP, C.NET_EMESH_HOP_COUNTER])
def test_mosi_round_halves_over_contexts(W, net, monkeypatch):
    """The multi-rank round (gg_round_pack / unpack / finish) with W contexts on
    one GPU under MOSI: INV_FLUSH_COMBINED_REQs cross shard boundaries with
    their single receiver; equal to one context and the oracle."""
    from tests.test_gpu_round import _run_ranks
    from oracle import pyoracle as po
    monkeypatch.setenv("GG_ROUND_SLOT", "1024")
    monkeypatch.delenv("GG_ROUND_BATCH0", raising=False)
    T, N, K = 64, 300, 8
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    stats = {"again": 0, "overflow": 0}
    got = _run_ranks(torch_dev(), W, K, {"T": T, "net": net, "protocol": C.PROTO_MOSI}, a, m, o, stats)
    cfg = C.default_config(T, num_shards=K, net_model=net, protocol=C.PROTO_MOSI)
    oc = po.OracleCoherent(cfg)
    ref = oc.run(a, m, o)
    assert np.array_equal(got[0], ref) and np.array_equal(got[1], oc.tile_stats())
    assert np.array_equal(got[2], oc.net_counters())


@pytest.mark.parametrize("name", ["mosi_hot16", "mosi_dir16"])
def test_mosi_dump_summary_has_the_reference_controller_blocks(name):
    """gg_dump_summary of a MOSI run: each tile's block carries the reference's
    L2 Cache Cntlr / Dram Directory Cntlr text (coh_*_summary.txt of
    coh_harness_mosi) after its cache summaries, then the directory cache and
    DRAM summaries (…mosi/memory_manager.cc:412-436)."""
    import golden_util as G
    cfg, a, m, o, exp = G.coh_case(name, G.coh_mosi_manifest()[name])
    torch = torch_dev()
    from graphite_amd import backend as B
    be = B.Backend(cfg)
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_run(to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32), o, out)
    torch.cuda.synchronize()
    txt = be.dump_summary()
    be.close()
    with open("tests/golden/coh_%s_summary.txt" % name) as f:
        ref = f.read().split("Tile ")[1:]
    blocks = txt.split("Tile ")[1:]
    assert len(blocks) == len(ref) == cfg.num_tiles
    for t, (mine, want) in enumerate(zip(blocks, ref)):
        body = want.split(":\n", 1)[1]                      # "Tile t:" dropped
        assert body in mine, t
        assert mine.index("Cache Summary:") < mine.index(body) < mine.index("Dram Directory Summary:") \
            < mine.index("Dram Performance Model Summary:")
