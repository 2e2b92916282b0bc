"""GPU parity of the shared-L2 protocols (pr_l1_sh_l2_msi, pr_l1_sh_l2_mesi) in
the coherent mode: the HIP path (k_c_step<false, 2 / 3>, Tile<..., PR = 2 / 3>)
against the fixtures of the reference's own shared-L2 controllers
(oracle/ref/coh_harness.cc -DGG_PROTO_SHL2 [-DGG_SHL2_MESI],
tests/golden/coh_shl2_* and coh_mesi_*) and against the oracle's restatement
(oracle/gg_coherent.inc) on other shapes and networks: access words, tile
statistics, L1-D / L2-slice and NoC counters, bit-exact."""
import numpy as np
import pytest

from graphite_amd import config as C
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
    r = (to_np(out, np.uint64), st, cc, be.noc_counters(), ri)
    be.close()
    return r


def _first_diff(name, x, y):
    d = np.argwhere(np.asarray(x) != np.asarray(y))
    return "%s differ at %d places, first %s: gpu %s expected %s" % (
        name, len(d), d[0], np.asarray(x)[tuple(d[0])], np.asarray(y)[tuple(d[0])])


PROTOS = [C.PROTO_SHL2_MSI, C.PROTO_SHL2_MESI]


def shl2_invariants(stats, cache, out, offs, mesi=False):
    """Size-independent properties of a shared-L2 run: every L1-D miss is one
    request to a home slice (the slices' accesses), answered once; no private
    L2 hits; every DRAM fetch answered; every message received."""
    S = {n: stats[:, i] for i, n in enumerate(C.TILE_STATS)}
    assert np.array_equal(S["accesses"].astype(np.int64), np.diff(np.asarray(offs, np.int64)))
    assert not S["l2_hits"].any()
    assert np.array_equal(S["l1_hits"] + S["l2_misses"], S["accesses"])
    lvl = (out & 3).astype(np.int64)
    assert int((lvl == 2).sum()) == int(S["l2_misses"].sum())
    acc = C.CACHE_COUNTERS.index("accesses")
    reqs = int((S["sent_ex_req"] + S["sent_sh_req"]).sum())
    assert reqs == int(S["l2_misses"].sum()) == int(cache[:, 1, acc].sum())
    reps = int((S["sent_ex_rep"] + S["sent_sh_rep"] + S["sent_upgrade_rep"]).sum())
    assert reps <= reqs if mesi else reps == reqs      # (MESI's SH_REP_EX counts in msgs_sent only)
    assert int(stats[:, C.CT_SENT_DRAM_FETCH_REQ].sum()) == int(stats[:, C.CT_SENT_DRAM_FETCH_REP].sum())
    assert S["msgs_sent"].sum() == S["msgs_received"].sum()


def _fixtures():
    import golden_util as G
    return [(n, G.coh_shl2_manifest) for n in sorted(G.coh_shl2_manifest())] + \
           [(n, G.coh_mesi_sh_manifest) for n in sorted(G.coh_mesi_sh_manifest())]


@pytest.mark.parametrize("name,manifest", _fixtures())
def test_shl2_matches_reference_fixtures(name, manifest):
    import golden_util as G
    cfg, a, m, o, exp = G.coh_case(name, manifest()[name])
    out, st, cc, nc, ri = _gpu_run(cfg, a, m, o)
    for label, x, y in (("access words", out, exp["out"]), ("tile stats", st, exp["stats"]),
                        ("cache counters", cc, exp["cache"]),
                        ("noc counters", nc[:, [C.NET_COUNTERS.index(k) for k in G.NET3]], exp["net"])):
        assert np.array_equal(x, y), _first_diff(label, x, y)
    assert ri[C.RUN_INFO.index("quanta")] == exp["quanta"]
    assert ri[C.RUN_INFO.index("steps")] == exp["steps"]
    shl2_invariants(st, cc, out, o, mesi=name.startswith("mesi_"))


def _compare(cfg, a, m, o):
    from oracle import pyoracle as po
    g = _gpu_run(cfg, a, m, o)
    oc = po.OracleCoherent(cfg)
    r = (oc.run(a, m, o), oc.tile_stats(), oc.cache_counters(), oc.net_counters(), oc.run_info())
    for label, x, y in zip(("access words", "tile stats", "cache counters", "noc counters"), g[:4], r[:4]):
        assert np.array_equal(x, y), _first_diff(label, x, y)
    for k in ("steps", "net_msgs", "self_msgs", "boundary_msgs"):
        i = C.RUN_INFO.index(k)
        assert g[4][i] == r[4][i], (k, g[4][i], r[4][i])
    shl2_invariants(g[1], g[2], g[0], o, mesi=cfg.protocol == C.PROTO_SHL2_MESI)
    return g


@pytest.mark.parametrize("T,N,hot,K,net", [
    (16, 1500, 8, 1, C.NET_EMESH_HOP_BY_HOP),       # router / link contention
    (16, 1200, 8, 2, C.NET_EMESH_HOP_BY_HOP),       # packets held at a shard edge
    (64, 600, 32, 8, C.NET_EMESH_HOP_BY_HOP),
    (256, 150, 64, 4, C.NET_EMESH_HOP_BY_HOP),
    (64, 1000, 32, 8, C.NET_EMESH_HOP_COUNTER),
    (1024, 48, 256, 8, C.NET_EMESH_HOP_BY_HOP),     # configs[3] shape, reduced length
])
@pytest.mark.parametrize("proto", PROTOS)
def test_shl2_matches_oracle(T, N, hot, K, net, proto):
    from oracle import pyoracle as po
    cfg = C.default_config(T, num_shards=K, net_model=net, protocol=proto)
    a, m, o = po.gen_trace(T, N, hot_lines=hot)
    g = _compare(cfg, a, m, o)
    assert proto == C.PROTO_SHL2_MESI or T > 256 or g[1][:, C.TILE_STATS.index("sent_upgrade_rep")].sum() > 0


@pytest.mark.parametrize("proto", PROTOS)
def test_shl2_slice_evictions_match_oracle(proto):
    """2-way slices under hop-by-hop: L2 evictions with NULLIFY of sharers and
    owners, dirty lines stored through the DRAM controller."""
    from oracle import pyoracle as po
    cfg = C.default_config(16, l2_assoc=2, net_model=C.NET_EMESH_HOP_BY_HOP, protocol=proto)
    a, m, o = po.gen_trace(16, 8000, hot_lines=64)
    g = _compare(cfg, a, m, o)
    assert g[2][:, 1, C.CACHE_COUNTERS.index("evictions")].sum() > 0
    assert g[1][:, C.CT_SENT_DRAM_STORE_REQ].sum() > 0


@pytest.mark.parametrize("proto", PROTOS)
def test_shl2_stress_generator_matches_oracle(proto):
    from oracle import pyoracle as po
    cfg = C.default_config(256, num_shards=8, l2_assoc=16, net_model=C.NET_EMESH_HOP_BY_HOP, protocol=proto)
    a, m, o = po.gen_stress_trace(256, 96)
    _compare(cfg, a, m, o)


@pytest.mark.parametrize("W", [2, 4])
@pytest.mark.parametrize("proto", PROTOS)
def test_shl2_round_halves_over_contexts(W, proto, monkeypatch):
    """The multi-rank round (gg_round_pack / unpack / finish) with W contexts on
    one GPU under the shared-L2 protocol: requests to remote home slices cross
    shard boundaries; equal to the oracle."""
    from tests.test_gpu_round import _run_ranks
    from oracle import pyoracle as po
    monkeypatch.setenv("GG_ROUND_SLOT", "1024")
    monkeypatch.delenv("GG_ROUND_BATCH0", raising=False)
    T, N, K = 64, 300, 8
    net = C.NET_EMESH_HOP_BY_HOP
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    stats = {"again": 0, "overflow": 0}
    got = _run_ranks(torch_dev(), W, K, {"T": T, "net": net, "protocol": proto}, a, m, o, stats)
    cfg = C.default_config(T, num_shards=K, net_model=net, protocol=proto)
    oc = po.OracleCoherent(cfg)
    ref = oc.run(a, m, o)
    assert np.array_equal(got[0], ref) and np.array_equal(got[1], oc.tile_stats())
    assert np.array_equal(got[2], oc.net_counters())
