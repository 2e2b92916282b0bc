"""The CPU oracle (oracle/gg_oracle.c) pinned against the reference's own
known-answer test and the fixtures produced by the reference's own code."""
import numpy as np
import pytest

from graphite_amd import config as C
from oracle import pyoracle as po
from golden_util import manifest, load, POLICY, compact_code
import golden_util as G

M = manifest()

# tests/unit/history_tree/history_tree.cc:9-20 (QueueModelHistoryTree(1), max_list_size 100, analytical on)
KAT = [(10, 10, 0), (21, 10, 0), (32, 10, 0), (43, 10, 0), (0, 1, 0),
       (0, 10, 53), (45, 10, 18), (60, 4, 13), (70, 8, 7), (75, 10, 10)]


def test_history_tree_kat():
    h = po.OracleHistoryTree(1, 100, True)
    assert [h.delay(t, p) for t, p, _ in KAT] == [d for _, _, d in KAT]
    assert M["htree_kat"]["rows"] == [list(r) for r in KAT]


@pytest.mark.parametrize("name", [k for k, v in M.items() if v["kind"] == "htree"])
def test_history_tree_reference_sequences(name):
    e = M[name]
    rows = load(e["file"], np.uint64).reshape(-1, 3)
    h = po.OracleHistoryTree(1, e["max_list_size"], e["analytical"])
    got = np.array([h.delay(int(t), int(p)) for t, p, _ in rows], np.uint64)
    np.testing.assert_array_equal(got, rows[:, 2])
    assert h.analytical_requests == e["analytical_requests"]


@pytest.mark.parametrize("name", [k for k, v in M.items() if v["kind"] in ("qlist", "qbasic")])
def test_other_queue_models_reference_sequences(name):
    """history_list (std::list restatement + reference QueueModelMG1) and basic
    (reference MovingAverage) fixtures from oracle/ref/ref_harness.cc."""
    e = M[name]
    rows = load(e["file"], np.uint64).reshape(-1, 3)
    if e["kind"] == "qlist":
        h = po.OracleQueueModel(C.QM_HISTORY_LIST, e["aux"], 1, e["max_list_size"], e["analytical"])
    else:
        h = po.OracleQueueModel(C.QM_BASIC, e["aux"])
    got = np.array([h.delay(int(t), int(p)) for t, p, _ in rows], np.uint64)
    np.testing.assert_array_equal(got, rows[:, 2])
    if e["kind"] == "qlist":
        assert h.analytical_requests == e["analytical_requests"]


@pytest.mark.parametrize("name", [k for k, v in M.items() if v["kind"] == "quartet"])
def test_cache_quartet_reference_sequences(name):
    e = M[name]
    rows = load(e["file"], np.uint64).reshape(-1, 10)
    level = e["level"]
    kw = dict(line_size=64)
    if level == 0:
        kw.update(l1d_size_kb=e["size_kb"], l1d_assoc=e["assoc"], l1d_policy=POLICY[e["policy"]])
    else:
        kw.update(l2_size_kb=e["size_kb"], l2_assoc=e["assoc"], l2_policy=POLICY[e["policy"]])
    oc = po.OracleCache(C.default_config(1, **kw))
    INV = 0xFFFFFFFFFFFFFFFF
    for r in rows:
        op, addr, ins, loc, ok, otag, ost, oloc, ev, evaddr = (int(x) for x in r)
        if op == 0:
            li = oc.get_line_info(0, level, addr)
            assert (li.tag, li.cstate, li.cached_loc) == (otag, ost, oloc)
        elif op == 1:
            tag = INV if ins == C.CSTATE_INVALID else addr >> 6
            rc = oc.set_line_info(0, level, addr, po.LineInfo(tag, ins, loc if ins else 0))
            assert (rc == 0) == bool(ok)
        elif op in (2, 3):
            rc = oc.access_line(0, level, addr, op == 3)
            assert (rc == 0) == bool(ok)
        else:
            if not ok:
                continue
            rc, e_, ea, evi = oc.insert_line(0, level, addr, po.LineInfo(addr >> 6, ins, loc))
            assert rc == 0
            assert (e_, ea, evi.tag, evi.cstate, evi.cached_loc) == (ev, evaddr & 0xFFFFFFFFFFFFFFFF, otag, ost, oloc)
    np.testing.assert_array_equal(oc.counters()[0, level], np.array(e["counters"], np.uint64))


def modep_trace(e):
    """The fixture's generator, restated (see ref_harness.cc gen_modep)."""
    T, N, LL = e["tiles"], e["per_tile"], e["lines_log2"]
    addrs, metas = [], []
    for t in range(T):
        seed = 0x9E3779B97F4A7C15 ^ t
        i = np.arange(N, dtype=np.uint64)
        z = _sm_vec(seed, i)
        mask = np.uint64((1 << LL) - 1)
        base = np.uint64(t << 26)
        if e["gen"] == 0:
            a = base + ((z & mask) << np.uint64(6))
            w = ((z >> np.uint64(32)) % np.uint64(3)) == 0
        else:
            sel = (z >> np.uint64(60)) & np.uint64(3)
            hot = base + (((z >> np.uint64(8)) & np.uint64(63)) << np.uint64(6))
            stride = base + (((i * np.uint64(17)) & mask) << np.uint64(6))
            uni = base + ((z & mask) << np.uint64(6))
            a = np.where(sel == 0, hot, np.where(sel == 1, stride, uni))
            w = ((z >> np.uint64(32)) & np.uint64(1)) == 0
        addrs.append(a.astype(np.uint64))
        metas.append(w.astype(np.uint32))
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    return np.concatenate(addrs), np.concatenate(metas), offs


def _sm_vec(seed, i):
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def modep_config(e):
    return C.default_config(e["tiles"], l1d_size_kb=e["l1d_size_kb"], l1d_assoc=e["l1d_assoc"],
                            l1d_policy=POLICY[e["l1d_policy"]], l2_size_kb=e["l2_size_kb"],
                            l2_assoc=e["l2_assoc"], l2_policy=POLICY[e["l2_policy"]])


def test_vectorized_generator_matches_oracle():
    a, m = po.gen_uniform(5, 100, 1000)
    e = {"tiles": 6, "per_tile": 1100, "lines_log2": 15, "gen": 0}
    A, Mt, offs = modep_trace(e)
    np.testing.assert_array_equal(A[5 * 1100 + 100:5 * 1100 + 1100], a)
    np.testing.assert_array_equal(Mt[5 * 1100 + 100:5 * 1100 + 1100], m)


@pytest.mark.parametrize("name", [k for k, v in M.items() if v["kind"] == "modep"])
def test_private_replay_reference_fixtures(name):
    e = M[name]
    addr, meta, offs = modep_trace(e)
    oc = po.OracleCache(modep_config(e))
    res, ev = oc.run(addr, meta, offs, want_evicted=True)
    np.testing.assert_array_equal(compact_code(res), load(e["result_file"], np.uint8))
    cnt = load(e["counters_file"], np.uint64).reshape(e["tiles"], 2, C.NUM_CACHE_COUNTERS)
    np.testing.assert_array_equal(oc.counters(), cnt)
    for t in range(e["tiles"]):
        sl = slice(int(offs[t]), int(offs[t + 1]))
        m = (res[sl] & C.RES_L2_EVICT) != 0
        assert int(ev[sl][m].sum(dtype=np.uint64)) == e["evicted_sum"][t]


def test_fixture_coverage():
    """The fixtures reach every result flag the private path can produce
    (GG_RES_L1_INVAL through the oracle's replay of them)."""
    flags = 0
    levels = set()
    abi = 0
    for k, e in M.items():
        if e["kind"] == "modep":
            r = load(e["result_file"], np.uint8)
            levels |= set(np.unique(r & 3).tolist())
            flags |= int(np.bitwise_or.reduce(r))
            addr, meta, offs = modep_trace(e)
            abi |= int(np.bitwise_or.reduce(po.OracleCache(modep_config(e)).run(addr, meta, offs)))
    assert levels == {0, 1, 2}
    for f in (4, 8, 16, 32, 64):
        assert flags & f, hex(f)
    for f in (C.RES_L1_MISS, C.RES_L2_MISS, C.RES_L1_INVAL, C.RES_L1_EVICT, C.RES_L2_EVICT, C.RES_L2_EVICT_DIRTY,
              C.RES_L2_EVICT_INV_L1, C.RES_UPGRADE):
        assert abi & f, hex(f)


def test_compact_code_mapping():
    r = np.array([0, C.RES_L1_MISS, C.RES_L1_MISS | C.RES_L2_MISS | C.RES_UPGRADE,
                  C.RES_L1_MISS | C.RES_L1_INVAL | C.RES_L2_MISS | C.RES_L1_EVICT | C.RES_L2_EVICT |
                  C.RES_L2_EVICT_DIRTY | C.RES_L2_EVICT_INV_L1], np.uint32)
    assert compact_code(r).tolist() == [0, 1, 2 | 4, 2 | 8 | 16 | 32 | 64]


def test_split_lines():
    # Core::initiateMemoryAccess (core.cc:167-201)
    assert po.split_lines(0x1000, 4) == [0x1000]
    assert po.split_lines(0x103E, 4) == [0x1000, 0x1040]
    assert po.split_lines(0x1000, 64) == [0x1000]      # zero-size tail skipped
    assert po.split_lines(0x1010, 128) == [0x1000, 0x1040, 0x1080]
    assert po.split_lines(0x1000, 0) == []


# ---- coherent mode: pinned by the reference's own MSI controllers ----------
@pytest.mark.parametrize("name", sorted(G.coh_manifest()))
def test_coherent_oracle_matches_reference_controllers(name):
    """oracle/gg_coherent.inc == L1CacheCntlr / L2CacheCntlr / DramDirectoryCntlr
    compiled from /root/reference and driven in the same canonical schedule
    (oracle/ref/coh_harness.cc): every access word, tile statistic, L1-D/L2
    counter and NoC counter, and the quantum / step counts."""
    from graphite_amd import config as C
    cfg, a, m, o, exp = G.coh_case(name, G.coh_manifest()[name])
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    np.testing.assert_array_equal(out, exp["out"])
    np.testing.assert_array_equal(oc.tile_stats(), exp["stats"])
    np.testing.assert_array_equal(oc.cache_counters(), exp["cache"])
    nc = oc.net_counters()[:, [C.NET_COUNTERS.index(k) for k in G.NET3]]
    np.testing.assert_array_equal(nc, exp["net"])
    ri = oc.run_info()
    assert ri[C.RUN_INFO.index("quanta")] == exp["quanta"]
    assert ri[C.RUN_INFO.index("steps")] == exp["steps"]


# ---- coherent mode, MOSI: pinned by the reference's own MOSI controllers ---
@pytest.mark.parametrize("name", sorted(G.coh_mosi_manifest()))
def test_coherent_mosi_oracle_matches_reference_controllers(name):
    """The MOSI restatement (oracle/gg_coherent.inc, protocol = GG_PROTO_MOSI)
    == pr_l1_pr_l2_dram_directory_mosi's L1CacheCntlr / L2CacheCntlr /
    DramDirectoryCntlr compiled from /root/reference (coh_harness_mosi):
    access words, tile statistics (INV_FLUSH_COMBINED_REQs in slot 29), cache
    and NoC counters, quanta / steps and the controllers' event counters."""
    from graphite_amd import config as C
    cfg, a, m, o, exp = G.coh_case(name, G.coh_mosi_manifest()[name])
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    np.testing.assert_array_equal(out, exp["out"])
    np.testing.assert_array_equal(oc.tile_stats(), exp["stats"])
    np.testing.assert_array_equal(oc.cache_counters(), exp["cache"])
    nc = oc.net_counters()[:, [C.NET_COUNTERS.index(k) for k in G.NET3]]
    np.testing.assert_array_equal(nc, exp["net"])
    np.testing.assert_array_equal(oc.proto_stats(), exp["proto"])
    ri = oc.run_info()
    assert ri[C.RUN_INFO.index("quanta")] == exp["quanta"]
    assert ri[C.RUN_INFO.index("steps")] == exp["steps"]


# ---- coherent mode, shared L2: pinned by the reference's pr_l1_sh_l2_msi ----
@pytest.mark.parametrize("name", sorted(G.coh_shl2_manifest()))
def test_coherent_shl2_oracle_matches_reference_controllers(name):
    """The shared-L2 restatement (oracle/gg_coherent.inc, protocol =
    GG_PROTO_SHL2_MSI) == pr_l1_sh_l2_msi's L1CacheCntlr / L2CacheCntlr /
    DramCntlr compiled from /root/reference (coh_harness_shl2): access words,
    tile statistics (DRAM_FETCH_REQ / STORE_REQ / FETCH_REP in slots 29-31),
    L1-D and L2-slice counters, NoC counters, quanta / steps."""
    _shl2_oracle_case(name, G.coh_shl2_manifest())


def _shl2_oracle_case(name, manifest):
    from graphite_amd import config as C
    cfg, a, m, o, exp = G.coh_case(name, manifest[name])
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    np.testing.assert_array_equal(out, exp["out"])
    np.testing.assert_array_equal(oc.tile_stats(), exp["stats"])
    np.testing.assert_array_equal(oc.cache_counters(), exp["cache"])
    nc = oc.net_counters()[:, [C.NET_COUNTERS.index(k) for k in G.NET3]]
    np.testing.assert_array_equal(nc, exp["net"])
    ri = oc.run_info()
    assert ri[C.RUN_INFO.index("quanta")] == exp["quanta"]
    assert ri[C.RUN_INFO.index("steps")] == exp["steps"]


@pytest.mark.parametrize("name", sorted(G.coh_mesi_sh_manifest()))
def test_coherent_shl2_mesi_oracle_matches_reference_controllers(name):
    """The shared-L2 MESI restatement (protocol = GG_PROTO_SHL2_MESI) ==
    pr_l1_sh_l2_mesi's controllers compiled from /root/reference
    (coh_harness_shl2_mesi): the same outputs as the MSI test above."""
    _shl2_oracle_case(name, G.coh_mesi_sh_manifest())


def test_shl2_fixtures_exercise_the_protocol():
    from graphite_amd import config as C_
    """The shared-L2 fixtures reach the slice's paths: remote L2 hits (SH_REPs
    beyond the DRAM fetches), upgrade replies, slice evictions with NULLIFY
    (invalidations of sharers, flushes of owners) and DRAM stores of dirty lines."""
    tot = {}
    for name in G.coh_shl2_manifest():
        cfg, a, m, o, exp = G.coh_case(name, G.coh_shl2_manifest()[name])
        tot[name] = (exp["stats"].sum(0), exp["cache"][:, 1].sum(0))
    mesi_sent = sum(int(G.coh_case(n, G.coh_mesi_sh_manifest()[n])[4]["stats"][:, C_.TILE_STATS.index("msgs_sent")].sum())
                    for n in ("mesi_hot16", "mesi_shard64"))
    msi_sent = sum(int(tot[n][0][C_.TILE_STATS.index("msgs_sent")]) for n in ("shl2_hot16", "shl2_shard64"))
    assert mesi_sent != msi_sent                      # EXCLUSIVE lines change the traffic
    from graphite_amd import config as C
    st = sum(t[0] for t in tot.values())
    by = lambda k: int(st[C.TILE_STATS.index("sent_%s" % k.lower())])
    assert by("UPGRADE_REP") > 0 and by("WB_REQ") > 0 and by("FLUSH_REQ") > 0
    assert by("SH_REP") + by("EX_REP") > int(st[C.CT_SENT_DRAM_FETCH_REP])    # L2 hits at the home slice
    assert int(tot["shl2_evict16"][1][C.CACHE_COUNTERS.index("evictions")]) > 0
    assert int(st[C.CT_SENT_DRAM_STORE_REQ]) > 0


def test_mosi_fixtures_exercise_the_protocol():
    """The MOSI fixtures reach what MSI lacks: upgrade replies, combined
    invalidate-flush requests, OWNED write-backs (dirty evictions / shared
    requests in OWNED state) and directory-entry nullifies."""
    tot = {}
    for name in G.coh_mosi_manifest():
        cfg, a, m, o, exp = G.coh_case(name, G.coh_mosi_manifest()[name])
        tot[name] = (exp["proto"].sum(0), exp["stats"][:, 29].sum())
    from graphite_amd import config as C
    P = {k: i for i, k in enumerate(C.PROTO_STATS)}
    assert sum(int(p[P["exreq_upgrade"]]) for p, _ in tot.values()) > 0
    assert sum(int(ifc) for _, ifc in tot.values()) > 0
    assert int(tot["mosi_dir16"][0][P["nullify"]]) > 0
    assert sum(int(p[P["shreq_shared"]]) for p, _ in tot.values()) > 0
