"""Multi-line accesses (core.cc:139-266) on the CPU: the
oracle's split against a literal restatement of the reference loop, the
per-access combine, and coherent runs of split traces (later lines issue at
the previous line's completion and are never cut at the lax barrier)."""
import numpy as np

from graphite_amd import config as C
from oracle import pyoracle as po
from tests.access_util import gen_multiline, split_reference


def test_split_matches_core_loop():
    addr, size, meta, offs = gen_multiline(8, 400)
    got = po.split_accesses(addr, size, meta, offs)
    ref = split_reference(addr, size, meta, offs)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    la, lm, first, loffs = got
    assert (lm[first[:-1][size > 0].astype(np.int64)] & np.uint32(0x80000000) == 0).all()
    assert ((lm & np.uint32(0x80000000)) != 0).sum() > 0            # some accesses span lines
    assert (np.diff(first)[size == 0] == 0).all()


def test_split_edge_cases():
    a = np.array([0x1000, 0x103E, 0x1000, 0x1010, 0x1000, 0x2000], np.uint64)
    s = np.array([4, 4, 64, 128, 0, 1], np.uint32)
    m = np.array([1 << 1, 0, 1, 2 << 1, 5 << 1, 3 << 1], np.uint32)
    la, lm, first, loffs = po.split_accesses(a, s, m, np.array([0, 6], np.uint64))
    assert la.tolist() == [0x1000, 0x1000, 0x1040, 0x1000, 0x1000, 0x1040, 0x1080, 0x2000]
    assert first.tolist() == [0, 1, 3, 4, 7, 7, 8]
    # the zero-size access's 5 gap cycles move to the next access (3 + 5)
    assert lm.tolist() == [2, 0, 0x80000000, 1, 4, 0x80000000, 0x80000000, 8 << 1]
    assert loffs.tolist() == [0, 8]


def test_combine_sums_lines():
    first = np.array([0, 2, 2, 5], np.uint64)
    lvl = [C.LVL_L1, C.LVL_L2, C.LVL_L1, C.LVL_DIR, C.LVL_L1] if hasattr(C, "LVL_L1") else [0, 1, 0, 2, 0]
    lat = [1000, 8000, 1000, 90000, 1000]
    out = np.array([(l << 2) | v for l, v in zip(lat, lvl)], np.uint64)
    L, M = po.combine_accesses(out, first)
    assert L.tolist() == [9000, 0, 92000]
    assert M.tolist() == [1, 0, 1]


def test_coherent_split_trace_runs():
    """A split trace runs to completion in the oracle: every line gets a word,
    the access latency is at least one L1-D hit per line."""
    addr, size, meta, offs = gen_multiline(16, 300)
    la, lm, first, loffs = po.split_accesses(addr, size, meta, offs)
    cfg = C.default_config(16)
    oc = po.OracleCoherent(cfg)
    out = oc.run(la, lm, loffs)
    lat, miss = po.combine_accesses(out, first)
    nlines = np.diff(first).astype(np.uint64)
    assert (lat >= nlines * np.uint64(1000)).all()
    assert (miss <= nlines).all()
    st = oc.tile_stats()
    assert st[:, C.TILE_STATS.index("accesses")].sum() == len(la)


def test_single_line_accesses_split_to_the_line_trace():
    """Accesses inside one line split to exactly the line trace (no GG_META_CONT)."""
    a, m, offs = po.gen_trace(4, 200, hot_lines=8)
    la, lm, first, loffs = po.split_accesses(a + np.uint64(3), np.full(len(a), 8, np.uint32), m, offs)
    np.testing.assert_array_equal(la, a)
    np.testing.assert_array_equal(lm, m)
