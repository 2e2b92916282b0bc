"""Parity of the HIP private-cache replay (gg_cache_access_batch and the Cache
quartet) with the reference fixtures and the CPU oracle.  Bit-exact."""
import numpy as np
import pytest

from graphite_amd import config as C
from graphite_amd import backend as B
from oracle import pyoracle as po
from golden_util import manifest, load, POLICY, compact_code
from gpu_util import torch_dev, to_dev, to_np
from test_oracle_golden import modep_trace, modep_config

pytestmark = pytest.mark.gpu
M = manifest()


def run_gpu(cfg, addr, meta, offs, torch, chunks=1, want_ev=True):
    be = B.Backend(cfg)
    n = len(addr)
    res = np.zeros(n, np.uint32)
    ev = np.zeros(n, np.uint64)
    # split every tile's records into `chunks` consecutive batches (state persists)
    T = cfg.num_tiles
    cuts = [[int(offs[t]) + (int(offs[t + 1]) - int(offs[t])) * k // chunks for k in range(chunks + 1)]
            for t in range(T)]
    for k in range(chunks):
        idx = np.concatenate([np.arange(cuts[t][k], cuts[t][k + 1]) for t in range(T)]).astype(np.int64)
        sub_off = np.zeros(T + 1, np.uint64)
        for t in range(T):
            sub_off[t + 1] = sub_off[t] + (cuts[t][k + 1] - cuts[t][k])
        a = to_dev(torch, addr[idx], torch.int64)
        m = to_dev(torch, meta[idx], torch.int32)
        r = torch.zeros(len(idx), dtype=torch.int32, device="cuda")
        e = torch.zeros(len(idx), dtype=torch.int64, device="cuda") if want_ev else None
        be.cache_access_batch(a, m, sub_off, r, e)
        torch.cuda.synchronize()
        res[idx] = to_np(r, np.uint32)
        if want_ev:
            ev[idx] = to_np(e, np.uint64)
    return be, res, ev


@pytest.mark.parametrize("name", [k for k, v in M.items() if v["kind"] == "modep"])
@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("kern", [0, 1, 2])       # 0 = streaming (else lean), 1 = sharded generic, 2 = sharded lean
def test_replay_matches_reference_fixtures(name, chunks, kern):
    torch = torch_dev()
    e = M[name]
    addr, meta, offs = modep_trace(e)
    cfg = modep_config(e)
    cfg.replay_kernel = kern
    be, res, ev = run_gpu(cfg, addr, meta, offs, torch, chunks=chunks)
    np.testing.assert_array_equal(compact_code(res), load(e["result_file"], np.uint8))
    cnt = load(e["counters_file"], np.uint64).reshape(e["tiles"], 2, C.NUM_CACHE_COUNTERS)
    np.testing.assert_array_equal(be.cache_counters(), cnt)
    for t in range(e["tiles"]):
        sl = slice(int(offs[t]), int(offs[t + 1]))
        m = (res[sl] & C.RES_L2_EVICT) != 0
        assert int(ev[sl][m].sum(dtype=np.uint64)) == e["evicted_sum"][t]
        assert np.all(ev[sl][~m] == np.uint64(0xFFFFFFFFFFFFFFFF))


def ragged_trace(T, seed, lines_log2, max_len):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len, T)
    lens[rng.integers(0, T)] = 0                          # an empty tile
    addrs, metas = [], []
    for t in range(T):
        a, m = po.gen_uniform(t, int(rng.integers(0, 1000)), int(lens[t]), lines_log2=lines_log2)
        addrs.append(a)
        metas.append(m)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return np.concatenate(addrs), np.concatenate(metas), offs


@pytest.mark.parametrize("geom", [
    dict(),                                                      # reference defaults
    dict(l2_assoc=16),                                           # configs[4]: 16-way L2
    dict(l2_assoc=16, l1d_policy=C.POLICY_ROUND_ROBIN, l2_policy=C.POLICY_ROUND_ROBIN),
    dict(l1d_size_kb=4, l1d_assoc=2, l2_size_kb=16, l2_assoc=4),
    dict(l1d_policy=C.POLICY_ROUND_ROBIN, l2_policy=C.POLICY_ROUND_ROBIN),
    dict(l1d_size_kb=16, l1d_assoc=8, l2_size_kb=256, l2_assoc=8),
])
@pytest.mark.parametrize("kern", [0, 1, 2])
def test_replay_matches_oracle_ragged(geom, kern):
    torch = torch_dev()
    T = 24
    addr, meta, offs = ragged_trace(T, 7, 12, 20000)
    cfg = C.default_config(T, replay_kernel=kern, **geom)
    oc = po.OracleCache(cfg)
    ref, ref_ev = oc.run(addr, meta, offs, want_evicted=True)
    be, res, ev = run_gpu(cfg, addr, meta, offs, torch, chunks=2)
    np.testing.assert_array_equal(res, ref)
    np.testing.assert_array_equal(ev, ref_ev)
    np.testing.assert_array_equal(be.cache_counters(), oc.counters())


def test_empty_batch_and_range_error():
    torch = torch_dev()
    cfg = C.default_config(4)
    be = B.Backend(cfg)
    e = torch.zeros(0, dtype=torch.int64, device="cuda")
    be.cache_access_batch(e, torch.zeros(0, dtype=torch.int32, device="cuda"), [0, 0, 0, 0, 0])
    assert int(be.cache_counters().sum()) == 0
    bad = torch.tensor([1 << 62], dtype=torch.int64, device="cuda")
    be.cache_access_batch(bad, torch.zeros(1, dtype=torch.int32, device="cuda"), [0, 1, 1, 1, 1])
    with pytest.raises(B.GGError) as ei:
        be.cache_counters()
    assert ei.value.code == -4


@pytest.mark.parametrize("name", [k for k, v in M.items() if v["kind"] == "quartet"])
def test_quartet_matches_reference(name):
    torch_dev()
    e = M[name]
    rows = load(e["file"], np.uint64).reshape(-1, 10)
    level = e["level"]
    kw = {}
    if level == 0:
        kw.update(l1d_size_kb=e["size_kb"], l1d_assoc=e["assoc"], l1d_policy=POLICY[e["policy"]],
                  l2_size_kb=max(e["size_kb"], 4), l2_assoc=8)
    else:
        kw.update(l2_size_kb=e["size_kb"], l2_assoc=e["assoc"], l2_policy=POLICY[e["policy"]],
                  l1d_size_kb=2, l1d_assoc=4)
    be = B.Backend(C.default_config(1, **kw))
    INV = 0xFFFFFFFFFFFFFFFF
    for r in rows[:1500]:
        op, addr, ins, loc, ok, otag, ost, oloc, ev, evaddr = (int(x) for x in r)
        if op == 0:
            li = be.get_line_info(0, level, addr)
            assert (li.tag, li.cstate, li.cached_loc) == (otag, ost, oloc)
        elif op == 1:
            tag = INV if ins == C.CSTATE_INVALID else addr >> 6
            rc = be.set_line_info(0, level, addr, B.LineInfo(tag, ins, loc if ins else 0))
            assert (rc == 0) == bool(ok)
        elif op in (2, 3):
            assert (be.access_line(0, level, addr, op == 3) == 0) == bool(ok)
        elif ok:
            rc, e_, ea, evi = be.insert_line(0, level, addr, B.LineInfo(addr >> 6, ins, loc))
            assert rc == 0
            assert (e_, ea, evi.tag, evi.cstate, evi.cached_loc) == (ev, evaddr, otag, ost, oloc)


def test_full_size_config2_subset_and_properties():
    """configs[1] at full per-tile length (2^22 records per tile): a subset of
    tiles against the oracle bit-for-bit, all tiles through size-independent
    properties of the counters."""
    torch = torch_dev()
    T, N = 64, 1 << 22
    cfg = C.default_config(T)
    be = B.Backend(cfg)
    addr = torch.empty(T * N, dtype=torch.int64, device="cuda")
    meta = torch.empty(T * N, dtype=torch.int32, device="cuda")
    B.gen_uniform_trace(addr, meta, 0, T, N)
    res = torch.empty(T * N, dtype=torch.int32, device="cuda")
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    be.cache_access_batch(addr, meta, offs, res)
    cnt = be.cache_counters()
    for t in (0, 37):
        a, m = po.gen_uniform(t, 0, N)
        np.testing.assert_array_equal(to_np(addr[t * N:(t + 1) * N], np.uint64), a)
        oc = po.OracleCache(C.default_config(1))
        r = oc.run(a - np.uint64(t << 26), m, np.array([0, N], np.uint64))
        np.testing.assert_array_equal(to_np(res[t * N:(t + 1) * N], np.uint32), r)
        np.testing.assert_array_equal(cnt[t], oc.counters()[0])
    l1, l2 = cnt[:, 0], cnt[:, 1]
    assert np.all(l1[:, 0] == N)                                   # every record reaches L1-D
    assert np.all(l2[:, 0] == l1[:, 1])                            # L1-D misses go to L2
    assert np.all(l1[:, 2] + l1[:, 4] == l1[:, 0])
    r = to_np(res, np.uint32)
    assert int(((r & C.RES_L2_MISS) != 0).sum()) == int(l2[:, 1].sum())   # directory requests = L2 misses
    assert int(((r & C.RES_L1_MISS) != 0).sum()) == int(l1[:, 1].sum())
    assert int(((r & C.RES_L2_EVICT) != 0).sum()) == int(l2[:, 6].sum())
    assert int(((r & C.RES_L2_EVICT_DIRTY) != 0).sum()) == int(l2[:, 7].sum())


def test_stream_idle_waves_alternating_bursts():
    """Streaming replay with consumer waves that go idle for long stretches:
    records come in bursts that name only the L1-D sets of one consumer wave
    (sets 0..63, then 64..127, ...), so the other wave polls an empty ring while
    it keeps its counters in byte fields.  Results and counters bit-exact vs the
    oracle (guards the counter-folding cadence against idle passes)."""
    torch = torch_dev()
    T, N = 16, 400000
    rng = np.random.default_rng(11)
    addrs, metas = [], []
    for t in range(T):
        a, m = po.gen_uniform(t, 0, N, lines_log2=16)
        line = a >> np.uint64(6)
        burst = np.cumsum(rng.integers(1500, 4000, N // 1500 + 1))
        half = (np.searchsorted(burst, np.arange(N), side="right") & 1).astype(np.uint64)
        s = (line & np.uint64(63)) | (half << np.uint64(6))
        line = (line & ~np.uint64(127)) | s
        addrs.append(line << np.uint64(6))
        metas.append(m)
    addr, meta = np.concatenate(addrs), np.concatenate(metas)
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    cfg = C.default_config(T)
    oc = po.OracleCache(cfg)
    ref = oc.run(addr, meta, offs)
    be, res, _ = run_gpu(cfg, addr, meta, offs, torch, want_ev=False)
    np.testing.assert_array_equal(res, ref)
    np.testing.assert_array_equal(be.cache_counters(), oc.counters())


def test_stream_broken_handoff_is_flagged_not_stored(monkeypatch):
    """The streaming replay's hand-off guard (the r05 pm0 fault: a broken
    hand-off named a record outside its tile and the consumer stored there):
    with GG_STREAM_BAD_INDEX=1 the producer hands each tile's first record
    over with an index one past the tile's end.  The consumer must flag it
    (GG_DERR_CAP -> gg_cache_get_counters fails with the hand-off message),
    store no result outside the batch, and every other record's result must
    still equal the oracle's (CacheSet::find / insert order, cache_set.cc:57-103)."""
    torch = torch_dev()
    T, N = 4, 3000
    addr, meta, offs = ragged_trace(T, 11, 12, N)
    cfg = C.default_config(T, replay_kernel=0)
    oc = po.OracleCache(cfg)
    ref, _ = oc.run(addr, meta, offs, want_evicted=True)
    n = int(offs[-1])
    be = B.Backend(cfg)
    a, m = to_dev(torch, addr, torch.int64), to_dev(torch, meta, torch.int32)
    # the batch's results sit inside a larger buffer: a store past the batch would land in the guard words
    guard = 4096
    big = torch.full((n + guard,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    monkeypatch.setenv("GG_STREAM_BAD_INDEX", "1")
    be.cache_access_batch(a, m, offs, big[:n], None)
    torch.cuda.synchronize()
    monkeypatch.delenv("GG_STREAM_BAD_INDEX")
    with pytest.raises(B.GGError) as ei:
        be.cache_counters()
    assert "hand-off" in str(ei.value)
    got = to_np(big, np.uint32)
    assert np.all(got[n:] == np.uint32(0x5A5A5A5A))              # nothing stored past the batch
    first = {int(offs[t]) for t in range(T) if offs[t + 1] > offs[t]}
    rest = np.array([i for i in range(n) if i not in first], dtype=np.int64)
    np.testing.assert_array_equal(got[rest], ref[rest])
    for i in first:                                              # the flagged records' words were not written
        assert got[i] == np.uint32(0x5A5A5A5A)
