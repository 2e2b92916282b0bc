"""GPU: the multi-rank lax-barrier round through its C-ABI halves
(gg_round_pack / gg_round_unpack / gg_round_finish, the code gg_round_exchange
runs around RCCL) with W = 2, 4 and 8 contexts on one GPU, each owning K/W of
the K = 8 logical shards, and the transport done by device copies (hipMemcpy):
the peers' send slots into their receive slots and the status words into every
rank's gathered words.  This is the multi-rank path of the RCCL round — the
peer slots, the imports of received records, the repeat of a round one rank
had not finished and the sized overflow round — which a one-GPU box cannot run
over RCCL (RCCL refuses two ranks on one device).  Every run must equal one
context running the whole mesh (gg_coherent_run) and the oracle, bit for bit.
Reference: the lax barrier (lax_barrier_sync_server.cc:57-160) and the
transport it replaces (socktransport.cc:401-448)."""
import ctypes
import os

import numpy as np
import pytest

from graphite_amd import config as C
from tests.gpu_util import torch_dev, to_dev, to_np

pytestmark = pytest.mark.gpu


def _hip():
    """The HIP runtime the process already uses (torch and libgraphite_gpu share it)."""
    for line in open("/proc/self/maps"):
        if "libamdhip64" in line:
            lib = ctypes.CDLL(line.split()[-1])
            lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            lib.hipMemcpy.restype = ctypes.c_int
            return lib
    raise RuntimeError("libamdhip64 is not loaded")


def _copy(hip, dst, src, nbytes):
    if nbytes:
        assert hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, 3) == 0   # hipMemcpyDeviceToDevice


def _run_ranks(torch, W, K, cfg_kw, a, m, o, stats):
    """The round protocol over W contexts with a device-copy transport;
    returns (access words, tile stats, noc counters) summed over the ranks."""
    from graphite_amd import backend as B
    from graphite_amd import coherent as CO
    hip = _hip()
    T = cfg_kw["T"]
    addr, meta = to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32)
    bes, outs = [], []
    for r in range(W):
        k0, k1 = CO.shard_range(r, W, K)
        be = B.Backend(C.default_config(T, num_shards=K, shard_begin=k0, shard_end=k1, net_model=cfg_kw["net"],
                                        protocol=cfg_kw.get("protocol", C.PROTO_MSI)))
        out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
        be.coherent_begin(addr, meta, o, out)
        bes.append(be); outs.append(out)
    rb = B.CMSG_RECORD_BYTES
    q, rounds = 0, 0
    while True:
        ios = [be.round_pack(W, r, q) for r, be in enumerate(bes)]
        torch.cuda.synchronize()
        # transport 1: the fixed slots to the peers, the words to everyone
        for r in range(W):
            for p in range(W):
                if p != r:
                    _copy(hip, ios[p].recv + r * ios[p].stride * rb, ios[r].send + p * ios[r].stride * rb,
                          (ios[r].slot + 1) * rb)
                _copy(hip, ios[p].words_all + r * B.ROUND_WORDS * 8, ios[r].words_own, B.ROUND_WORDS * 8)
        torch.cuda.synchronize()
        for r, be in enumerate(bes):
            be.round_unpack(ios[r])
        states = {io.state for io in ios}
        assert len(states) == 1, states                       # every rank decides alike
        state = states.pop()
        rounds += 1
        if state == B.ROUND_AGAIN:
            stats["again"] += 1
            continue
        if state == B.ROUND_OVERFLOW:
            stats["overflow"] += 1
            for r in range(W):                                # transport 2: the remainder of each slot
                for p in range(W):
                    n = ios[r].send_count[p]
                    if p != r:
                        assert ios[p].recv_count[r] == n      # the header travelled with transport 1
                    if p != r and n > ios[r].slot:
                        off = 1 + ios[r].slot
                        _copy(hip, ios[p].recv + (r * ios[p].stride + off) * rb, ios[r].send + (p * ios[r].stride + off) * rb,
                              (n - ios[r].slot) * rb)
            torch.cuda.synchronize()
            for r, be in enumerate(bes):
                be.round_finish(ios[r])
        assert len({(io.next_q, io.done) for io in ios}) == 1
        if ios[0].done:
            break
        q = ios[0].next_q
    torch.cuda.synchronize()
    stats["rounds"] = rounds
    got = sum(to_np(x, np.uint64) for x in outs)
    st = sum(be.coherent_stats()[0] for be in bes)
    nc = sum(be.noc_counters() for be in bes)
    for be in bes:
        be.close()
    return got, st, nc


def _single(torch, cfg, a, m, o):
    from graphite_amd import backend as B
    be = B.Backend(cfg)
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_run(to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32), o, out)
    torch.cuda.synchronize()
    r = (to_np(out, np.uint64), be.coherent_stats()[0], be.noc_counters())
    be.close()
    return r


@pytest.mark.parametrize("W", [2, 4, 8])
@pytest.mark.parametrize("net", [C.NET_EMESH_HOP_BY_HOP, C.NET_EMESH_HOP_COUNTER])
@pytest.mark.parametrize("mode", ["plain", "slot1", "short_batch"])
def test_round_halves_over_contexts_equal_one_context(W, net, mode, monkeypatch):
    """plain: the fixed slots; slot1: one record per slot (GG_ROUND_SLOT=1),
    so nearly every quantum takes the sized overflow round; short_batch:
    rank 0's first batches are one step (GG_ROUND_BATCH0), so its quantum is
    unfinished while the other ranks have finished theirs and the round
    repeats with commit and import skipped on every rank."""
    torch = torch_dev()
    from oracle import pyoracle as po
    T, N, K = 64, 300, 8
    monkeypatch.setenv("GG_ROUND_SLOT", "1" if mode == "slot1" else "1024")
    if mode == "short_batch":
        monkeypatch.setenv("GG_ROUND_BATCH0", "1,16")
    else:
        monkeypatch.delenv("GG_ROUND_BATCH0", raising=False)
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    stats = {"again": 0, "overflow": 0}
    got = _run_ranks(torch, W, K, {"T": T, "net": net}, a, m, o, stats)
    cfg = C.default_config(T, num_shards=K, net_model=net)
    one = _single(torch, cfg, a, m, o)
    for name, x, y in zip(("access words", "tile stats", "noc counters"), got, one):
        assert np.array_equal(x, y), name
    oc = po.OracleCoherent(cfg)
    ref = oc.run(a, m, o)
    assert np.array_equal(got[0], ref) and np.array_equal(got[1], oc.tile_stats())
    assert np.array_equal(got[2], oc.net_counters())
    if mode == "slot1":
        assert stats["overflow"] > 0, stats
    if mode == "short_batch":
        assert stats["again"] > 0, stats


def _round_loop(torch, bes, W, max_rounds=100000):
    """pack / device-copy transport / unpack (/ finish) over the contexts until
    the run ends or fails; returns (rounds, failure) where failure is None or
    (round, [message per rank]) — every rank must fail in the same call, or
    none."""
    from graphite_amd import backend as B
    hip = _hip()
    rb = B.CMSG_RECORD_BYTES
    q, rounds = 0, 0

    def every(fn):
        res = []
        for r, be in enumerate(bes):
            try:
                fn(r, be)
                res.append(None)
            except B.GGError as e:
                res.append(str(e))
        failed = [x is not None for x in res]
        assert all(failed) or not any(failed), res       # collective: all or none
        return res if all(failed) else None

    while rounds < max_rounds:
        ios = [be.round_pack(W, r, q) for r, be in enumerate(bes)]
        torch.cuda.synchronize()
        for r in range(W):
            for p in range(W):
                if p != r:
                    _copy(hip, ios[p].recv + r * ios[p].stride * rb, ios[r].send + p * ios[r].stride * rb,
                          (ios[r].slot + 1) * rb)
                _copy(hip, ios[p].words_all + r * B.ROUND_WORDS * 8, ios[r].words_own, B.ROUND_WORDS * 8)
        torch.cuda.synchronize()
        f = every(lambda r, be: be.round_unpack(ios[r]))
        rounds += 1
        if f:
            return rounds, (rounds, f)
        state = {io.state for io in ios}
        assert len(state) == 1, state
        state = state.pop()
        if state == B.ROUND_AGAIN:
            continue
        if state == B.ROUND_OVERFLOW:
            for r in range(W):
                for p in range(W):
                    n = ios[r].send_count[p]
                    if p != r and n > ios[r].slot:
                        off = 1 + ios[r].slot
                        _copy(hip, ios[p].recv + (r * ios[p].stride + off) * rb,
                              ios[r].send + (p * ios[r].stride + off) * rb, (n - ios[r].slot) * rb)
            torch.cuda.synchronize()
            f = every(lambda r, be: be.round_finish(ios[r]))
            if f:
                return rounds, (rounds, f)
        assert len({(io.next_q, io.done) for io in ios}) == 1
        if ios[0].done:
            return rounds, None
        q = ios[0].next_q
    raise AssertionError("the run did not end")


def _contexts(torch, W, K, T, net, a, m, o):
    from graphite_amd import backend as B
    from graphite_amd import coherent as CO
    addr, meta = to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32)
    bes, outs = [], []
    for r in range(W):
        k0, k1 = CO.shard_range(r, W, K)
        be = B.Backend(C.default_config(T, num_shards=K, shard_begin=k0, shard_end=k1, net_model=net))
        out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
        be.coherent_begin(addr, meta, o, out)
        bes.append(be); outs.append(out)
    return bes, outs, addr, meta


@pytest.mark.parametrize("W", [2, 4])
@pytest.mark.parametrize("where", ["import", "finish"])
def test_round_failure_after_collective_is_collective(W, where, monkeypatch):
    """A failure a rank finds after the round's collective (its commit /
    import in unpack, or the sized import of finish) is kept as that rank's
    pending failure: every rank decides the round alike, and in the NEXT
    round every rank's unpack returns the error — no rank continues into a
    round its peer will not post (lax_barrier_sync_server.cc:57-160: the
    barrier releases all or none).  The failing rank reports its own message,
    its peers 'failed on another rank'."""
    torch = torch_dev()
    from oracle import pyoracle as po
    T, N, K = 64, 300, 8
    net = C.NET_EMESH_HOP_BY_HOP
    monkeypatch.delenv("GG_ROUND_BATCH0", raising=False)
    monkeypatch.setenv("GG_ROUND_SLOT", "1" if where == "finish" else "1024")
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    bad, at = W - 1, 3                                   # the rank and its 0-based unpack / finish call
    monkeypatch.setenv("GG_ROUND_FAIL_IMPORT" if where == "import" else "GG_ROUND_FAIL_FINISH", "%d,%d" % (bad, at))
    bes, outs, _, _ = _contexts(torch, W, K, T, net, a, m, o)
    try:
        rounds, fail = _round_loop(torch, bes, W)
    finally:
        for be in bes:
            be.close()
    assert fail is not None, "the injected failure was lost"
    rnd, msgs = fail
    assert rnd >= at + 2                                  # reported by the round after the failing call
    knob = "GG_ROUND_FAIL_IMPORT" if where == "import" else "GG_ROUND_FAIL_FINISH"
    assert knob in msgs[bad], msgs
    assert all("another rank" in x for r, x in enumerate(msgs) if r != bad), msgs


def test_round_abandoned_after_again_then_fresh_run(monkeypatch):
    """A run abandoned after unpack said GG_ROUND_AGAIN (the round in
    progress: its step offset, attempt and repeat flag) leaves nothing behind:
    gg_coherent_begin starts a new run, whose rounds start at step 0, and the
    result equals one context and the oracle bit for bit."""
    torch = torch_dev()
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    hip = _hip()
    T, N, K, W = 64, 300, 8, 2
    net = C.NET_EMESH_HOP_BY_HOP
    monkeypatch.setenv("GG_ROUND_SLOT", "1024")
    monkeypatch.setenv("GG_ROUND_BATCH0", "1,16")            # rank 0's first batch is one step: AGAIN
    monkeypatch.delenv("GG_ROUND_FAIL_IMPORT", raising=False)
    monkeypatch.delenv("GG_ROUND_FAIL_FINISH", raising=False)
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    bes, outs, addr, meta = _contexts(torch, W, K, T, net, a, m, o)
    rb = B.CMSG_RECORD_BYTES
    ios = [be.round_pack(W, r, 0) for r, be in enumerate(bes)]
    torch.cuda.synchronize()
    for r in range(W):
        for p in range(W):
            if p != r:
                _copy(hip, ios[p].recv + r * ios[p].stride * rb, ios[r].send + p * ios[r].stride * rb,
                      (ios[r].slot + 1) * rb)
            _copy(hip, ios[p].words_all + r * B.ROUND_WORDS * 8, ios[r].words_own, B.ROUND_WORDS * 8)
    torch.cuda.synchronize()
    for r, be in enumerate(bes):
        be.round_unpack(ios[r])
    assert {io.state for io in ios} == {B.ROUND_AGAIN}
    # abandon: a new run on the same contexts
    for be, out in zip(bes, outs):
        out.zero_()
        be.coherent_begin(addr, meta, o, out)
    try:
        _, fail = _round_loop(torch, bes, W)
        assert fail is None, fail
        torch.cuda.synchronize()
        got = sum(to_np(x, np.uint64) for x in outs)
        st = sum(be.coherent_stats()[0] for be in bes)
    finally:
        for be in bes:
            be.close()
    cfg = C.default_config(T, num_shards=K, net_model=net)
    one = _single(torch, cfg, a, m, o)
    assert np.array_equal(got, one[0]) and np.array_equal(st, one[1])
