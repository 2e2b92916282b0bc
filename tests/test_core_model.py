"""Core timing: the simple core model over a coherent run's
per-access results (SimpleCoreModel::handleInstruction,
common/tile/core/models/simple_core_model.cc:43-96).

CPU tests pin the C oracle (oracle_core_model) against a Python loop over
instructions written from the reference function, and check the run-level
property that the model's completion time is the coherent engine's clock.
GPU tests compare gg_core_model_run with the oracle bit for bit: coherent
runs of single-line and split multi-line traces, and long synthetic traces
whose tiles span several device tasks with CONT runs across task edges.
Parity of this row is pinned by the restatement only: the reference's core
model needs McPAT and a Pin instruction stream to run."""
import numpy as np
import pytest

from graphite_amd import config as C

CONT, WRITE, BARRIER = 0x80000000, 1, 0xFFFFFFFF


def py_core_model(meta, acc, offs, f=1.0):
    """simple_core_model.cc:43-96 per instruction, one memory operand each."""
    import math
    cyc = int(math.ceil(1000.0 / f))
    T = len(offs) - 1
    out = np.zeros((T, 8), np.uint64)
    for t in range(T):
        n = tm = mem = ex = rd = wr = 0
        r, e = int(offs[t]), int(offs[t + 1])
        ns = sy = 0
        while r < e:
            if int(meta[r]) == BARRIER:          # sync_client.cc:306-314: a SyncInstruction if it stalled
                lat = int(acc[r]) >> 2
                if lat:
                    n += 1; ns += 1; sy += lat; tm += lat
                r += 1
                continue
            read = not (int(meta[r]) & WRITE)
            lat = int(acc[r]) >> 2
            cost = ((int(meta[r]) & 0x7FFFFFFF) >> 1) * cyc
            r += 1
            while r < e and (int(meta[r]) & CONT) and int(meta[r]) != BARRIER:
                lat += int(acc[r]) >> 2
                r += 1
            n += 1
            if read:
                rd += lat
            else:
                wr += lat
            mem += lat
            ex += cost
            tm += lat + cost
        out[t, :8] = (n, tm, mem, ex, rd, wr, ns, sy)
    return out


def synthetic(T, per_tile, seed, cont_frac=0.3, max_gap=40):
    """Tile-major meta / access words with CONT runs (heads keep a WRITE bit
    and a gap; CONT records carry WRITE | CONT and gap 0, as gg_split_accesses
    writes them); every tile starts with a head."""
    rng = np.random.default_rng(seed)
    n = T * per_tile
    meta = np.zeros(n, np.uint32)
    cont = rng.random(n) < cont_frac
    cont[::per_tile] = False
    head_meta = (rng.integers(0, max_gap, n).astype(np.uint32) << 1) | rng.integers(0, 2, n).astype(np.uint32)
    meta[:] = np.where(cont, np.uint32(CONT | WRITE), head_meta)
    bar = rng.random(n) < 0.02                     # BARRIER records (a stall or none), before a head
    nxt = np.concatenate([~cont[1:], [True]])
    bar &= nxt
    bar[::per_tile] = False
    meta[bar] = np.uint32(BARRIER)
    lat = rng.integers(1000, 400000, n).astype(np.uint64)
    acc = (lat << np.uint64(2)) | rng.integers(0, 3, n).astype(np.uint64)
    acc[bar & (rng.random(n) < 0.3)] = np.uint64(3)  # released without a stall
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(per_tile)
    return meta, acc, offs


def test_oracle_core_model_matches_reference_loop():
    from oracle import pyoracle as po
    meta, acc, offs = synthetic(5, 700, 3)
    offs = np.array([0, 0, 500, 1600, 1601, 3500], np.uint64)      # empty and one-record tiles
    for t in range(len(offs) - 1):                                   # a tile starts with a head
        if offs[t] < offs[t + 1]:
            meta[offs[t]] &= ~np.uint32(CONT)
    for f in (1.0, 2.5):
        np.testing.assert_array_equal(po.core_model(meta, acc, offs, f), py_core_model(meta, acc, offs, f))


def test_oracle_core_time_equals_engine_clock():
    """curr_time advances by cost + latency per instruction: the coherent
    engine's clock rule (start = clock + gap, completion = start + latency)."""
    from oracle import pyoracle as po
    T, N = 16, 300
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_COUNTER)
    a, m, o = po.gen_trace(T, N, hot_lines=16)
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    st = oc.tile_stats()
    core = po.core_model(m, out, o, cfg.frequency_ghz)
    np.testing.assert_array_equal(core[:, C.CORE_STATS.index("time_ps")], st[:, C.TILE_STATS.index("clock_ps")])
    np.testing.assert_array_equal(core[:, C.CORE_STATS.index("memory_stall_ps")],
                                  st[:, C.TILE_STATS.index("latency_ps")])
    np.testing.assert_array_equal(core[:, 0], np.diff(o))


@pytest.mark.gpu
@pytest.mark.parametrize("net", [C.NET_EMESH_HOP_COUNTER, C.NET_EMESH_HOP_BY_HOP])
def test_gpu_core_model_after_coherent_run(net):
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev, to_np
    torch = torch_dev()
    T, N = 64, 300
    cfg = C.default_config(T, num_shards=8, net_model=net)
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    be = B.Backend(cfg)
    addr, meta = to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32)
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_run(addr, meta, o, out)
    be.core_model_run(meta, o, out)
    core = be.core_stats()
    st = be.coherent_stats()[0]
    ref = po.core_model(m, to_np(out, np.uint64), o, cfg.frequency_ghz)
    np.testing.assert_array_equal(core, ref)
    np.testing.assert_array_equal(core[:, C.CORE_STATS.index("time_ps")], st[:, C.TILE_STATS.index("clock_ps")])
    text = be.dump_summary()
    assert text.count("Core Summary:") == T and text.index("Core Summary:") < text.index("Cache Summary:")
    t0 = text.split("Tile 1 Summary:")[0]
    ns = -(-int(st[0, C.TILE_STATS.index("clock_ps")]) // 1000)
    assert "    Completion Time (in nanoseconds): %d\n" % ns in t0
    assert "    Total Instructions: %d\n" % N in t0


@pytest.mark.gpu
def test_gpu_core_model_multiline_accesses():
    """Split accesses: a CONT line record belongs to its head's instruction."""
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.access_util import gen_multiline
    from tests.gpu_util import torch_dev, to_dev, to_np
    torch = torch_dev()
    T, N = 16, 400
    addr, size, meta, offs = gen_multiline(T, N)
    la, lm, first, loffs = po.split_accesses(addr, size, meta, offs)
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_COUNTER, quantum_ns=20)
    be = B.Backend(cfg)
    dm = to_dev(torch, lm, torch.int32)
    out = torch.zeros(len(la), dtype=torch.int64, device="cuda")
    be.coherent_run(to_dev(torch, la, torch.int64), dm, loffs, out)
    be.core_model_run(dm, loffs, out)
    core = be.core_stats()
    np.testing.assert_array_equal(core, po.core_model(lm, to_np(out, np.uint64), loffs, cfg.frequency_ghz))
    assert int(core[:, 0].sum()) == int((size > 0).sum())
    np.testing.assert_array_equal(core[:, C.CORE_STATS.index("time_ps")],
                                  be.coherent_stats()[0][:, C.TILE_STATS.index("clock_ps")])


@pytest.mark.gpu
@pytest.mark.parametrize("T,per_tile,f", [(3, 100000, 1.0), (40, 16384 * 2 + 77, 2.0), (1, 1, 1.0)])
def test_gpu_core_model_long_traces(T, per_tile, f):
    """Tiles of several device tasks (16384 records each): the CONT runs that
    cross a task edge take the WRITE bit of their head in the previous task."""
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev
    torch = torch_dev()
    meta, acc, offs = synthetic(T, per_tile, 11 + T, cont_frac=0.6)
    cfg = C.default_config(T, frequency_ghz=f)
    be = B.Backend(cfg)
    be.core_model_run(to_dev(torch, meta, torch.int32), offs, to_dev(torch, acc, torch.int64))
    np.testing.assert_array_equal(be.core_stats(), po.core_model(meta, acc, offs, f))


@pytest.mark.gpu
def test_gpu_core_model_errors():
    from graphite_amd import backend as B
    from tests.gpu_util import torch_dev
    torch = torch_dev()
    be = B.Backend(C.default_config(4))
    with pytest.raises(B.GGError):
        be.core_stats()                                  # not run yet: GG_ERR_STATE
    meta = torch.zeros(8, dtype=torch.int32, device="cuda")
    acc = torch.zeros(8, dtype=torch.int64, device="cuda")
    with pytest.raises(B.GGError):
        be.core_model_run(meta, np.array([0, 4, 2, 6, 8], np.uint64), acc)   # offsets decrease


def orphan_cont(T, per_tile, seed):
    """synthetic() with CONT records that have no head before them: at a
    tile's start, at a task edge, and right after a BARRIER record."""
    meta, acc, offs = synthetic(T, per_tile, seed, cont_frac=0.5)
    rng = np.random.default_rng(seed + 1)
    for t in range(T):
        b = int(offs[t])
        meta[b] = np.uint32(CONT | (t & 1))                       # the tile starts with a CONT record
        for k in rng.integers(1, per_tile - 1, 6):
            meta[b + k] = np.uint32(BARRIER)
            meta[b + k + 1] = np.uint32(CONT | ((t + int(k)) & 1))  # a CONT record right after a BARRIER
    if per_tile > 16384:
        meta[16383] = np.uint32(BARRIER)                          # ... on the last record of a device task
        meta[16384] = np.uint32(CONT)
    return meta, acc, offs


def test_oracle_core_model_orphan_cont():
    from oracle import pyoracle as po
    meta, acc, offs = orphan_cont(4, 900, 5)
    np.testing.assert_array_equal(po.core_model(meta, acc, offs, 1.0), py_core_model(meta, acc, offs, 1.0))


@pytest.mark.gpu
def test_gpu_core_model_orphan_cont():
    """A CONT record with no head before it (the tile's first record, or the
    one after a BARRIER) is an instruction of its own, as in the oracle."""
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev
    torch = torch_dev()
    for T, per_tile in ((5, 900), (2, 16384 * 2 + 5)):
        meta, acc, offs = orphan_cont(T, per_tile, 7 + T)
        be = B.Backend(C.default_config(T))
        be.core_model_run(to_dev(torch, meta, torch.int32), offs, to_dev(torch, acc, torch.int64))
        np.testing.assert_array_equal(be.core_stats(), po.core_model(meta, acc, offs, 1.0))
