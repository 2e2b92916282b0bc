"""configs[0] on the reference's own program: tests/benchmarks/fft/fft.C
(-p16) captured by tools/fft_trace (TSan access hooks + the PARMACS macros of
tools/fft_trace/parmacs.h, standing in for Graphite's Pin front end,
pin/lite/memory_modeling.cc:13-89).  The committed fixtures
tests/golden/fft_real_p16_m{10,14}.npz were written by
tools/fft_trace/make_traces.py; when the reference is mounted (this container)
the m10 capture is redone and must equal the fixture.  The GPU replays the
traces in Mode C bit-exact against the oracle.  The traces' BARRIER positions
become GG_META_BARRIER records (load_fft_trace): the tiles wait for each
other and continue at the latest arrival (SimBarrier, sync_server.cc:133-170),
on the GPU and in the oracle alike."""
import os

import numpy as np
import pytest

from graphite_amd import capture as cp
from graphite_amd import config as C
from tests.coherent_util import check_invariants

REF = os.environ.get("GRAPHITE_REFERENCE", "/root/reference")


@pytest.mark.parametrize("m", [10, 14])
def test_fixture_structure(m):
    a, meta, offs, bars = cp.load_fft_trace(cp.REAL_FFT_TRACES[m], barriers=False)
    assert len(offs) == 17 and offs[0] == 0 and offs[-1] == len(a) == len(meta)
    n = np.diff(offs.astype(np.int64))
    assert n.min() > 0 and n.max() - n.min() < 0.01 * n.max()     # equal shares of the transform
    assert all(len(b) == 7 for b in bars)                          # the seven BARRIER calls of SlaveStart
    assert all(np.all(np.diff(b.astype(np.int64)) >= 0) and int(b[-1]) <= int(c) for b, c in zip(bars, n))
    assert np.all(a >= (1 << 32)) and np.all(a % 8 == 0)            # heap arena, 8-B operands
    assert np.all((meta >> 1) == 1)                                # one cycle per access
    w = (meta & 1).astype(bool)
    assert 0.25 < w.mean() < 0.5
    lines = [set((a[offs[t]:offs[t + 1]] >> 6).tolist()) for t in range(2)]
    assert len(lines[0] & lines[1]) > 0                            # the transposes share the matrix


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "tests", "benchmarks", "fft", "fft.C")),
                    reason="the reference is not mounted")
def test_capture_reproduces_fixture(tmp_path):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "m10.npz")
    subprocess.check_call([sys.executable, os.path.join(root, "tools", "fft_trace", "make_traces.py"), out, "10"],
                          stdout=subprocess.DEVNULL)
    got, ref = cp.load_fft_trace(out, False), cp.load_fft_trace(cp.REAL_FFT_TRACES[10], False)
    for x, y in zip(got[:3], ref[:3]):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(got[3], ref[3]):
        np.testing.assert_array_equal(x, y)


def barrier_times(meta, out, offs, gap_ps=1000):
    """Per tile, the clock right after each released barrier, from the access
    words alone: the sum of gaps and latencies up to the barrier plus its stall."""
    res = []
    for t in range(len(offs) - 1):
        s, e = int(offs[t]), int(offs[t + 1])
        m, w = meta[s:e], out[s:e]
        bar = m == C.META_BARRIER
        step = np.where(bar, 0, (m & 0x7FFFFFFF) >> 1).astype(np.uint64) * np.uint64(gap_ps) + (w >> np.uint64(2))
        res.append(np.cumsum(step)[bar])
    return np.array(res)


def test_oracle_simulates_real_fft():
    from oracle import pyoracle as po
    cfg = C.default_config(16, net_model=C.NET_EMESH_HOP_COUNTER)
    a, meta, offs, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[10], barriers=False)
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, meta, offs)
    check_invariants(oc.tile_stats(), oc.cache_counters(), out, offs)
    assert oc.tile_stats()[:, C.TILE_STATS.index("l2_misses")].sum() > 0


def test_oracle_barriers_release_at_latest_arrival():
    """Every tile leaves barrier i at the same time = the latest arrival, the
    barrier records' words carry GG_LVL_SYNC, and the core model's completion
    time (with the sync stalls) is the engine's clock."""
    from oracle import pyoracle as po
    cfg = C.default_config(16, net_model=C.NET_EMESH_HOP_COUNTER)
    a, meta, offs, bars = cp.load_fft_trace(cp.REAL_FFT_TRACES[10])
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, meta, offs)
    st = oc.tile_stats()
    bar = meta == C.META_BARRIER
    assert int(bar.sum()) == 16 * 7 and np.all((out[bar] & 3) == C.LVL_SYNC)
    bt = barrier_times(meta, out, offs)
    assert bt.shape == (16, 7) and np.all(bt == bt[0])
    assert np.all(np.diff(bt[0].astype(np.int64)) >= 0)
    assert np.all((out[bar] >> 2).reshape(16, 7).min(axis=0) == 0)      # the last arrival waits for nobody
    core = po.core_model(meta, out, offs, cfg.frequency_ghz)
    np.testing.assert_array_equal(core[:, C.CORE_STATS.index("time_ps")], st[:, C.TILE_STATS.index("clock_ps")])
    assert np.all(core[:, C.CORE_STATS.index("sync_instructions")] <= 7)
    # accesses only: the same program without its barriers runs differently
    a2, m2, o2, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[10], barriers=False)
    oc2 = po.OracleCoherent(cfg)
    oc2.run(a2, m2, o2)
    assert not np.array_equal(oc2.tile_stats()[:, 0], st[:, 0])
    # barrier traces are released by the whole run only, not quantum by quantum
    oc3 = po.OracleCoherent(cfg)
    oc3.begin(a, meta, offs)
    with pytest.raises(Exception):
        oc3.quantum(0)


@pytest.mark.gpu
@pytest.mark.parametrize("m,barriers", [(10, True), (10, False), (14, True)])
def test_gpu_replays_real_fft(m, barriers):
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev, to_np
    torch = torch_dev()
    a, meta, offs, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[m], barriers=barriers)
    cfg = C.default_config(16, net_model=C.NET_EMESH_HOP_COUNTER)
    be = B.Backend(cfg)
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_run(to_dev(torch, a, torch.int64), to_dev(torch, meta, torch.int32), offs, out)
    st, cc, _ = be.coherent_stats()
    oc = po.OracleCoherent(cfg)
    ref = oc.run(a, meta, offs)
    np.testing.assert_array_equal(to_np(out, np.uint64), ref)
    np.testing.assert_array_equal(st, oc.tile_stats())
    np.testing.assert_array_equal(cc, oc.cache_counters())
    np.testing.assert_array_equal(be.noc_counters(), oc.net_counters())

    if barriers:
        be.core_model_run(to_dev(torch, meta, torch.int32), offs, out)
        np.testing.assert_array_equal(be.core_stats(), po.core_model(meta, ref, offs, cfg.frequency_ghz))


@pytest.mark.gpu
def test_gpu_barrier_trace_needs_whole_run():
    """gg_coherent_quantum (per-quantum / multi-rank driving) rejects a trace
    with BARRIER records: the release is gg_coherent_run's quantum-end rule."""
    from graphite_amd import backend as B
    from tests.gpu_util import torch_dev, to_dev
    torch = torch_dev()
    a, meta, offs, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[10])
    be = B.Backend(C.default_config(16, net_model=C.NET_EMESH_HOP_COUNTER))
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_begin(to_dev(torch, a, torch.int64), to_dev(torch, meta, torch.int32), offs, out)
    with pytest.raises(B.GGError):
        be.coherent_quantum(0)


def with_barriers(a, m, offs, every):
    """The hotspot trace with a BARRIER record after every `every` accesses of each tile."""
    A, M = [], []
    for t in range(len(offs) - 1):
        s, e = int(offs[t]), int(offs[t + 1])
        pos = np.arange(every, e - s, every)
        A.append(np.insert(a[s:e], pos, np.uint64(0)))
        M.append(np.insert(m[s:e], pos, np.uint32(C.META_BARRIER)))
    o = np.concatenate([[0], np.cumsum([len(x) for x in A])]).astype(np.uint64)
    return np.concatenate(A), np.concatenate(M), o


@pytest.mark.parametrize("T,N,net,K", [(16, 300, C.NET_EMESH_HOP_COUNTER, 1), (64, 200, C.NET_EMESH_HOP_BY_HOP, 8)])
def test_oracle_barriers_on_hotspot(T, N, net, K):
    from oracle import pyoracle as po
    a, m, o = po.gen_trace(T, N, hot_lines=16)
    a, m, o = with_barriers(a, m, o, N // 4)
    cfg = C.default_config(T, num_shards=K, net_model=net)
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, m, o)
    bt = barrier_times(m, out, o)
    assert bt.shape == (T, 3) and np.all(bt == bt[0])


@pytest.mark.gpu
@pytest.mark.parametrize("T,N,net,K", [(16, 300, C.NET_EMESH_HOP_COUNTER, 1), (64, 200, C.NET_EMESH_HOP_BY_HOP, 8),
                                       (256, 120, C.NET_EMESH_HOP_COUNTER, 8), (256, 100, C.NET_EMESH_HOP_BY_HOP, 8)])
def test_gpu_barriers_on_hotspot(T, N, net, K):
    """BARRIER records through the persistent small-mesh kernel (<= 64 tiles)
    and the per-step launches (256 tiles), closed-form and hop-by-hop networks:
    bit-exact against the oracle."""
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev, to_np
    torch = torch_dev()
    a, m, o = po.gen_trace(T, N, hot_lines=16)
    a, m, o = with_barriers(a, m, o, N // 4)
    cfg = C.default_config(T, num_shards=K, net_model=net)
    be = B.Backend(cfg)
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_run(to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32), o, out)
    st, cc, _ = be.coherent_stats()
    oc = po.OracleCoherent(cfg)
    ref = oc.run(a, m, o)
    np.testing.assert_array_equal(to_np(out, np.uint64), ref)
    np.testing.assert_array_equal(st, oc.tile_stats())
    np.testing.assert_array_equal(cc, oc.cache_counters())
    np.testing.assert_array_equal(be.noc_counters(), oc.net_counters())


@pytest.mark.gpu
@pytest.mark.parametrize("kern", [0, 1, 2])       # streaming, sharded generic, sharded lean
def test_gpu_private_mode_rejects_barriers(kern):
    """The private-cache batch has no barriers: a BARRIER record (the FFT
    trace loaded with barriers=True) is reported as GG_ERR_UNSUPPORTED by the
    next counter read instead of being replayed as a WRITE to address 0; the
    same trace without them replays normally.  gg_split_accesses rejects
    BARRIER records in its access trace too."""
    from graphite_amd import backend as B
    from tests.gpu_util import torch_dev, to_dev
    torch = torch_dev()
    for barriers in (True, False):
        a, meta, offs, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[10], barriers=barriers)
        cfg = C.default_config(16)
        cfg.replay_kernel = kern
        be = B.Backend(cfg)
        r = torch.zeros(len(a), dtype=torch.int32, device="cuda")
        be.cache_access_batch(to_dev(torch, a, torch.int64), to_dev(torch, meta, torch.int32), offs, r)
        if barriers:
            with pytest.raises(B.GGError, match="BARRIER"):
                be.cache_counters()
        else:
            assert int(be.cache_counters()[:, 0, C.CACHE_COUNTERS.index("accesses")].sum()) == len(a)
    a, meta, offs, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[10], barriers=True)
    size = torch.full((len(a),), 8, dtype=torch.int32, device="cuda")
    with pytest.raises(B.GGError, match="BARRIER"):
        B.split_accesses(to_dev(torch, a, torch.int64), size, to_dev(torch, meta, torch.int32), offs)
