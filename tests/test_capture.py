"""Trace-capture front end (BASELINE configs[0]): the source-instrumented
six-step FFT computes the right transform, its traces have the gg_trace
format and structure, and the coherent oracle simulates them (CPU)."""
import numpy as np
import pytest

from graphite_amd import capture as cp
from graphite_amd import config as C
from tests.coherent_util import check_invariants


@pytest.mark.parametrize("m,p", [(2, 1), (4, 2), (6, 8), (8, 4), (10, 16), (12, 16)])
def test_captured_fft_is_correct(m, p):
    a, meta, offs, X = cp.capture_fft(m, p)
    ref = np.fft.fft(cp.fft_input(m))
    assert np.abs(X - ref).max() <= 1e-9 * np.abs(ref).max()
    assert len(offs) == p + 1 and offs[-1] == len(a) == len(meta)


def test_trace_format_and_structure():
    m, p = 8, 4
    a, meta, offs, _ = cp.capture_fft(m, p)
    n = np.diff(offs.astype(np.int64))
    assert np.all(n == n[0])                       # threads do equal work in every phase
    assert np.all(a % 8 == 0) and np.all(a < (1 << 48))
    assert np.all((meta >> 31) == 0)               # bit 31 reserved
    w = (meta & 1).astype(bool)
    # every store is to an address the thread also loads (in-place FFT, transposes write what others read)
    assert 0.3 < w.mean() < 0.6
    # the shared matrix is touched by every thread: sharing across tiles exists
    lines = [set((a[offs[t]:offs[t + 1]] >> 6).tolist()) for t in range(p)]
    assert len(lines[0] & lines[1]) > 0
    # deterministic
    a2, meta2, offs2, _ = cp.capture_fft(m, p)
    assert np.array_equal(a, a2) and np.array_equal(meta, meta2) and np.array_equal(offs, offs2)


def test_bad_arguments_rejected():
    for m, p in ((3, 1), (8, 3), (4, 8), (0, 1)):
        with pytest.raises(ValueError):
            cp.capture_fft(m, p)


def test_oracle_simulates_fft_trace():
    """configs[0] shape at small size: MSI directory + emesh_hop_counter on
    the FFT trace; every access completes and the run is deterministic."""
    from oracle import pyoracle as po
    m, p = 6, 4
    a, meta, offs, _ = cp.capture_fft(m, p)
    cfg = C.default_config(p, net_model=C.NET_EMESH_HOP_COUNTER)
    o1 = po.OracleCoherent(cfg)
    out1 = o1.run(a, meta, offs)
    o2 = po.OracleCoherent(cfg)
    out2 = o2.run(a, meta, offs)
    assert np.array_equal(out1, out2) and np.array_equal(o1.tile_stats(), o2.tile_stats())
    check_invariants(o1.tile_stats(), o1.cache_counters(), out1, offs, per_tile_expected=int(offs[1] - offs[0]))
    st = o1.tile_stats()
    assert st[:, C.TILE_STATS.index("l2_misses")].sum() > 0
