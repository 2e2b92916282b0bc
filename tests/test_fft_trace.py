"""configs[0] on the reference's own program: tests/benchmarks/fft/fft.C
(-p16) captured by tools/fft_trace (TSan access hooks + the PARMACS macros of
tools/fft_trace/parmacs.h, standing in for Graphite's Pin front end,
pin/lite/memory_modeling.cc:13-89).  The committed fixtures
tests/golden/fft_real_p16_m{10,14}.npz were written by
tools/fft_trace/make_traces.py; when the reference is mounted (this container)
the m10 capture is redone and must equal the fixture.  The GPU replays the
traces in Mode C bit-exact against the oracle.  The traces' BARRIER positions
are kept but not modelled by the replayer."""
import os

import numpy as np
import pytest

from graphite_amd import capture as cp
from graphite_amd import config as C
from tests.coherent_util import check_invariants

REF = os.environ.get("GRAPHITE_REFERENCE", "/root/reference")


@pytest.mark.parametrize("m", [10, 14])
def test_fixture_structure(m):
    a, meta, offs, bars = cp.load_fft_trace(cp.REAL_FFT_TRACES[m])
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
    got, ref = cp.load_fft_trace(out), cp.load_fft_trace(cp.REAL_FFT_TRACES[10])
    for x, y in zip(got[:3], ref[:3]):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(got[3], ref[3]):
        np.testing.assert_array_equal(x, y)


def test_oracle_simulates_real_fft():
    from oracle import pyoracle as po
    a, meta, offs, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[10])
    cfg = C.default_config(16, net_model=C.NET_EMESH_HOP_COUNTER)
    oc = po.OracleCoherent(cfg)
    out = oc.run(a, meta, offs)
    check_invariants(oc.tile_stats(), oc.cache_counters(), out, offs)
    assert oc.tile_stats()[:, C.TILE_STATS.index("l2_misses")].sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("m", [10, 14])
def test_gpu_replays_real_fft(m):
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev, to_np
    torch = torch_dev()
    a, meta, offs, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[m])
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
