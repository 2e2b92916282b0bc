"""Traces of the reference's own FFT program (BASELINE configs[0]), captured
by tools/fft_trace (the reference's tests/benchmarks/fft/fft.C compiled in
place with compiler-inserted access hooks): the committed
fixtures and the -m20 capture build() writes, and their loader.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

ROOT = os.path.dirname(HERE)
# the reference's own FFT (tests/benchmarks/fft/fft.C) captured by tools/fft_trace:
# small committed fixtures, and the configs[0]-size -m20 trace build() writes
REAL_FFT_TRACES = {10: os.path.join(ROOT, "tests", "golden", "fft_real_p16_m10.npz"),
                   14: os.path.join(ROOT, "tests", "golden", "fft_real_p16_m14.npz"),
                   20: os.path.join(ROOT, "tools", "fft_trace", "out", "fft_p16_m20.npz")}


def load_fft_trace(path, barriers=True):
    """A captured SPLASH-2 FFT trace (tools/fft_trace/make_traces.py) ->
    (addr u64[n], meta u32[n], tile_offsets u64[p+1], bars), bars = per tile
    the positions of its BARRIER calls among its accesses.  barriers=True puts
    a GG_META_BARRIER record (address 0) into the tile's trace at each of them,
    so the coherent run models the barrier waits; False: accesses only."""
    z = np.load(path, allow_pickle=False)
    addr = np.cumsum(z["addr_delta"]).astype(np.uint64)
    meta = np.ascontiguousarray(z["meta"], np.uint32)
    offs = np.ascontiguousarray(z["tile_offsets"], np.uint64)
    b, bo = z["barriers"], z["barrier_offsets"]
    bars = [np.asarray(b[int(bo[t]):int(bo[t + 1])], np.uint64) for t in range(len(bo) - 1)]
    if barriers and sum(len(x) for x in bars):
        A, M = [], []
        for t in range(len(offs) - 1):
            s, e = int(offs[t]), int(offs[t + 1])
            pos = bars[t].astype(np.int64)
            A.append(np.insert(addr[s:e], pos, np.uint64(0)))
            M.append(np.insert(meta[s:e], pos, np.uint32(0xFFFFFFFF)))
        addr, meta = np.concatenate(A), np.concatenate(M)
        offs = np.concatenate([[0], np.cumsum([len(x) for x in A])]).astype(np.uint64)
    return addr, meta, offs, bars
