"""Trace capture front end (BASELINE configs[0]): ctypes binding of
libgg_capture.so (include/graphite_capture.h), and the loader of the traces
of the reference's own FFT program captured by tools/fft_trace
(load_fft_trace, REAL_FFT_TRACES).

capture_fft(m, p) runs the source-instrumented six-step FFT of 2^m points on p
threads and returns its per-thread traces in the gg_trace layout (addr u64,
meta u32, tile offsets) plus the transform's output, so a caller can check the
captured program computed a correct FFT before simulating its memory trace.
The reference captures with Pin (pin/lite/memory_modeling.cc:13-89), which is
not available; graphite_amd/capture/fft_capture.cpp documents the mapping.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgg_capture.so")
_lib = None

EXPORTS = ["gg_fft_capture_create", "gg_fft_capture_counts", "gg_fft_capture_copy",
           "gg_fft_capture_output", "gg_fft_capture_input", "gg_fft_capture_destroy"]


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError("%s is not built (make -C graphite_amd/capture)" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        lib.gg_fft_capture_create.restype = ctypes.c_void_p
        lib.gg_fft_capture_create.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        for f in ("gg_fft_capture_counts", "gg_fft_capture_copy", "gg_fft_capture_output",
                  "gg_fft_capture_destroy"):
            getattr(lib, f).restype = None
        lib.gg_fft_capture_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.gg_fft_capture_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.gg_fft_capture_output.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.gg_fft_capture_input.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
        lib.gg_fft_capture_input.restype = None
        lib.gg_fft_capture_destroy.argtypes = [ctypes.c_void_p]
        _lib = lib
    return _lib


def capture_fft(m, p):
    """-> (addr u64[n], meta u32[n], offsets u64[p+1], X complex128[2^m])."""
    lib = load()
    h = lib.gg_fft_capture_create(m, p)
    if not h:
        raise ValueError("bad FFT capture arguments: m=%d p=%d (m even, p a power of two <= 2^(m/2))" % (m, p))
    try:
        counts = np.zeros(p, np.uint64)
        lib.gg_fft_capture_counts(h, counts.ctypes.data)
        n = int(counts.sum())
        addr = np.zeros(n, np.uint64)
        meta = np.zeros(n, np.uint32)
        lib.gg_fft_capture_copy(h, addr.ctypes.data, meta.ctypes.data)
        out = np.zeros(2 << m, np.float64)
        lib.gg_fft_capture_output(h, out.ctypes.data)
    finally:
        lib.gg_fft_capture_destroy(h)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    return addr, meta, offs, out[0::2] + 1j * out[1::2]


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


def fft_input(m):
    x = np.zeros(2 << m, np.float64)
    load().gg_fft_capture_input(m, x.ctypes.data)
    return x[0::2] + 1j * x[1::2]
