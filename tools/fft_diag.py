#!/usr/bin/env python3
"""configs[0] per-step diagnostics: the reference FFT trace (first PER records
of each tile, barriers dropped) through per-step launches (GG_COH_NO_PERSIST)
of the diagnostics build, so GG_COH_TRACE / tools/coh_trace.py see its steps.
usage: fft_diag.py [PER]  (GG_LIB = the diagnostics build)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from graphite_amd import capture as cp
    per = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    a, m, o, _ = cp.load_fft_trace(os.path.join(root, "tools/fft_trace/out/fft_p16_m20.npz"), barriers=False)
    T = len(o) - 1
    A = np.concatenate([a[int(o[t]):int(o[t]) + per] for t in range(T)])
    M = np.concatenate([m[int(o[t]):int(o[t]) + per] for t in range(T)])
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(per)
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_COUNTER)
    be = B.Backend(cfg)
    addr = torch.from_numpy(A.astype(np.int64)).cuda()
    meta = torch.from_numpy(M.view(np.int32)).cuda()
    out = torch.zeros(len(A), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    be.coherent_run(addr, meta, offs, out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st, cc, ri = be.coherent_stats()
    print("fft prefix %d x %d: %.3f s, %.3g acc/s, steps %d, %.2f us/step" % (T, per, dt, len(A) / dt, ri[1], 1e6 * dt / max(ri[1], 1)))


if __name__ == "__main__":
    main()
