#!/usr/bin/env python3
"""configs[0]: the reference FFT (tools/fft_trace capture, m in 10 / 14 / 20) through gg_coherent_run once (GG_COH_PROFILE=1 prints the phase profile)."""
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
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    a, meta, offs, _ = cp.load_fft_trace(cp.REAL_FFT_TRACES[m])
    cfg = C.default_config(16, net_model=C.NET_EMESH_HOP_COUNTER)
    be = B.Backend(cfg)
    addr = torch.from_numpy(a.view(np.int64)).cuda()
    mt = torch.from_numpy(meta.view(np.int32)).cuda()
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    for it in range(runs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        be.coherent_run(addr, mt, offs, out)
        torch.cuda.synchronize()
        print("run %d: %.3f s, %.3g acc/s" % (it, time.perf_counter() - t0, len(a) / (time.perf_counter() - t0)), flush=True)


if __name__ == "__main__":
    main()
