#!/usr/bin/env python3
"""Coherent-mode (Mode C) timing experiment: GPU gg_coherent_run vs the C
oracle on the same hotspot trace.  usage: coh_bench.py T N [K] [hot] [--no-oracle] [--hbh] [--warm] [--no-timing] [--heartbeat]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if "--heartbeat" in sys.argv:            # long oracle runs: a line every 30 s (gpurun's idle watchdog)
        import threading

        def beat():
            while True:
                time.sleep(30)
                print("... %.0f s" % (time.perf_counter() - t_start), flush=True)
        t_start = time.perf_counter()
        threading.Thread(target=beat, daemon=True).start()
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    T, N = int(args[0]), int(args[1])
    K = int(args[2]) if len(args) > 2 else 1
    hot = int(args[3]) if len(args) > 3 else 64
    net = C.NET_EMESH_HOP_BY_HOP if "--hbh" in sys.argv else C.NET_EMESH_HOP_COUNTER
    cfg = C.default_config(T, num_shards=K, net_model=net)
    be = B.Backend(cfg)
    be.set_timing("--no-timing" not in sys.argv)
    addr = torch.empty(T * N, dtype=torch.int64, device="cuda")
    meta = torch.empty(T * N, dtype=torch.int32, device="cuda")
    out = torch.zeros(T * N, dtype=torch.int64, device="cuda")
    B.gen_hotspot_trace(addr, meta, 0, T, N, hot_lines=hot)
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    if "--warm" in sys.argv:
        be.coherent_run(addr, meta, offs, out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    be.coherent_run(addr, meta, offs, out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st, cc, ri = be.coherent_stats()
    print("gpu  %s T=%d N=%d K=%d: %.3f s  %.3g acc/s  quanta %d steps %d msgs %d  clk max %d ns" %
          ("hbh" if net == C.NET_EMESH_HOP_BY_HOP else "hc", T, N, K, dt, T * N / dt, ri[0], ri[1], ri[2] + ri[3], st[:, 0].max() // 1000), flush=True)
    if "--no-oracle" not in sys.argv:
        from oracle import pyoracle as po
        a, m, o = po.gen_trace(T, N, hot_lines=hot)
        oc = po.OracleCoherent(cfg)
        t0 = time.perf_counter()
        ref = oc.run(a, m, o)
        dto = time.perf_counter() - t0
        ok = np.array_equal(out.cpu().numpy().view(np.uint64), ref) and np.array_equal(st, oc.tile_stats())
        print("cpu  oracle 1 thread: %.3f s  %.3g acc/s  bit-exact %s" % (dto, T * N / dto, ok), flush=True)


if __name__ == "__main__":
    main()
