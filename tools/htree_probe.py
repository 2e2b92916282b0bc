#!/usr/bin/env python3
"""Cost of one history-tree request on the GPU (gg_queue_delay_batch: one
wave, LDS image) by stream shape.  Prints ns per request."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def stream(n, back, seed=1):
    rng = np.random.default_rng(seed)
    base = np.cumsum(rng.integers(0, 12, n)).astype(np.int64) + 5000
    t = base.copy()
    m = rng.random(n) < back
    t[m] -= rng.integers(0, 4000, int(m.sum()))
    return np.maximum(t, 0).astype(np.uint64), rng.integers(1, 10, n).astype(np.uint64)


def main():
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    torch.cuda.init()
    n = 200000
    for ms in (16, 100):
        for an in (0, 1):
            for back in (0.0, 0.3):
                t, p = stream(n, back)
                be = B.Backend(C.default_config(4, max_list_size=ms, analytical_enabled=an))
                be.queue_delay_batch(t[:1000], p[:1000])
                t0 = time.perf_counter()
                be.queue_delay_batch(t, p)
                dt = time.perf_counter() - t0
                print("max_size %3d analytical %d backward %.1f: %.0f ns per request" % (ms, an, back, dt / n * 1e9),
                      flush=True)
                be.close()


if __name__ == "__main__":
    main()
