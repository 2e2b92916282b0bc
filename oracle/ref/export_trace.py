#!/usr/bin/env python3
"""Export a captured FFT trace fixture (tests/golden/fft_real_p16_m*.npz,
accesses only) to the raw files coh_harness.cc reads: <prefix>.addr (u64),
.meta (u32), .offs (u64).  TEST INFRASTRUCTURE ONLY (make_golden.sh)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    from graphite_amd import capture as cp
    src, prefix = sys.argv[1], sys.argv[2]
    a, m, o, _ = cp.load_fft_trace(src, barriers=False)
    a.astype("<u8").tofile(prefix + ".addr")
    m.astype("<u4").tofile(prefix + ".meta")
    o.astype("<u8").tofile(prefix + ".offs")


if __name__ == "__main__":
    main()
