#!/usr/bin/env python3
"""Capture the reference's SPLASH-2 FFT (tests/benchmarks/fft/fft.C) with
tools/fft_trace (see fft_capture_rt.cpp) and store the per-thread traces as a
compressed .npz: per-tile address deltas (int64), meta words, tile offsets and
the barrier positions.  graphite_amd.capture.load_fft_trace reads it.

usage: make_traces.py OUT.npz M [P]   (needs /root/reference; run by
__graft_entry__.build() for the bench's -m20 trace, and by hand for the
committed fixtures tests/golden/fft_real_p16_m{10,14}.npz)."""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def read_ggft(path):
    b = open(path, "rb").read()
    h = np.frombuffer(b[:12], np.uint32)
    if int(h[0]) != 0x54464747 or int(h[1]) != 1:
        raise ValueError("%s: not a GGFT v1 trace" % path)
    P = int(h[2])
    cnt = np.frombuffer(b[12:12 + 8 * P], np.uint64).astype(np.int64)
    nb = np.frombuffer(b[12 + 8 * P:12 + 16 * P], np.uint64).astype(np.int64)
    off = 12 + 16 * P
    A, M, B = [], [], []
    for t in range(P):
        A.append(np.frombuffer(b[off:off + 8 * cnt[t]], np.uint64)); off += 8 * cnt[t]
        M.append(np.frombuffer(b[off:off + 4 * cnt[t]], np.uint32)); off += 4 * cnt[t]
    for t in range(P):
        B.append(np.frombuffer(b[off:off + 8 * nb[t]], np.uint64)); off += 8 * nb[t]
    return A, M, B


def main():
    out, m = sys.argv[1], int(sys.argv[2])
    p = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    ref = os.environ.get("GRAPHITE_REFERENCE", "/root/reference")
    subprocess.check_call(["make", "-s", "-C", HERE, "REF=" + ref])
    raw = os.path.join(HERE, "out", "fft_p%d_m%d.ggft" % (p, m))
    env = dict(os.environ, GG_FFT_TRACE_OUT=raw)
    with open(os.devnull, "w") as dn:
        subprocess.check_call([os.path.join(HERE, "out", "fft_capture"), "-p%d" % p, "-m%d" % m], env=env, stdout=dn)
    A, M, B = read_ggft(raw)
    offs = np.concatenate([[0], np.cumsum([len(a) for a in A])]).astype(np.uint64)
    addr = np.concatenate(A)
    delta = np.diff(addr.astype(np.int64), prepend=np.int64(0))
    boffs = np.concatenate([[0], np.cumsum([len(b) for b in B])]).astype(np.uint64)
    np.savez_compressed(out, addr_delta=delta, meta=np.concatenate(M), tile_offsets=offs,
                        barriers=np.concatenate(B) if B else np.zeros(0, np.uint64), barrier_offsets=boffs,
                        m=np.int64(m), p=np.int64(p),
                        source=np.array("tests/benchmarks/fft/fft.C -p%d -m%d, tools/fft_trace capture" % (p, m)))
    os.remove(raw)
    print("%s: %d records, %d tiles, %d barriers per tile" % (out, len(addr), p, len(B[0]) if B else 0))


if __name__ == "__main__":
    main()
