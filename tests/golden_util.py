"""Loader for the fixtures in tests/golden/ (written by oracle/ref/make_golden.sh
from the reference's own CacheSet / replacement policies / line-info classes,
IntervalTree and QueueModelMG1, compiled from /root/reference)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load(name, dtype):
    return np.fromfile(os.path.join(GOLDEN, name), dtype=dtype)


POLICY = {"lru": 0, "round_robin": 1}


# Fixture result encoding (oracle/ref/ref_harness.cc, enum R_*): level in bits
# 0-1 (0 = L1-D hit, 1 = L2 hit, 2 = directory), UPGRADE 4, L1_EVICT 8,
# L2_EVICT 16, L2_EVICT_DIRTY 32, L2_EVICT_INV_L1 64.  The ABI result word
# (include/graphite_gpu.h GG_RES_*) carries the same facts one flag per 4-bit
# field, plus GG_RES_L1_INVAL, which the fixtures pin through the L1-D
# tag-write counter instead (its only counter effect).
def compact_code(res):
    from graphite_amd import config as C
    r = np.asarray(res, np.uint32)
    level = np.where(r & C.RES_L2_MISS, 2, np.where(r & C.RES_L1_MISS, 1, 0)).astype(np.uint8)
    out = level.copy()
    for bit, f in ((4, C.RES_UPGRADE), (8, C.RES_L1_EVICT), (16, C.RES_L2_EVICT),
                   (32, C.RES_L2_EVICT_DIRTY), (64, C.RES_L2_EVICT_INV_L1)):
        out |= np.where(r & f, bit, 0).astype(np.uint8)
    return out
