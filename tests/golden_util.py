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


def coh_manifest():
    with open(os.path.join(GOLDEN, "coh_manifest.json")) as f:
        return json.load(f)


def coh_mosi_manifest():
    with open(os.path.join(GOLDEN, "coh_mosi_manifest.json")) as f:
        return json.load(f)


def coh_shl2_manifest():
    with open(os.path.join(GOLDEN, "coh_shl2_manifest.json")) as f:
        return json.load(f)


def coh_mesi_sh_manifest():
    with open(os.path.join(GOLDEN, "coh_mesi_manifest.json")) as f:
        return json.load(f)


def coh_case(name, m):
    """(cfg, addr, meta, offsets, expected dict) of a coherent-mode fixture written
    by oracle/ref/coh_harness.cc (the reference's MSI controllers; "mosi_*"
    names: coh_harness_mosi, the MOSI controllers, plus their event counters;
    "shl2_*": coh_harness_shl2, the shared-L2 MSI controllers; "mesi_*":
    coh_harness_shl2_mesi, the shared-L2 MESI controllers)."""
    from graphite_amd import config as C
    from oracle import pyoracle as po
    T, N = m["tiles"], m["per_tile"]
    kw = dict(num_shards=m["num_shards"], net_model=C.NET_EMESH_HOP_COUNTER if m["net"] == 1 else C.NET_MAGIC)
    if m["dir_entries"]:
        kw.update(dir_total_entries=m["dir_entries"], dir_assoc=m["dir_assoc"])
    kw.update(l2_assoc=m.get("l2_assoc", 8))
    mosi = name.startswith("mosi_")
    if mosi:
        kw.update(protocol=C.PROTO_MOSI)
    if name.startswith("shl2_"):                     # coh_harness_shl2: pr_l1_sh_l2_msi
        kw.update(protocol=C.PROTO_SHL2_MSI)
    if name.startswith("mesi_"):                     # coh_harness_shl2_mesi: pr_l1_sh_l2_mesi
        kw.update(protocol=C.PROTO_SHL2_MESI)
    cfg = C.default_config(T, **kw)
    wl = m.get("workload", "hotspot")
    if wl == "stress":
        a, meta, o = po.gen_stress_trace(T, N)
    elif wl.startswith("fft_real_"):                 # configs[0]: the captured reference FFT, accesses only
        from graphite_amd import capture as cp
        a, meta, o, _ = cp.load_fft_trace(os.path.join(GOLDEN, wl + ".npz"), barriers=False)
    else:
        a, meta, o = po.gen_trace(T, N, hot_lines=m["hot_lines"])
    exp = {"out": load("coh_%s_out.u64" % name, np.uint64),
           "stats": load("coh_%s_stats.u64" % name, np.uint64).reshape(T, 32),
           "cache": load("coh_%s_cache.u64" % name, np.uint64).reshape(T, 2, 12),
           "net": load("coh_%s_net.u64" % name, np.uint64).reshape(T, 3),
           "quanta": m["quanta"], "steps": m["steps"]}
    if mosi:
        exp["proto"] = load("coh_%s_proto.u64" % name, np.uint64).reshape(T, 32)
    return cfg, a, meta, o, exp


NET3 = ["packets_sent", "packets_received", "total_latency_ps"]
