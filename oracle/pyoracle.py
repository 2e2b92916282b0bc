"""ctypes view of the C oracle (oracle/gg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  The product (graphite_amd/)
never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

from graphite_amd.config import (GGConfig, NUM_CACHE_COUNTERS, NUM_NET_COUNTERS, NUM_TILE_STATS,
                                 NUM_RUN_INFO, CMSG_DTYPE, BROADCAST)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")


def build(force=False):
    """Compile the oracle with gcc (plain C99, -ffp-contract=off)."""
    src = os.path.join(HERE, "gg_oracle.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        L.oracle_splitmix64_at.restype = ctypes.c_uint64
        L.oracle_splitmix64_at.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_gen_uniform.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint32, ctypes.c_uint32, _u64p, _u32p]
        L.oracle_cache_create.restype = vp
        L.oracle_cache_create.argtypes = [ctypes.POINTER(GGConfig)]
        L.oracle_cache_destroy.argtypes = [vp]
        L.oracle_cache_run.restype = ctypes.c_int
        L.oracle_cache_run.argtypes = [vp, _u64p, _u32p, _u64p, ctypes.c_uint32, ctypes.c_uint32, vp, vp]
        L.oracle_cache_counters.argtypes = [vp, _u64p]
        L.oracle_cache_get_line_info.argtypes = [vp, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64, vp]
        L.oracle_cache_set_line_info.argtypes = [vp, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64, vp]
        L.oracle_cache_access_line.argtypes = [vp, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
        L.oracle_cache_insert_line.argtypes = [vp, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64, vp,
                                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64), vp]
        L.oracle_htree_create.restype = vp
        L.oracle_htree_create.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.oracle_htree_destroy.argtypes = [vp]
        L.oracle_qmodel_create.restype = vp
        L.oracle_qmodel_create.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.oracle_htree_delay.restype = ctypes.c_uint64
        L.oracle_htree_delay.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_htree_analytical_requests.restype = ctypes.c_uint64
        L.oracle_htree_analytical_requests.argtypes = [vp]
        L.oracle_noc_create.restype = vp
        L.oracle_noc_create.argtypes = [ctypes.POINTER(GGConfig)]
        L.oracle_noc_destroy.argtypes = [vp]
        L.oracle_noc_route.restype = ctypes.c_int
        L.oracle_noc_route.argtypes = [vp, ctypes.c_uint64, _u32p, _u32p, _u32p, _u64p, _u64p, _u64p, _u64p]
        L.oracle_noc_route_tree.restype = ctypes.c_int
        L.oracle_noc_route_tree.argtypes = [vp, ctypes.c_uint64, _u32p, _u32p, _u32p, _u64p] + [_u64p] * 6
        L.oracle_noc_counters.argtypes = [vp, _u64p]
        L.oracle_split_lines.restype = ctypes.c_uint32
        L.oracle_split_lines.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _u64p, ctypes.c_uint32]
        L.oracle_split_accesses.restype = ctypes.c_uint64
        L.oracle_split_accesses.argtypes = [_u64p, _u32p, _u32p, _u64p, ctypes.c_uint32, ctypes.c_uint32, _u64p, vp, vp]
        L.oracle_combine_accesses.argtypes = [_u64p, _u64p, ctypes.c_uint64, _u64p, _u32p]
        L.oracle_core_model.argtypes = [_u32p, _u64p, _u64p, ctypes.c_uint32, ctypes.c_double, _u64p]
        L.oracle_core_model.restype = None
        L.oracle_iocoom.argtypes = [vp, vp, _u64p, _u64p, _u32p, _u64p, _u64p, ctypes.c_uint32, ctypes.c_double, _u64p]
        L.oracle_iocoom.restype = ctypes.c_int
        L.oracle_gen_hotspot.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u64p, _u32p]
        L.oracle_gen_stress.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u64p, _u32p]
        L.oracle_shard_map.restype = ctypes.c_int
        L.oracle_shard_map.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _u32p]
        L.oracle_coh_run_parallel.restype = ctypes.c_int
        L.oracle_coh_run_parallel.argtypes = [ctypes.POINTER(GGConfig), ctypes.c_int, _u64p, _u32p, _u64p, vp, vp, vp,
                                              vp, vp]
        L.oracle_coh_create.restype = vp
        L.oracle_coh_create.argtypes = [ctypes.POINTER(GGConfig)]
        L.oracle_coh_set_threads.restype = ctypes.c_int
        L.oracle_coh_set_threads.argtypes = [vp, ctypes.c_int]
        L.oracle_coh_destroy.argtypes = [vp]
        L.oracle_coh_begin.restype = ctypes.c_int
        L.oracle_coh_begin.argtypes = [vp, _u64p, _u32p, _u64p, vp]
        L.oracle_coh_quantum.restype = ctypes.c_int
        L.oracle_coh_quantum.argtypes = [vp, ctypes.c_uint64, _u64p]
        L.oracle_coh_export.restype = ctypes.c_uint64
        L.oracle_coh_export.argtypes = [vp, vp, ctypes.c_uint64]
        L.oracle_coh_import.restype = ctypes.c_int
        L.oracle_coh_import.argtypes = [vp, vp, ctypes.c_uint64]
        L.oracle_coh_run.restype = ctypes.c_int
        L.oracle_coh_run.argtypes = [vp, _u64p, _u32p, _u64p, vp]
        for n in ("oracle_coh_tile_stats", "oracle_coh_cache_counters", "oracle_coh_net_counters",
                  "oracle_coh_run_info", "oracle_coh_miss_types", "oracle_coh_proto_stats", "oracle_cache_miss_types"):
            getattr(L, n).argtypes = [vp, _u64p]
            getattr(L, n).restype = None
        _lib = L
    return _lib


class LineInfo(ctypes.Structure):
    _fields_ = [("tag", ctypes.c_uint64), ("cstate", ctypes.c_uint32), ("cached_loc", ctypes.c_uint32)]


def gen_uniform(tile, first, n, lines_log2=15, base_shift=26):
    addr = np.empty(n, np.uint64)
    meta = np.empty(n, np.uint32)
    lib().oracle_gen_uniform(tile, first, n, lines_log2, base_shift, addr, meta)
    return addr, meta


def gen_hotspot(tile, first, n, lines_log2=15, base_shift=26, hot_lines=64, hot_frac256=51):
    addr = np.empty(n, np.uint64)
    meta = np.empty(n, np.uint32)
    lib().oracle_gen_hotspot(tile, first, n, lines_log2, base_shift, hot_lines, hot_frac256, addr, meta)
    return addr, meta


def gen_stress(tile, first, n, num_tiles, lines_log2=15, base_shift=26, pool_lines=4096, pool_frac256=77):
    """configs[4] stress records of one tile (oracle_gen_stress)."""
    addr = np.zeros(n, np.uint64)
    meta = np.zeros(n, np.uint32)
    lib().oracle_gen_stress(tile, first, n, lines_log2, base_shift, num_tiles, pool_lines, pool_frac256, addr, meta)
    return addr, meta


def gen_stress_trace(tiles, per_tile, **kw):
    """Tile-major configs[4] stress trace of `tiles` tiles x `per_tile` records + offsets."""
    parts = [gen_stress(t, 0, per_tile, tiles, **kw) for t in range(tiles)]
    addr = np.concatenate([p[0] for p in parts]) if parts else np.zeros(0, np.uint64)
    meta = np.concatenate([p[1] for p in parts]) if parts else np.zeros(0, np.uint32)
    offs = np.arange(tiles + 1, dtype=np.uint64) * np.uint64(per_tile)
    return addr, meta, offs


def gen_trace(tiles, per_tile, **kw):
    """Tile-major hotspot trace of `tiles` tiles x `per_tile` records + offsets."""
    parts = [gen_hotspot(t, 0, per_tile, **kw) for t in range(tiles)]
    addr = np.concatenate([p[0] for p in parts]) if parts else np.zeros(0, np.uint64)
    meta = np.concatenate([p[1] for p in parts]) if parts else np.zeros(0, np.uint32)
    offs = np.arange(tiles + 1, dtype=np.uint64) * np.uint64(per_tile)
    return addr, meta, offs


def coherent_run_parallel(cfg, addr, meta, tile_offsets, threads):
    """The coherent run as one oracle context per logical shard, the shards'
    quanta on `threads` OpenMP threads (the all-core CPU baseline); returns
    (access words, tile stats, cache counters, net counters, run info)."""
    T = cfg.num_tiles
    out = np.zeros(len(addr), np.uint64)
    st = np.zeros((T, NUM_TILE_STATS), np.uint64)
    cc = np.zeros((T, 2, NUM_CACHE_COUNTERS), np.uint64)
    nc = np.zeros((T, NUM_NET_COUNTERS), np.uint64)
    ri = np.zeros(NUM_RUN_INFO, np.uint64)
    rc = lib().oracle_coh_run_parallel(ctypes.byref(cfg), threads, np.ascontiguousarray(addr, np.uint64),
                                       np.ascontiguousarray(meta, np.uint32),
                                       np.ascontiguousarray(tile_offsets, np.uint64), out.ctypes.data,
                                       st.ctypes.data, cc.ctypes.data, nc.ctypes.data, ri.ctypes.data)
    if rc != 0:
        raise RuntimeError("coherent oracle (parallel) rc=%d" % rc)
    return out, st, cc, nc, ri


def shard_map(num_tiles, num_shards):
    """tile -> logical shard of the oracle (hop_by_hop.cc:367-433 restated)."""
    out = np.zeros(num_tiles, np.uint32)
    if lib().oracle_shard_map(num_tiles, num_shards, out) != 0:
        raise ValueError("no shard map for %d tiles in %d shards" % (num_tiles, num_shards))
    return out


class OracleCoherent:
    """Coherent (Mode C) run: MSI directory + DRAM + NoC + lax-barrier quanta,
    canonical schedule (oracle/gg_coherent.inc)."""

    def __init__(self, cfg, threads=1):
        """threads > 1: tile-parallel steps (each step's tiles, then the
        hop-by-hop routing stage by stage, on OpenMP threads): the all-core CPU
        baseline, bit-identical to one thread."""
        self.cfg = cfg
        self.h = lib().oracle_coh_create(ctypes.byref(cfg))
        if threads > 1:
            lib().oracle_coh_set_threads(self.h, int(threads))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_coh_destroy(self.h)
            self.h = None

    def run(self, addr, meta, tile_offsets):
        """Whole run (context owns every shard); returns the per-access words."""
        self._keep = (np.ascontiguousarray(addr, np.uint64), np.ascontiguousarray(meta, np.uint32),
                      np.ascontiguousarray(tile_offsets, np.uint64))
        out = np.zeros(len(addr), np.uint64)
        self._out = out
        rc = lib().oracle_coh_run(self.h, *self._keep, out.ctypes.data)
        if rc != 0:
            raise RuntimeError("coherent oracle rc=%d (the reference would abort / deadlock)" % rc)
        return out

    # -- sharded (multi-rank) driving ------------------------------------
    def begin(self, addr, meta, tile_offsets):
        self._keep = (np.ascontiguousarray(addr, np.uint64), np.ascontiguousarray(meta, np.uint32),
                      np.ascontiguousarray(tile_offsets, np.uint64))
        self._out = np.zeros(len(addr), np.uint64)
        rc = lib().oracle_coh_begin(self.h, *self._keep, self._out.ctypes.data)
        if rc != 0:
            raise RuntimeError("coherent oracle begin rc=%d" % rc)
        return self._out

    def quantum(self, q):
        st = np.zeros(5, np.uint64)
        rc = lib().oracle_coh_quantum(self.h, q, st)
        if rc != 0:
            raise RuntimeError("coherent oracle quantum rc=%d" % rc)
        return {"steps": int(st[0]), "boundary_msgs": int(st[1]), "min_next_ps": int(st[2]),
                "active_tiles": int(st[3]), "blocked_tiles": int(st[4])}

    def export(self, cap):
        buf = np.zeros(cap, CMSG_DTYPE)
        n = lib().oracle_coh_export(self.h, buf.ctypes.data, cap)
        if n == 0xFFFFFFFFFFFFFFFF:
            raise RuntimeError("export buffer too small")
        return buf[:n]

    def import_(self, msgs):
        msgs = np.ascontiguousarray(msgs, CMSG_DTYPE)
        rc = lib().oracle_coh_import(self.h, msgs.ctypes.data, len(msgs))
        if rc != 0:
            raise RuntimeError("coherent oracle import rc=%d" % rc)

    def _get(self, fn, shape):
        out = np.zeros(int(np.prod(shape)), np.uint64)
        getattr(lib(), fn)(self.h, out)
        return out.reshape(shape)

    def tile_stats(self):
        return self._get("oracle_coh_tile_stats", (self.cfg.num_tiles, NUM_TILE_STATS))

    def cache_counters(self):
        return self._get("oracle_coh_cache_counters", (self.cfg.num_tiles, 2, NUM_CACHE_COUNTERS))

    def net_counters(self):
        return self._get("oracle_coh_net_counters", (self.cfg.num_tiles, NUM_NET_COUNTERS))

    def run_info(self):
        return self._get("oracle_coh_run_info", (NUM_RUN_INFO,))

    def miss_types(self):
        return self._get("oracle_coh_miss_types", (self.cfg.num_tiles, 2, 3))

    def proto_stats(self):
        """MOSI event counters [tile][NUM_PROTO_STATS] (zeros under MSI)."""
        return self._get("oracle_coh_proto_stats", (self.cfg.num_tiles, 32))


class OracleCache:
    """Private-mode (decoupled) replay of L1-D/L2 per tile."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.h = lib().oracle_cache_create(ctypes.byref(cfg))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_cache_destroy(self.h)
            self.h = None

    def run(self, addr, meta, tile_offsets, tile_begin=0, tile_end=None, want_evicted=False):
        n = len(addr)
        addr = np.ascontiguousarray(addr, np.uint64)
        meta = np.ascontiguousarray(meta, np.uint32)
        offs = np.ascontiguousarray(tile_offsets, np.uint64)
        res = np.zeros(n, np.uint32)
        ev = np.zeros(n, np.uint64) if want_evicted else None
        tile_end = self.cfg.num_tiles if tile_end is None else tile_end
        rc = lib().oracle_cache_run(self.h, addr, meta, offs, tile_begin, tile_end,
                                    res.ctypes.data, ev.ctypes.data if ev is not None else None)
        if rc != 0:
            raise RuntimeError("oracle: reference would abort (LOG_ASSERT_ERROR), rc=%d" % rc)
        return (res, ev) if want_evicted else res

    def counters(self):
        out = np.zeros(self.cfg.num_tiles * 2 * NUM_CACHE_COUNTERS, np.uint64)
        lib().oracle_cache_counters(self.h, out)
        return out.reshape(self.cfg.num_tiles, 2, NUM_CACHE_COUNTERS)

    def miss_types(self):
        out = np.zeros(self.cfg.num_tiles * 2 * 3, np.uint64)
        lib().oracle_cache_miss_types(self.h, out)
        return out.reshape(self.cfg.num_tiles, 2, 3)

    def get_line_info(self, tile, level, addr, default=None):
        li = default or LineInfo(0xFFFFFFFFFFFFFFFF, 0, 0)
        rc = lib().oracle_cache_get_line_info(self.h, tile, level, addr, ctypes.addressof(li))
        assert rc == 0
        return li

    def set_line_info(self, tile, level, addr, li):
        return lib().oracle_cache_set_line_info(self.h, tile, level, addr, ctypes.addressof(li))

    def access_line(self, tile, level, addr, is_store):
        return lib().oracle_cache_access_line(self.h, tile, level, addr, int(is_store))

    def insert_line(self, tile, level, addr, li):
        ev = ctypes.c_int(0)
        ea = ctypes.c_uint64(0)
        evi = LineInfo(0xFFFFFFFFFFFFFFFF, 0, 0)
        rc = lib().oracle_cache_insert_line(self.h, tile, level, addr, ctypes.addressof(li),
                                            ctypes.byref(ev), ctypes.byref(ea), ctypes.addressof(evi))
        return rc, ev.value, ea.value, evi


class OracleHistoryTree:
    def __init__(self, min_proc=1, max_list_size=100, analytical=True):
        self.h = lib().oracle_htree_create(min_proc, max_list_size, int(analytical))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_htree_destroy(self.h)
            self.h = None

    def delay(self, t, p):
        return lib().oracle_htree_delay(self.h, t, p)

    @property
    def analytical_requests(self):
        return lib().oracle_htree_analytical_requests(self.h)


class OracleQueueModel(OracleHistoryTree):
    """Any QueueModel::create type (queue_model.cc:19-39): qtype = QM_*; aux =
    history_list_no_interleaving (history_list) or basic_moving_avg (basic)."""

    def __init__(self, qtype, aux=0, min_proc=1, max_list_size=100, analytical=True):
        self.h = lib().oracle_qmodel_create(qtype, aux, min_proc, max_list_size, int(analytical))


class OracleNoc:
    def __init__(self, cfg):
        self.cfg = cfg
        self.h = lib().oracle_noc_create(ctypes.byref(cfg))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_noc_destroy(self.h)
            self.h = None

    def route(self, src, dst, length_bits, time_ps):
        n = len(src)
        arr = np.zeros(n, np.uint64)
        zl = np.zeros(n, np.uint64)
        ct = np.zeros(n, np.uint64)
        rc = lib().oracle_noc_route(self.h, n, np.ascontiguousarray(src, np.uint32),
                                    np.ascontiguousarray(dst, np.uint32),
                                    np.ascontiguousarray(length_bits, np.uint32),
                                    np.ascontiguousarray(time_ps, np.uint64), arr, zl, ct)
        if rc != 0:
            raise RuntimeError("oracle noc rc=%d" % rc)
        return arr, zl, ct

    def route_tree(self, src, dst, length_bits, time_ps):
        """Broadcast-tree batch (oracle_noc_route_tree): (arrival, zl, ct) per packet
        and (arrival, zl, ct)[broadcast ordinal, tile] of the broadcast deliveries."""
        n, T = len(src), self.cfg.num_tiles
        dst = np.ascontiguousarray(dst, np.uint32)
        nb = int((dst == BROADCAST).sum())
        o = [np.zeros(n, np.uint64) for _ in range(3)]
        b = [np.zeros(max(nb, 1) * T, np.uint64) for _ in range(3)]
        rc = lib().oracle_noc_route_tree(self.h, n, np.ascontiguousarray(src, np.uint32), dst,
                                         np.ascontiguousarray(length_bits, np.uint32),
                                         np.ascontiguousarray(time_ps, np.uint64), *o, *b)
        if rc != 0:
            raise RuntimeError("oracle noc rc=%d" % rc)
        return o, [x[:nb * T].reshape(nb, T) for x in b]

    def counters(self):
        out = np.zeros(self.cfg.num_tiles * NUM_NET_COUNTERS, np.uint64)
        lib().oracle_noc_counters(self.h, out)
        return out.reshape(self.cfg.num_tiles, NUM_NET_COUNTERS)


def split_accesses(addr, size, meta, tile_offsets, line=64):
    """Multi-line accesses -> (line_addr, line_meta, first, line_tile_offsets) (oracle_split_accesses)."""
    addr = np.ascontiguousarray(addr, np.uint64)
    size = np.ascontiguousarray(size, np.uint32)
    meta = np.ascontiguousarray(meta, np.uint32)
    offs = np.ascontiguousarray(tile_offsets, np.uint64)
    tiles = len(offs) - 1
    first = np.zeros(len(addr) + 1, np.uint64)
    n = lib().oracle_split_accesses(addr, size, meta, offs, tiles, line, first, None, None)
    if n == (1 << 64) - 1:
        raise ValueError("carried gap above 2^30 cycles")
    la = np.zeros(max(n, 1), np.uint64)
    lm = np.zeros(max(n, 1), np.uint32)
    lib().oracle_split_accesses(addr, size, meta, offs, tiles, line, first,
                                la.ctypes.data_as(ctypes.c_void_p), lm.ctypes.data_as(ctypes.c_void_p))
    return la[:n], lm[:n], first, first[offs.astype(np.int64)]


def combine_accesses(line_out, first):
    """Per-access (latency_ps, misses) of a split trace's line results (oracle_combine_accesses)."""
    n = len(first) - 1
    lat = np.zeros(max(n, 1), np.uint64)
    miss = np.zeros(max(n, 1), np.uint32)
    lib().oracle_combine_accesses(np.ascontiguousarray(line_out, np.uint64), np.ascontiguousarray(first, np.uint64),
                                  n, lat, miss)
    return lat[:n], miss[:n]


def core_model(meta, access_out, tile_offsets, frequency_ghz=1.0):
    """[tiles][GG_NUM_CORE_STATS] of the simple core model (oracle_core_model)."""
    offs = np.ascontiguousarray(tile_offsets, np.uint64)
    T = len(offs) - 1
    out = np.zeros(max(T, 1) * 8, np.uint64)
    lib().oracle_core_model(np.ascontiguousarray(meta, np.uint32), np.ascontiguousarray(access_out, np.uint64), offs,
                            T, float(frequency_ghz), out)
    return out[:T * 8].reshape(T, 8)


def iocoom(params, ins, ins_offsets, addr, meta, lat, acc_offsets, frequency_ghz=1.0):
    """[tiles][GG_NUM_IOCOOM_STATS] of the iocoom core model (oracle_iocoom);
    raises ValueError when the instruction and access streams disagree."""
    from graphite_amd.config import INS_DTYPE, NUM_IOCOOM_STATS
    ins = np.ascontiguousarray(ins, INS_DTYPE)
    io = np.ascontiguousarray(ins_offsets, np.uint64)
    ao = np.ascontiguousarray(acc_offsets, np.uint64)
    T = len(io) - 1
    out = np.zeros(max(T, 1) * NUM_IOCOOM_STATS, np.uint64)
    r = lib().oracle_iocoom(ctypes.byref(params), ins.ctypes.data_as(ctypes.c_void_p), io,
                            np.ascontiguousarray(addr, np.uint64), np.ascontiguousarray(meta, np.uint32),
                            np.ascontiguousarray(lat, np.uint64), ao, T, float(frequency_ghz), out)
    if r:
        raise ValueError("oracle_iocoom: the instruction and access streams disagree")
    return out[:T * NUM_IOCOOM_STATS].reshape(T, NUM_IOCOOM_STATS)


def split_lines(addr, size, line=64):
    buf = np.zeros(64, np.uint64)
    n = lib().oracle_split_lines(addr, size, line, buf, 64)
    return [int(x) for x in buf[:min(n, 64)]]
