"""Python binding of the C ABI (include/graphite_gpu.h) over ctypes.

This is host plumbing only: every computation runs in libgraphite_gpu.so's
HIP kernels.  There is no CPU fallback — if the library or a GPU is missing the
calls raise.  Device buffers are torch tensors on the ROCm device (PyTorch is
used for allocation and streams only).
"""
import ctypes
import os

import numpy as np

from .config import (GGConfig, NUM_CACHE_COUNTERS, NUM_NET_COUNTERS, NUM_TILE_STATS, NUM_RUN_INFO, NUM_CORE_STATS,
                     CMSG_DTYPE)

CMSG_BYTES = CMSG_DTYPE.itemsize

HERE = os.path.dirname(os.path.abspath(__file__))
# GG_LIB (diagnostics only): load an alternative in-tree build for A/B kernel runs
LIB_PATH = os.environ.get("GG_LIB") or os.path.join(HERE, "libgraphite_gpu.so")

GG_OK = 0
_ERR = {-1: "GG_ERR_INVALID", -2: "GG_ERR_HIP", -3: "GG_ERR_UNSUPPORTED", -4: "GG_ERR_RANGE", -5: "GG_ERR_STATE"}


class GGError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (_ERR.get(code, code), msg))
        self.code = code


class LineInfo(ctypes.Structure):
    _fields_ = [("tag", ctypes.c_uint64), ("cstate", ctypes.c_uint32), ("cached_loc", ctypes.c_uint32)]


class _Trace(ctypes.Structure):
    _fields_ = [("addr_dev", ctypes.c_void_p), ("meta_dev", ctypes.c_void_p),
                ("tile_offsets", ctypes.POINTER(ctypes.c_uint64)), ("num_records", ctypes.c_uint64)]


class _Packets(ctypes.Structure):
    _fields_ = [("src_dev", ctypes.c_void_p), ("dst_dev", ctypes.c_void_p),
                ("length_bits_dev", ctypes.c_void_p), ("time_ps_dev", ctypes.c_void_p),
                ("num_packets", ctypes.c_uint64)]


class _PacketOut(ctypes.Structure):
    _fields_ = [("arrival_ps_dev", ctypes.c_void_p), ("zero_load_ps_dev", ctypes.c_void_p),
                ("contention_ps_dev", ctypes.c_void_p)]


# every symbol include/graphite_gpu.h declares (checked by tests/test_abi.py)
EXPORTS = ["gg_abi_version", "gg_last_error", "gg_config_default", "gg_create", "gg_destroy", "gg_reset",
           "gg_cache_access_batch", "gg_cache_get_counters", "gg_cache_get_line_info",
           "gg_cache_set_line_info", "gg_cache_access_line", "gg_cache_insert_line",
           "gg_noc_route_batch", "gg_noc_route_tree", "gg_noc_get_counters", "gg_queue_delay_batch",
           "gg_gen_uniform_trace", "gg_kernel_time_ms", "gg_set_timing",
           "gg_coherent_begin", "gg_coherent_quantum", "gg_coherent_export", "gg_coherent_import",
           "gg_coherent_run", "gg_coherent_get_stats", "gg_gen_hotspot_trace", "gg_shard_map",
           "gg_kernel_stats", "gg_round_exchange", "gg_coherent_run_ranks", "gg_gen_stress_trace",
           "gg_split_accesses", "gg_combine_accesses", "gg_dump_summary", "gg_core_model_run", "gg_core_get_stats", "gg_coherent_get_miss_types",
           "gg_coherent_get_protocol_stats", "gg_iocoom_run", "gg_iocoom_get_stats",
           "gg_round_pack", "gg_round_unpack", "gg_round_finish"]


class RoundIO(ctypes.Structure):
    """gg_round_io: the device buffers of one rank's round (gg_round_pack)."""
    _fields_ = [("send", ctypes.c_void_p), ("recv", ctypes.c_void_p), ("words_own", ctypes.c_void_p),
                ("words_all", ctypes.c_void_p), ("stride", ctypes.c_uint64), ("slot", ctypes.c_uint64),
                ("send_count", ctypes.POINTER(ctypes.c_uint64)), ("recv_count", ctypes.POINTER(ctypes.c_uint64)),
                ("next_q", ctypes.c_uint64), ("done", ctypes.c_int32), ("state", ctypes.c_int32)]


ROUND_WORDS = 8
ROUND_DONE, ROUND_AGAIN, ROUND_OVERFLOW = 0, 1, 2
CMSG_RECORD_BYTES = 64


class _CStatus(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_uint64), ("boundary_msgs", ctypes.c_uint64), ("min_next_ps", ctypes.c_uint64),
                ("active_tiles", ctypes.c_uint32), ("blocked_tiles", ctypes.c_uint32)]

_lib = None


def load():
    """Load libgraphite_gpu.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("graphite_amd: %s is missing — run __graft_entry__.build() "
                           "(make -C graphite_amd/csrc); there is no CPU fallback" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    L.gg_abi_version.restype = i32
    L.gg_last_error.restype = ctypes.c_char_p
    L.gg_config_default.argtypes = [ctypes.POINTER(GGConfig), u32]
    L.gg_create.restype = vp
    L.gg_create.argtypes = [ctypes.POINTER(GGConfig), ctypes.POINTER(i32)]
    L.gg_destroy.argtypes = [vp]
    L.gg_reset.argtypes = [vp]
    L.gg_cache_access_batch.argtypes = [vp, ctypes.POINTER(_Trace), vp, vp, vp]
    L.gg_cache_get_counters.argtypes = [vp, vp]
    L.gg_cache_get_line_info.argtypes = [vp, u32, i32, u64, ctypes.POINTER(LineInfo)]
    L.gg_cache_set_line_info.argtypes = [vp, u32, i32, u64, ctypes.POINTER(LineInfo)]
    L.gg_cache_access_line.argtypes = [vp, u32, i32, u64, i32]
    L.gg_cache_insert_line.argtypes = [vp, u32, i32, u64, ctypes.POINTER(LineInfo), ctypes.POINTER(i32),
                                       ctypes.POINTER(u64), ctypes.POINTER(LineInfo)]
    L.gg_noc_route_batch.argtypes = [vp, ctypes.POINTER(_Packets), ctypes.POINTER(_PacketOut), vp]
    L.gg_noc_route_tree.argtypes = [vp, ctypes.POINTER(_Packets), ctypes.POINTER(_PacketOut),
                                    ctypes.POINTER(_PacketOut), u64, vp]
    L.gg_noc_get_counters.argtypes = [vp, vp]
    L.gg_queue_delay_batch.argtypes = [vp, u64, vp, vp, u64, vp]
    L.gg_gen_uniform_trace.argtypes = [vp, vp, u32, u32, u64, u64, u32, u32, vp]
    L.gg_kernel_time_ms.restype = ctypes.c_float
    L.gg_kernel_time_ms.argtypes = [vp, ctypes.c_char_p]
    L.gg_set_timing.argtypes = [vp, i32]
    L.gg_coherent_begin.argtypes = [vp, ctypes.POINTER(_Trace), vp, vp]
    L.gg_coherent_quantum.argtypes = [vp, u64, ctypes.POINTER(_CStatus)]
    L.gg_coherent_export.argtypes = [vp, vp, u64, vp]
    L.gg_coherent_import.argtypes = [vp, vp, u64]
    L.gg_coherent_run.argtypes = [vp, ctypes.POINTER(_Trace), vp, vp]
    L.gg_coherent_get_stats.argtypes = [vp, vp, vp, vp]
    L.gg_gen_hotspot_trace.argtypes = [vp, vp, u32, u32, u64, u64, u32, u32, u32, u32, vp]
    L.gg_shard_map.argtypes = [u32, u32, vp]
    L.gg_kernel_stats.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64)]
    L.gg_round_exchange.argtypes = [vp, vp, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(i32)]
    L.gg_gen_stress_trace.argtypes = [vp, vp, u32, u32, u64, u64, u32, u32, u32, u32, u32, vp]
    L.gg_coherent_run_ranks.argtypes = [vp, vp, ctypes.POINTER(_Trace), vp, vp]
    L.gg_split_accesses.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp, vp, u64, ctypes.POINTER(u64), vp, vp]
    L.gg_combine_accesses.argtypes = [vp, vp, u64, vp, vp, vp]
    L.gg_dump_summary.argtypes = [vp, i32, ctypes.c_char_p, u64, ctypes.POINTER(u64)]
    L.gg_core_model_run.argtypes = [vp, ctypes.POINTER(_Trace), vp, vp]
    L.gg_core_get_stats.argtypes = [vp, vp]
    L.gg_iocoom_run.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.gg_iocoom_get_stats.argtypes = [vp, vp]
    L.gg_coherent_get_miss_types.argtypes = [vp, vp]
    L.gg_coherent_get_protocol_stats.argtypes = [vp, vp]
    L.gg_round_pack.argtypes = [vp, u32, u32, u64, ctypes.POINTER(RoundIO)]
    L.gg_round_unpack.argtypes = [vp, ctypes.POINTER(RoundIO)]
    L.gg_round_finish.argtypes = [vp, ctypes.POINTER(RoundIO)]
    for name in ["gg_kernel_stats", "gg_shard_map", "gg_coherent_begin", "gg_coherent_quantum", "gg_coherent_export",
                 "gg_coherent_import", "gg_coherent_run", "gg_coherent_get_stats", "gg_gen_hotspot_trace",
                 "gg_round_exchange", "gg_coherent_run_ranks", "gg_gen_stress_trace", "gg_split_accesses",
                 "gg_combine_accesses", "gg_dump_summary", "gg_core_model_run", "gg_core_get_stats",
                 "gg_coherent_get_miss_types", "gg_coherent_get_protocol_stats", "gg_iocoom_run",
                 "gg_iocoom_get_stats", "gg_round_pack", "gg_round_unpack", "gg_round_finish"]:
        getattr(L, name).restype = i32
    for name in ["gg_reset", "gg_cache_access_batch", "gg_cache_get_counters", "gg_cache_get_line_info",
                 "gg_cache_set_line_info", "gg_cache_access_line", "gg_cache_insert_line",
                 "gg_noc_route_batch", "gg_noc_route_tree", "gg_noc_get_counters", "gg_queue_delay_batch",
                 "gg_gen_uniform_trace"]:
        getattr(L, name).restype = i32
    _lib = L
    return L


def _check(rc):
    if rc != GG_OK:
        raise GGError(rc, load().gg_last_error().decode(errors="replace"))


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _need_dev(t, dtype, n=None):
    import torch
    if not t.is_cuda:
        raise ValueError("expected a device tensor")
    if t.dtype != dtype or not t.is_contiguous():
        raise ValueError("expected a contiguous %s device tensor" % dtype)
    if n is not None and t.numel() != n:
        raise ValueError("expected %d elements, got %d" % (n, t.numel()))


class Backend:
    """One context per GPU (gg_create): device-resident private caches of
    every tile and the NoC router state."""

    def __init__(self, cfg: GGConfig):
        L = load()
        st = ctypes.c_int(0)
        self.cfg = cfg
        self.h = L.gg_create(ctypes.byref(cfg), ctypes.byref(st))
        if not self.h:
            _check(st.value or -1)

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.gg_destroy(self.h)
            self.h = None

    __del__ = close

    def reset(self):
        _check(load().gg_reset(self.h))

    def set_timing(self, on=True, every_launch=False):
        """Kernel timing: off, sampled HIP events (coherent launches: 1 in 16),
        or every_launch=True: every coherent step / walk launch stamps its
        span (first workgroup start, last workgroup end) in-kernel."""
        load().gg_set_timing(self.h, (2 if every_launch else 1) if on else 0)

    def kernel_time_ms(self, name):
        return load().gg_kernel_time_ms(self.h, name.encode())

    def kernel_stats(self, name):
        """(total device ms, launches) of a coherent-mode kernel since the last
        coherent begin (timing must be on): mean over the timed launches (every
        16th, or every one) x launches."""
        ms, n = ctypes.c_double(0), ctypes.c_uint64(0)
        _check(load().gg_kernel_stats(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    # ---- cache ----------------------------------------------------------
    def cache_access_batch(self, addr, meta, tile_offsets, result=None, evicted=None, stream=None):
        """Replay a tile-major trace batch (device tensors addr: uint64 as
        int64, meta: int32).  tile_offsets: host sequence of num_tiles+1."""
        import torch
        n = addr.numel()
        _need_dev(addr, torch.int64, n)
        _need_dev(meta, torch.int32, n)
        if result is not None:
            _need_dev(result, torch.int32, n)
        if evicted is not None:
            _need_dev(evicted, torch.int64, n)
        offs = np.ascontiguousarray(tile_offsets, dtype=np.uint64)
        if offs.size != self.cfg.num_tiles + 1:
            raise ValueError("tile_offsets needs num_tiles + 1 entries")
        tr = _Trace(addr.data_ptr(), meta.data_ptr(), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n)
        self._keep = offs
        _check(load().gg_cache_access_batch(self.h, ctypes.byref(tr), _ptr(result), _ptr(evicted), _stream(stream)))

    def cache_counters(self):
        out = np.zeros(self.cfg.num_tiles * 2 * NUM_CACHE_COUNTERS, np.uint64)
        _check(load().gg_cache_get_counters(self.h, out.ctypes.data_as(ctypes.c_void_p)))
        return out.reshape(self.cfg.num_tiles, 2, NUM_CACHE_COUNTERS)

    def get_line_info(self, tile, level, addr, default=None):
        li = default or LineInfo(0xFFFFFFFFFFFFFFFF, 0, 0)
        _check(load().gg_cache_get_line_info(self.h, tile, level, addr, ctypes.byref(li)))
        return li

    def set_line_info(self, tile, level, addr, li):
        return load().gg_cache_set_line_info(self.h, tile, level, addr, ctypes.byref(li))

    def access_line(self, tile, level, addr, is_store):
        return load().gg_cache_access_line(self.h, tile, level, addr, int(is_store))

    def insert_line(self, tile, level, addr, li):
        ev = ctypes.c_int(0)
        ea = ctypes.c_uint64(0)
        evi = LineInfo(0xFFFFFFFFFFFFFFFF, 0, 0)
        rc = load().gg_cache_insert_line(self.h, tile, level, addr, ctypes.byref(li), ctypes.byref(ev),
                                         ctypes.byref(ea), ctypes.byref(evi))
        return rc, ev.value, ea.value, evi

    # ---- NoC ------------------------------------------------------------
    def noc_route_batch(self, src, dst, length_bits, time_ps, arrival, zero_load, contention, stream=None):
        import torch
        n = src.numel()
        for t, dt in ((src, torch.int32), (dst, torch.int32), (length_bits, torch.int32), (time_ps, torch.int64),
                      (arrival, torch.int64), (zero_load, torch.int64), (contention, torch.int64)):
            _need_dev(t, dt, n)
        pk = _Packets(src.data_ptr(), dst.data_ptr(), length_bits.data_ptr(), time_ps.data_ptr(), n)
        out = _PacketOut(arrival.data_ptr(), zero_load.data_ptr(), contention.data_ptr())
        _check(load().gg_noc_route_batch(self.h, ctypes.byref(pk), ctypes.byref(out), _stream(stream)))

    def noc_route_tree(self, src, dst, length_bits, time_ps, arrival, zero_load, contention,
                       b_arrival, b_zero_load, b_contention, num_broadcasts, stream=None):
        """gg_noc_route_tree: dst == config.BROADCAST takes the hop-by-hop broadcast
        tree; b_* hold num_broadcasts x num_tiles deliveries (batch order)."""
        import torch
        n = src.numel()
        for t, dt in ((src, torch.int32), (dst, torch.int32), (length_bits, torch.int32), (time_ps, torch.int64),
                      (arrival, torch.int64), (zero_load, torch.int64), (contention, torch.int64)):
            _need_dev(t, dt, n)
        nbt = num_broadcasts * self.cfg.num_tiles
        for t in (b_arrival, b_zero_load, b_contention):
            _need_dev(t, torch.int64, nbt)
        pk = _Packets(src.data_ptr(), dst.data_ptr(), length_bits.data_ptr(), time_ps.data_ptr(), n)
        out = _PacketOut(arrival.data_ptr(), zero_load.data_ptr(), contention.data_ptr())
        bout = _PacketOut(b_arrival.data_ptr(), b_zero_load.data_ptr(), b_contention.data_ptr())
        _check(load().gg_noc_route_tree(self.h, ctypes.byref(pk), ctypes.byref(out), ctypes.byref(bout),
                                        num_broadcasts, _stream(stream)))

    def noc_counters(self):
        out = np.zeros(self.cfg.num_tiles * NUM_NET_COUNTERS, np.uint64)
        _check(load().gg_noc_get_counters(self.h, out.ctypes.data_as(ctypes.c_void_p)))
        return out.reshape(self.cfg.num_tiles, NUM_NET_COUNTERS)

    # ---- coherent mode (Mode C) ----------------------------------------
    def _trace(self, addr, meta, tile_offsets):
        import torch
        n = addr.numel()
        _need_dev(addr, torch.int64, n)
        _need_dev(meta, torch.int32, n)
        offs = np.ascontiguousarray(tile_offsets, dtype=np.uint64)
        if offs.size != self.cfg.num_tiles + 1:
            raise ValueError("tile_offsets needs num_tiles + 1 entries")
        self._keep = offs
        return _Trace(addr.data_ptr(), meta.data_ptr(), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n)

    def coherent_run(self, addr, meta, tile_offsets, out=None, stream=None):
        """Whole coherent run (the context must own every shard).  out: int64
        device tensor, one word per record ((latency_ps << 2) | level)."""
        import torch
        if out is not None:
            _need_dev(out, torch.int64, addr.numel())
        tr = self._trace(addr, meta, tile_offsets)
        _check(load().gg_coherent_run(self.h, ctypes.byref(tr), _ptr(out), _stream(stream)))

    def coherent_run_ranks(self, comm_ptr, addr, meta, tile_offsets, out=None, stream=None):
        """The whole coherent run over the ranks of an RCCL communicator
        (gg_coherent_run_ranks; comm_ptr = ncclComm_t as an int, e.g.
        ProcessGroupNCCL._comm_ptr()).  This context owns the rank's shards."""
        import torch
        if out is not None:
            _need_dev(out, torch.int64, addr.numel())
        tr = self._trace(addr, meta, tile_offsets)
        _check(load().gg_coherent_run_ranks(self.h, ctypes.c_void_p(comm_ptr), ctypes.byref(tr), _ptr(out),
                                            _stream(stream)))

    def coherent_begin(self, addr, meta, tile_offsets, out=None, stream=None):
        import torch
        if out is not None:
            _need_dev(out, torch.int64, addr.numel())
        tr = self._trace(addr, meta, tile_offsets)
        _check(load().gg_coherent_begin(self.h, ctypes.byref(tr), _ptr(out), _stream(stream)))

    def round_pack(self, world, rank, q):
        """gg_round_pack: quantum q's steps + the tail on the context's stream;
        returns the RoundIO with the device slots / words to move."""
        io = RoundIO()
        _check(load().gg_round_pack(self.h, world, rank, q, ctypes.byref(io)))
        return io

    def round_unpack(self, io):
        _check(load().gg_round_unpack(self.h, ctypes.byref(io)))
        return io

    def round_finish(self, io):
        _check(load().gg_round_finish(self.h, ctypes.byref(io)))
        return io

    def coherent_quantum(self, q):
        st = _CStatus()
        _check(load().gg_coherent_quantum(self.h, q, ctypes.byref(st)))
        return {"steps": st.steps, "boundary_msgs": st.boundary_msgs, "min_next_ps": st.min_next_ps,
                "active_tiles": st.active_tiles, "blocked_tiles": st.blocked_tiles}

    def coherent_export(self, out_buf, cap):
        """Held cross-shard records -> out_buf (uint8 device tensor of cap*CMSG_BYTES
        bytes), grouped by destination shard; returns per-shard counts."""
        K = self.cfg.num_shards or 1
        counts = np.zeros(K, np.uint64)
        _check(load().gg_coherent_export(self.h, _ptr(out_buf), cap, counts.ctypes.data_as(ctypes.c_void_p)))
        return counts

    def coherent_import(self, buf, n):
        _check(load().gg_coherent_import(self.h, _ptr(buf), n))

    def coherent_stats(self):
        T = self.cfg.num_tiles
        st = np.zeros(T * NUM_TILE_STATS, np.uint64)
        cc = np.zeros(T * 2 * NUM_CACHE_COUNTERS, np.uint64)
        ri = np.zeros(NUM_RUN_INFO, np.uint64)
        _check(load().gg_coherent_get_stats(self.h, st.ctypes.data_as(ctypes.c_void_p),
                                            cc.ctypes.data_as(ctypes.c_void_p), ri.ctypes.data_as(ctypes.c_void_p)))
        return st.reshape(T, NUM_TILE_STATS), cc.reshape(T, 2, NUM_CACHE_COUNTERS), ri

    def core_model_run(self, meta, tile_offsets, access_out, stream=None):
        """The simple core model over a coherent run's access words
        (gg_core_model_run): meta (int32/uint32 device tensor of the trace's
        meta words), host tile offsets, access_out (int64 device tensor)."""
        import torch
        self._offs = np.ascontiguousarray(tile_offsets, np.uint64)
        if self._offs.size != self.cfg.num_tiles + 1:
            raise ValueError("tile_offsets needs num_tiles + 1 entries")
        n = int(self._offs[-1])
        _need_dev(meta, torch.int32, n)
        _need_dev(access_out, torch.int64, n)
        tr = _Trace(None, meta.data_ptr(), self._offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n)
        _check(load().gg_core_model_run(self.h, ctypes.byref(tr), access_out.data_ptr(), _stream(stream)))

    def iocoom_run(self, params, ins, ins_offsets, addr, meta, lat, acc_offsets, stream=None):
        """The iocoom core model (gg_iocoom_run): params (config.IocoomParams),
        ins (device tensor holding the gg_ins records, 16 B each), host
        instruction tile offsets, the access stream's addr (int64), meta
        (int32) and latency (int64, ps) device tensors, host access tile
        offsets."""
        import torch
        T = self.cfg.num_tiles
        io = np.ascontiguousarray(ins_offsets, np.uint64)
        ao = np.ascontiguousarray(acc_offsets, np.uint64)
        if io.size != T + 1 or ao.size != T + 1:
            raise ValueError("tile offsets need num_tiles + 1 entries")
        if not ins.is_cuda or not ins.is_contiguous() or ins.numel() * ins.element_size() < 16 * int(io[-1]):
            raise ValueError("ins: a contiguous device tensor of %d gg_ins records" % int(io[-1]))
        n = int(ao[-1])
        _need_dev(addr, torch.int64, n)
        _need_dev(meta, torch.int32, n)
        _need_dev(lat, torch.int64, n)
        self._io_offs = (io, ao)
        self._io_params = params
        _check(load().gg_iocoom_run(self.h, ctypes.byref(params), ins.data_ptr(), io.ctypes.data, addr.data_ptr(),
                                    meta.data_ptr(), lat.data_ptr(), ao.ctypes.data, _stream(stream)))

    def iocoom_stats(self):
        """[tiles][NUM_IOCOOM_STATS] (gg_iocoom_get_stats)."""
        from graphite_amd.config import NUM_IOCOOM_STATS
        T = self.cfg.num_tiles
        out = np.zeros(T * NUM_IOCOOM_STATS, np.uint64)
        _check(load().gg_iocoom_get_stats(self.h, out.ctypes.data_as(ctypes.c_void_p)))
        return out.reshape(T, NUM_IOCOOM_STATS)

    def miss_types(self):
        """[tiles][2][3] cold / capacity / sharing misses of the L1-D and L2
        (gg_coherent_get_miss_types; zeros for an untracked cache)."""
        T = self.cfg.num_tiles
        out = np.zeros(T * 2 * 3, np.uint64)
        _check(load().gg_coherent_get_miss_types(self.h, out.ctypes.data_as(ctypes.c_void_p)))
        return out.reshape(T, 2, 3)

    def protocol_stats(self):
        """[tiles][NUM_PROTO_STATS] MOSI event counters (gg_coherent_get_protocol_stats; zeros under MSI)."""
        T = self.cfg.num_tiles
        out = np.zeros(T * 32, np.uint64)
        _check(load().gg_coherent_get_protocol_stats(self.h, out.ctypes.data_as(ctypes.c_void_p)))
        return out.reshape(T, 32)

    def core_stats(self):
        T = self.cfg.num_tiles
        out = np.zeros(T * NUM_CORE_STATS, np.uint64)
        _check(load().gg_core_get_stats(self.h, out.ctypes.data_as(ctypes.c_void_p)))
        return out.reshape(T, NUM_CORE_STATS)

    def dump_summary(self, table=False):
        """The sim.out text of the context's statistics (gg_dump_summary): one
        "Tile t Summary:" block per tile, or TileManager's table."""
        L = load()
        need = ctypes.c_uint64(0)
        fmt = 1 if table else 0
        _check(L.gg_dump_summary(self.h, fmt, None, 0, ctypes.byref(need)))
        buf = ctypes.create_string_buffer(need.value)
        _check(L.gg_dump_summary(self.h, fmt, buf, need.value, ctypes.byref(need)))
        return buf.value.decode()

    def queue_delay_batch(self, pkt_time, proc_time, min_processing_time=1):
        t = np.ascontiguousarray(pkt_time, np.uint64)
        p = np.ascontiguousarray(proc_time, np.uint64)
        d = np.zeros(t.size, np.uint64)
        _check(load().gg_queue_delay_batch(self.h, min_processing_time, t.ctypes.data_as(ctypes.c_void_p),
                                           p.ctypes.data_as(ctypes.c_void_p), t.size,
                                           d.ctypes.data_as(ctypes.c_void_p)))
        return d


def shard_map(num_tiles, num_shards):
    """tile -> logical shard through the ABI (gg_shard_map)."""
    out = np.zeros(num_tiles, np.uint32)
    _check(load().gg_shard_map(num_tiles, num_shards, out.ctypes.data_as(ctypes.c_void_p)))
    return out


def gen_uniform_trace(addr, meta, tile_begin, tiles, per_tile, first=0, lines_log2=15, base_shift=26, stream=None):
    """Fill device tensors with the configs[1] synthetic trace."""
    _check(load().gg_gen_uniform_trace(_ptr(addr), _ptr(meta), tile_begin, tiles, per_tile, first,
                                       lines_log2, base_shift, _stream(stream)))


def gen_hotspot_trace(addr, meta, tile_begin, tiles, per_tile, first=0, lines_log2=15, base_shift=26,
                      hot_lines=64, hot_frac256=51, stream=None):
    """Fill device tensors with the configs[2..4] hotspot trace."""
    _check(load().gg_gen_hotspot_trace(_ptr(addr), _ptr(meta), tile_begin, tiles, per_tile, first, lines_log2,
                                       base_shift, hot_lines, hot_frac256, _stream(stream)))


def gen_stress_trace(addr, meta, tile_begin, tiles, per_tile, num_tiles, first=0, lines_log2=15, base_shift=26,
                     pool_lines=4096, pool_frac256=77, stream=None):
    """Fill device tensors with the configs[4] coherent stress trace."""
    _check(load().gg_gen_stress_trace(_ptr(addr), _ptr(meta), tile_begin, tiles, per_tile, first, lines_log2,
                                      base_shift, num_tiles, pool_lines, pool_frac256, _stream(stream)))


def split_accesses(addr, size, meta, tile_offsets, line_size=64, stream=None):
    """Multi-line accesses -> line records (gg_split_accesses, core.cc:139-266).
    addr (int64 byte addresses), size (int32 bytes), meta (int32) are device
    tensors of a tile-major access trace with host tile_offsets [tiles + 1].
    Returns (line_addr, line_meta, first, line_tile_offsets): device tensors
    of the line trace (later lines GG_META_CONT), each access's first line
    (n + 1 entries) and the line trace's host tile offsets."""
    import torch
    offs = np.ascontiguousarray(tile_offsets, dtype=np.uint64)
    tiles = len(offs) - 1
    n = int(offs[-1]) if tiles > 0 else 0
    first = torch.empty(n + 1, dtype=torch.int64, device=addr.device)
    nl = ctypes.c_uint64(0)
    loffs = np.zeros(tiles + 1, np.uint64)
    L = load()
    _check(L.gg_split_accesses(_ptr(addr), _ptr(size), _ptr(meta), offs.ctypes.data_as(ctypes.c_void_p), tiles,
                               line_size, _ptr(first), None, None, 0, ctypes.byref(nl), None, _stream(stream)))
    la = torch.empty(max(nl.value, 1), dtype=torch.int64, device=addr.device)
    lm = torch.empty(max(nl.value, 1), dtype=torch.int32, device=addr.device)
    _check(L.gg_split_accesses(_ptr(addr), _ptr(size), _ptr(meta), offs.ctypes.data_as(ctypes.c_void_p), tiles,
                               line_size, _ptr(first), _ptr(la), _ptr(lm), nl.value, ctypes.byref(nl),
                               loffs.ctypes.data_as(ctypes.c_void_p), _stream(stream)))
    return la[:nl.value], lm[:nl.value], first, loffs


def combine_accesses(line_out, first, stream=None):
    """Per-access (latency_ps, misses) of a coherent run over a split trace
    (gg_combine_accesses, core.cc:239-266): device int64 / int32 tensors."""
    import torch
    n = first.numel() - 1
    lat = torch.empty(max(n, 0), dtype=torch.int64, device=first.device)
    miss = torch.empty(max(n, 0), dtype=torch.int32, device=first.device)
    _check(load().gg_combine_accesses(_ptr(line_out), _ptr(first), max(n, 0), _ptr(lat), _ptr(miss), _stream(stream)))
    return lat, miss


def gen_iocoom_streams(T, per_tile, seed, regs=24, addrs=24, p_sync=0.01, max_lat=300000):
    """Tile-major instructions (random read / write registers from `regs`
    registers, 0-2 memory reads and 0-1 memory writes, simple-mov loads,
    atomics, fences, SyncInstructions) and the access stream their memory
    operands consume in order (addresses from `addrs` per tile, so loads hit
    the store buffer; 0xFFFFFFFF records with and without a stall)."""
    from . import config as C_
    rng = np.random.default_rng(seed)
    n = T * per_tile
    ins = np.zeros(n, C_.INS_DTYPE)
    sync = rng.random(n) < p_sync
    nr = rng.integers(0, 4, n)
    nw = np.minimum(rng.integers(0, 3, n), 6 - nr)
    nrd = rng.choice(3, n, p=[0.55, 0.35, 0.10])
    nwm = (rng.random(n) < 0.25).astype(np.int64)
    smov = (nrd == 1) & (nwm == 0) & (nw == 1) & (rng.random(n) < 0.6)
    fence = np.where(rng.random(n) < 0.03, rng.integers(1, 4, n), 0)
    atomic = rng.random(n) < 0.02
    nr[sync] = 0; nw[sync] = 0; nrd[sync] = 0; nwm[sync] = 0; smov[sync] = False; fence[sync] = 0; atomic[sync] = False
    ins["cost"] = rng.choice(np.array([0, 1, 1, 1, 3, 5, 6, 18]), n)
    ins["ops"] = (nrd | (nwm << 2) | np.where(smov, C_.INS_SIMPLE_MOV_LOAD, 0) |
                  np.where(atomic, C_.INS_ATOMIC, 0) | (fence << C_.INS_FENCE_SHIFT)).astype(np.uint8)
    ins["regs"] = (nr | (nw << 3) | np.where(sync, C_.INS_SYNC, 0)).astype(np.uint8)
    ins["reg"] = rng.integers(0, regs, (n, 6)).astype(np.uint16)
    ins_offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(per_tile)
    cnt = np.where(sync, 1, nrd + nwm)
    tot = int(cnt.sum())
    owner = np.repeat(np.arange(n), cnt)
    pos = np.arange(tot) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    is_bar = sync[owner]
    is_wr = ~is_bar & (pos >= nrd[owner])
    meta = np.where(is_bar, np.uint32(0xFFFFFFFF), np.where(is_wr, np.uint32(1), np.uint32(0))).astype(np.uint32)
    meta[~is_bar] |= (rng.integers(0, 8, int((~is_bar).sum())) << 1).astype(np.uint32)   # gap bits: ignored
    tile = owner // per_tile
    addr = (tile.astype(np.uint64) << np.uint64(20)) + rng.integers(0, addrs, tot).astype(np.uint64) * np.uint64(8)
    lat = rng.integers(1000, max_lat, tot).astype(np.uint64)
    lat[is_bar & (rng.random(tot) < 0.3)] = 0
    per = np.bincount(tile, minlength=T)
    acc_offs = np.concatenate([[0], np.cumsum(per)]).astype(np.uint64)
    return ins, ins_offs, addr, meta, lat, acc_offs


class CoherentEngine:
    """A Backend context behind the engine surface of graphite_amd.coherent.run
    (one rank: the shards [cfg.shard_begin, cfg.shard_end))."""

    def __init__(self, backend, addr, meta, tile_offsets, out=None):
        import torch
        self.be = backend
        self.dev = addr.device
        backend.coherent_begin(addr, meta, tile_offsets, out)
        self.cap = 64 * backend.cfg.num_tiles + 65536
        self.buf = torch.empty(self.cap * CMSG_BYTES, dtype=torch.uint8, device=self.dev)

    def quantum(self, q):
        return self.be.coherent_quantum(q)

    def export(self):
        counts = self.be.coherent_export(self.buf, self.cap)
        n = int(counts.sum())
        return self.buf[:n * CMSG_BYTES], counts

    def import_(self, buf):
        n = buf.numel() // CMSG_BYTES
        if n:
            self.be.coherent_import(buf.contiguous(), n)
