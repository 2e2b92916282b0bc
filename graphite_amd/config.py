"""Configuration of the batch backend: the ctypes mirror of ``gg_config``
(include/graphite_gpu.h) and the reference defaults of ``carbon_sim.cfg``.

Reference keys (nmtrmail/Graphite carbon_sim.cfg): l1_dcache/T1 (:219-228),
l2_cache/T1 (:230-239), network/emesh_* (:290-313), queue_model/history_tree
(:388-392), DVFS domain 1 GHz (:147-155).
"""
import ctypes
import math

import numpy as np

POLICY_LRU = 0
POLICY_ROUND_ROBIN = 1
NET_MAGIC = 0
NET_EMESH_HOP_COUNTER = 1
NET_EMESH_HOP_BY_HOP = 2
# queue model types (QueueModel::create, queue_model.cc:19-39) and queue_model/basic moving averages
QM_HISTORY_TREE = 0
QM_HISTORY_LIST = 1
QM_BASIC = 2
MAVG_ARITHMETIC_MEAN = 0
MAVG_MEDIAN = 1
MAVG_NONE = 2
MAVG_GEOMETRIC_MEAN = 3

L1D = 0
L2 = 1

CSTATE_INVALID = 0
CSTATE_SHARED = 1
CSTATE_OWNED = 2      # MOSI
CSTATE_EXCLUSIVE = 3  # MESI
CSTATE_MODIFIED = 4
PROTO_MSI, PROTO_MOSI, PROTO_SHL2_MSI, PROTO_SHL2_MESI = 0, 1, 2, 3   # GG_PROTO_* (caching_protocol/type)
MOSI_RNG_SEED = 1                     # GG_MOSI_RNG_SEED
LOC_INVALID = 0
LOC_L1D = 3

META_WRITE = 1

RES_L1_MISS = 1 << 0
RES_L2_MISS = 1 << 4
RES_L1_INVAL = 1 << 8
RES_L1_EVICT = 1 << 12
RES_L2_EVICT = 1 << 16
RES_L2_EVICT_DIRTY = 1 << 20
RES_L2_EVICT_INV_L1 = 1 << 24
RES_UPGRADE = 1 << 28

CACHE_COUNTERS = ["accesses", "misses", "read_accesses", "read_misses",
                  "write_accesses", "write_misses", "evictions", "dirty_evictions",
                  "tag_reads", "tag_writes", "data_reads", "data_writes"]
NET_COUNTERS = ["packets_sent", "flits_sent", "bits_sent", "packets_received",
                "flits_received", "bits_received", "total_latency_ps",
                "total_contention_ps", "buffer_writes", "buffer_reads",
                "switch_alloc", "crossbar", "link_traversals",
                "router_contention_cycles", "router_packets", "analytical_requests"] + \
               ["port%d_utilized_cycles" % p for p in range(5)] + ["port%d_last_cycles" % p for p in range(5)] + \
               ["packets_broadcasted", "flits_broadcasted", "bits_broadcasted"] + \
               ["crossbar%d" % m for m in range(2, 6)]
BROADCAST = 0xDEADBABE   # NetPacket::BROADCAST (network.h:54), GG_BROADCAST
NUM_CACHE_COUNTERS = len(CACHE_COUNTERS)

# coherent mode (include/graphite_gpu.h)
MSG_TYPES = ["EX_REQ", "SH_REQ", "INV_REQ", "FLUSH_REQ", "WB_REQ", "EX_REP", "SH_REP",
             "UPGRADE_REP", "INV_REP", "FLUSH_REP", "WB_REP"]
MSG = {n: i + 1 for i, n in enumerate(MSG_TYPES)}
MSG["NULLIFY_REQ"], MSG["INV_FLUSH_COMBINED_REQ"] = 12, 13
MSG["DRAM_FETCH_REQ"], MSG["DRAM_STORE_REQ"], MSG["DRAM_FETCH_REP"] = 14, 15, 16   # pr_l1_sh_l2_msi
MSG["DOWNGRADE_REQ"], MSG["SH_REP_EX"], MSG["DOWNGRADE_REP"] = 17, 18, 19            # pr_l1_sh_l2_mesi
CT_SENT_INV_FLUSH_COMBINED = 29       # GG_CT_SENT_INV_FLUSH_COMBINED (MOSI)
CT_SENT_DRAM_FETCH_REQ, CT_SENT_DRAM_STORE_REQ, CT_SENT_DRAM_FETCH_REP = 29, 30, 31   # pr_l1_sh_l2_msi
# MOSI event counters, [tile][NUM_PROTO_STATS] (GG_PS_*)
PROTO_STATS = ["exreq", "exreq_modified", "exreq_shared", "exreq_upgrade", "exreq_uncached",
               "exreq_serialization_ps", "exreq_processing_ps",
               "shreq", "shreq_modified", "shreq_shared", "shreq_uncached",
               "shreq_serialization_ps", "shreq_processing_ps",
               "nullify", "nullify_modified", "nullify_shared", "nullify_uncached",
               "nullify_serialization_ps", "nullify_processing_ps",
               "inv_unicast", "inv_broadcast", "inv_sharers_unicast", "inv_sharers_broadcast",
               "inv_processing_unicast_ps", "inv_processing_broadcast_ps",
               "l2_invalidations", "l2_evictions", "l2_dirty_evictions_exreq", "l2_clean_evictions_exreq",
               "l2_dirty_evictions_shreq", "l2_clean_evictions_shreq"]
NUM_PROTO_STATS = 32
LVL_L1, LVL_L2, LVL_DIR = 0, 1, 2
TILE_STATS = ["clock_ps", "accesses", "l1_hits", "l2_hits", "l2_misses", "latency_ps",
              "dir_accesses", "dir_evictions", "dir_back_invalidations",
              "dram_accesses", "dram_latency_ns", "dram_queue_delay_ns",
              "dram_queue_requests", "dram_queue_analytical", "msgs_sent", "msgs_received"] + \
             ["sent_" + n.lower() for n in MSG_TYPES] + ["dram_queue_utilized_ns", "dram_queue_last_ns"]
NUM_TILE_STATS = 32
RUN_INFO = ["quanta", "steps", "net_msgs", "self_msgs", "boundary_msgs", "final_quantum"]
NUM_RUN_INFO = 8
# gg_core_model_run statistics (include/graphite_gpu.h GG_CORE_*)
CORE_STATS = ["instructions", "time_ps", "memory_stall_ps", "execution_stall_ps", "l1d_read_stall_ps",
              "l1d_write_stall_ps", "sync_instructions", "sync_stall_ps"]
MISS_TYPES = ["cold", "capacity", "sharing"]   # GG_MT_* (Cache::MissType)
META_BARRIER = 0xFFFFFFFF     # GG_META_BARRIER: a BARRIER record of the trace
LVL_SYNC = 3                  # GG_LVL_SYNC: its access word (stall << 2) | 3
NUM_CORE_STATS = 8
# gg_iocoom_run (include/graphite_gpu.h gg_ins, GG_INS_*, GG_IOCOOM_*)
INS_DTYPE = np.dtype([("cost", "<u2"), ("ops", "u1"), ("regs", "u1"), ("reg", "<u2", (6,))])
INS_SIMPLE_MOV_LOAD, INS_ATOMIC, INS_FENCE_SHIFT, INS_SYNC = 0x10, 0x20, 6, 0x80
IOCOOM_NUM_REGISTERS = 512
IOCOOM_STATS = ["instructions", "time_ps", "memory_stall_ps", "execution_stall_ps", "sync_instructions",
                "sync_stall_ps", "load_queue_stall_ps", "store_queue_stall_ps", "l1i_stall_ps",
                "intra_l1d_stall_ps", "inter_l1d_stall_ps", "intra_exec_stall_ps", "inter_exec_stall_ps",
                "explicit_fences", "implicit_mfences", "data_accesses", "data_latency_ps"]
NUM_IOCOOM_STATS = 17


class IocoomParams(ctypes.Structure):
    """gg_iocoom_params; defaults = carbon_sim.cfg [core/iocoom]."""
    _fields_ = [("num_load_queue_entries", ctypes.c_uint32), ("num_store_queue_entries", ctypes.c_uint32),
                ("speculative_loads_enabled", ctypes.c_uint32),
                ("multiple_outstanding_RFOs_enabled", ctypes.c_uint32)]

    def __init__(self, lq=8, sq=8, spec=1, rfo=1):
        super().__init__(lq, sq, spec, rfo)


CMSG_DTYPE = None  # filled below (numpy view of gg_cmsg)
NUM_NET_COUNTERS = len(NET_COUNTERS)


class GGConfig(ctypes.Structure):
    _fields_ = [
        ("num_tiles", ctypes.c_uint32),
        ("line_size", ctypes.c_uint32),
        ("l1d_size_kb", ctypes.c_uint32),
        ("l1d_assoc", ctypes.c_uint32),
        ("l1d_policy", ctypes.c_uint32),
        ("l2_size_kb", ctypes.c_uint32),
        ("l2_assoc", ctypes.c_uint32),
        ("l2_policy", ctypes.c_uint32),
        ("net_model", ctypes.c_uint32),
        ("flit_width", ctypes.c_uint32),
        ("router_delay", ctypes.c_uint32),
        ("link_delay", ctypes.c_uint32),
        ("queue_model_enabled", ctypes.c_uint32),
        ("max_list_size", ctypes.c_uint32),
        ("analytical_enabled", ctypes.c_uint32),
        ("total_tiles", ctypes.c_uint32),
        ("frequency_ghz", ctypes.c_double),
        ("device", ctypes.c_int32),
        ("replay_kernel", ctypes.c_uint32),
        ("l1d_data_cycles", ctypes.c_uint32),
        ("l1d_tags_cycles", ctypes.c_uint32),
        ("l2_data_cycles", ctypes.c_uint32),
        ("l2_tags_cycles", ctypes.c_uint32),
        ("dir_assoc", ctypes.c_uint32),
        ("dir_total_entries", ctypes.c_uint32),
        ("dir_access_cycles", ctypes.c_uint32),
        ("dram_latency_ns", ctypes.c_uint32),
        ("dram_bandwidth", ctypes.c_float),
        ("dram_queue_model_enabled", ctypes.c_uint32),
        ("quantum_ns", ctypes.c_uint32),
        ("num_shards", ctypes.c_uint32),
        ("shard_begin", ctypes.c_uint32),
        ("shard_end", ctypes.c_uint32),
        ("queue_model_type", ctypes.c_uint32),
        ("dram_queue_model_type", ctypes.c_uint32),
        ("basic_moving_avg", ctypes.c_uint32),
        ("history_list_no_interleaving", ctypes.c_uint32),
        ("l1i_track_miss_types", ctypes.c_uint32),
        ("l2_track_miss_types", ctypes.c_uint32),
        ("miss_track_lines", ctypes.c_uint32),
        ("protocol", ctypes.c_uint32),
        ("l1d_track_miss_types", ctypes.c_uint32),
    ]


def default_config(num_tiles, **overrides):
    """The carbon_sim.cfg defaults for ``num_tiles`` application tiles."""
    c = GGConfig()
    c.num_tiles = num_tiles
    c.line_size = 64
    c.l1d_size_kb, c.l1d_assoc, c.l1d_policy = 32, 4, POLICY_LRU
    c.l2_size_kb, c.l2_assoc, c.l2_policy = 512, 8, POLICY_LRU
    c.net_model = NET_EMESH_HOP_COUNTER
    c.flit_width = 64
    c.router_delay = 1
    c.link_delay = 1
    c.queue_model_enabled = 1
    c.max_list_size = 100
    c.analytical_enabled = 1
    c.total_tiles = 0
    c.frequency_ghz = 1.0
    c.device = 0
    c.replay_kernel = 0
    # coherent mode (carbon_sim.cfg:97, 219-273)
    c.l1d_data_cycles, c.l1d_tags_cycles = 1, 1
    c.l2_data_cycles, c.l2_tags_cycles = 8, 3
    c.dir_assoc, c.dir_total_entries, c.dir_access_cycles = 16, 0, 0
    c.dram_latency_ns, c.dram_bandwidth, c.dram_queue_model_enabled = 100, 5.0, 1
    c.quantum_ns = 1000
    c.num_shards = 1
    c.shard_begin, c.shard_end = 0, 0
    for k, v in overrides.items():
        if not hasattr(c, k):
            raise KeyError(k)
        setattr(c, k, v)
    return c


def tile_id_bits(num_tiles):
    """Config::computeTileIDLength = ceilLog2(application tiles) (config.cc:149-152)."""
    return int(math.ceil(math.log2(num_tiles))) if num_tiles > 1 else 0


def shmem_modeled_bits(num_tiles, with_data):
    """Modeled length of an MSI ShmemMsg packet in bits: 2 * tile-id bits
    (network_model.cc:185-200) + 4 msg-type + 48 address bits (+ 64 B of data)
    (pr_l1_pr_l2_dram_directory_msi/shmem_msg.cc:100-125, shmem_msg.h:81)."""
    return 2 * tile_id_bits(num_tiles) + 4 + 48 + (512 if with_data else 0)


def _cmsg_dtype():
    import numpy as np
    return np.dtype([("addr", "<u8"), ("send_ps", "<u8"), ("arrival_ps", "<u8"), ("zero_load_ps", "<u8"),
                     ("src", "<u4"), ("dst", "<u4"), ("requester", "<u4"), ("seq", "<u4"), ("type", "<u4"),
                     ("link", "<u4"), ("hop", "<u4"), ("single_rx", "<u4")])


CMSG_DTYPE = _cmsg_dtype()


HOP_NONE = 0xFFFFFFFF


def shard_map(num_tiles, num_shards):
    """Logical shard of every tile: on a full W x H mesh
    the 2-D block the reference gives process k of num_shards under
    emesh_hop_by_hop (NetworkModelEMeshHopByHop::computeProcessToTileMapping,
    network_model_emesh_hop_by_hop.cc:367-433); contiguous tile ranges
    otherwise.  Same rule as the ABI's gg_shard_map."""
    import numpy as np
    T, K = int(num_tiles), int(num_shards or 1)
    if K < 1 or K > T:
        raise ValueError("num_shards must be in [1, num_tiles]")
    W = int(math.floor(math.sqrt(T)))
    H = int(math.ceil(T / W))
    if W * H != T:
        return (np.arange(T, dtype=np.int64) * K // T).astype(np.uint32)
    out = np.full(T, 0xFFFFFFFF, np.uint32)
    pw = int(math.floor(math.sqrt(K)))
    ph = int(math.floor(K / pw))
    mhl = int((1.0 * H * pw * ph) / K)
    for i in range(pw):
        for j in range(ph):
            sx, sy = W // pw, mhl // ph
            bx, by = i * sx, j * sy
            if i == pw - 1:
                sx = W - (pw - 1) * sx
            if j == ph - 1:
                sy = mhl - (ph - 1) * sy
            for jj in range(sy):
                out[(by + jj) * W + bx:(by + jj) * W + bx + sx] = i + j * pw
    left = K - pw * ph
    for i in range(pw * ph, K):
        sx = W // left
        sy, bx, by = H - mhl, (i - pw * ph) * sx, mhl
        if i == K - 1:
            sx = W - (left - 1) * sx
        for jj in range(sy):
            out[(by + jj) * W + bx:(by + jj) * W + bx + sx] = i
    if (out >= K).any() or len(np.unique(out)) != K:
        raise ValueError("no shard map for %d tiles in %d shards" % (T, K))
    return out


def shard_of_tile(tile, num_tiles, num_shards):
    """Logical shard of a tile (shard_map)."""
    return int(shard_map(num_tiles, num_shards)[tile])
