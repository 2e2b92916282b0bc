"""Configuration of the batch backend: the ctypes mirror of ``gg_config``
(include/graphite_gpu.h) and the reference defaults of ``carbon_sim.cfg``.

Reference keys (nmtrmail/Graphite carbon_sim.cfg): l1_dcache/T1 (:219-228),
l2_cache/T1 (:230-239), network/emesh_* (:290-313), queue_model/history_tree
(:388-392), DVFS domain 1 GHz (:147-155).
"""
import ctypes
import math

POLICY_LRU = 0
POLICY_ROUND_ROBIN = 1
NET_MAGIC = 0
NET_EMESH_HOP_COUNTER = 1
NET_EMESH_HOP_BY_HOP = 2

L1D = 0
L2 = 1

CSTATE_INVALID = 0
CSTATE_SHARED = 1
CSTATE_MODIFIED = 4
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
                "router_contention_cycles", "router_packets", "analytical_requests"]
NUM_CACHE_COUNTERS = len(CACHE_COUNTERS)
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
        ("reserved", ctypes.c_uint32 * 6),
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
