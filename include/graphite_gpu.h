/*
 * graphite_gpu.h — C ABI of the MI355X batch backend for Graphite's
 * memory-subsystem hot path (private L1-D/L2 cache simulation and EMesh NoC
 * packet latency).
 *
 * This is the drop-in boundary.  Every entry point below replaces one
 * in-process C++ interface of the reference simulator (paths relative to
 * nmtrmail/Graphite):
 *
 *   gg_cache_access_batch      batched Cache line access: the per-access state
 *                              machine L1CacheCntlr::processMemOpFromCore
 *                              (common/tile/memory_subsystem/
 *                              pr_l1_pr_l2_dram_directory_msi/l1_cache_cntlr.cc:89-180)
 *                              + L2CacheCntlr (l2_cache_cntlr.cc:74-527) driving
 *                              Cache::accessCacheLine / insertCacheLine /
 *                              getCacheLineInfo / setCacheLineInfo
 *                              (common/tile/memory_subsystem/cache/cache.h:87-92),
 *                              i.e. the "accessSingleLine" entry of the north star
 *                              applied to a whole trace batch.
 *   gg_cache_access_line       Cache::accessCacheLine            (cache.cc:84-112)
 *   gg_cache_insert_line       Cache::insertCacheLine            (cache.cc:114-184)
 *   gg_cache_get_line_info     Cache::getCacheLineInfo           (cache.cc:187-205)
 *   gg_cache_set_line_info     Cache::setCacheLineInfo           (cache.cc:218-241)
 *   gg_cache_get_counters      the counters printed by Cache::outputSummary
 *                              (cache.cc:419-477)
 *   gg_noc_route_batch         NetworkModel::__routePacket -> routePacket
 *                              (common/network/network_model.cc:87-116,
 *                              network_model.h:188) for every hop of each packet,
 *                              plus NetworkModel::__processReceivedPacket
 *                              (network_model.cc:118-150) at the receiver:
 *                              emesh_hop_counter (models/network_model_emesh_hop_counter.cc:143-157)
 *                              and emesh_hop_by_hop (models/network_model_emesh_hop_by_hop.cc:146-264)
 *   gg_noc_route_tree          the same with broadcast packets (receiver GG_BROADCAST):
 *                              the emesh_hop_by_hop broadcast tree
 *                              (network_model_emesh_hop_by_hop.cc:163-221,
 *                              network/emesh_hop_by_hop/broadcast_tree_enabled)
 *   gg_noc_get_counters        NetworkModel / RouterModel counters
 *                              (network_model.cc:228-316, router_model.cc:120-145)
 *   gg_queue_delay_batch       QueueModelHistoryTree::computeQueueDelay
 *                              (common/shared_models/queue_models/queue_model_history_tree.cc:44-126)
 *
 * Conventions: every function returns a gg_status (0 = OK, negative = error);
 * no exception crosses the ABI; pointers named *_dev are HIP device pointers,
 * all others are host pointers owned by the caller; one host thread per
 * context, one context per GPU.  The reference reports misuse with
 * LOG_ASSERT_ERROR (aborting, common/misc/log.h:112-135); this ABI returns
 * GG_ERR_* instead and records a message retrievable with gg_last_error().
 */
#ifndef GRAPHITE_GPU_H
#define GRAPHITE_GPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GG_ABI_VERSION 10

typedef int gg_status;
enum {
  GG_OK = 0,
  GG_ERR_INVALID = -1,      /* bad argument / inconsistent config            */
  GG_ERR_HIP = -2,          /* HIP runtime error                             */
  GG_ERR_UNSUPPORTED = -3,  /* configuration outside what the backend builds */
  GG_ERR_RANGE = -4,        /* address / time outside the encodable range    */
  GG_ERR_STATE = -5         /* reference would LOG_ASSERT_ERROR here          */
};

/* Replacement policies: CacheReplacementPolicy::parse (cache_replacement_policy.cc:33-46) */
enum { GG_POLICY_LRU = 0, GG_POLICY_ROUND_ROBIN = 1 };

/* Network models: NetworkModel::parseNetworkType (network_model.cc:318-335) */
enum { GG_NET_MAGIC = 0, GG_NET_EMESH_HOP_COUNTER = 1, GG_NET_EMESH_HOP_BY_HOP = 2 };

/* Cache levels (pr_l1_pr_l2_dram_directory_msi/cache_level.h) */
enum { GG_L1D = 0, GG_L2 = 1 };

/* Cache line states, numerically identical to CacheState::Type (cache_state.h:11-21) */
enum { GG_CSTATE_INVALID = 0, GG_CSTATE_SHARED = 1, GG_CSTATE_OWNED = 2 /* MOSI */, GG_CSTATE_EXCLUSIVE = 3 /* MESI */,
       GG_CSTATE_MODIFIED = 4 };

/* Cached-location values of a private L2 line, MemComponent::Type subset
 * (PrL2CacheLineInfo::_cached_loc, pr_l1_pr_l2_dram_directory_msi/cache_line_info.h) */
enum { GG_LOC_INVALID = 0, GG_LOC_L1I = 2, GG_LOC_L1D = 3 };

/* Access trace record metadata word (gg_trace.meta[i]):
 *   bit 0      : 1 = WRITE (Core::WRITE), 0 = READ (Core::READ)
 *   bits 1..30 : gap in core cycles before this access (coherent/timing modes;
 *                ignored by the private-cache mode)
 *   bit 31     : GG_META_CONT — a later line of a multi-line access
 *                (gg_split_accesses): coherent mode issues it at the previous
 *                record's completion and never cuts it at the lax barrier (the
 *                access is one instruction, core.cc:139-266); gap must be 0.
 *                The private-cache mode ignores it.                          */
#define GG_META_WRITE 1u
#define GG_META_CONT 0x80000000u
/* A BARRIER record (CarbonBarrierWait / SPLASH BARRIER, sync_client.cc:265-316;
 * a CONT code with a nonzero gap, which no access carries; addr ignored):
 * the tile waits until every tile with an unfinished trace waits at a
 * barrier (SimBarrier::wait, sync_server.cc:133-170 with the count = those
 * tiles), then all continue at the latest arrival time (SyncServer::
 * barrierWait replies max_time, :357-383; the MCP is a system tile, so the
 * messages cost no network time).  gg_coherent_run applies the release at the
 * quantum boundary after the last arrival and writes the record's access
 * word as (stall_ps << 2) | GG_LVL_SYNC.  Only gg_coherent_run takes traces
 * with barriers (the per-quantum and multi-rank entry points return
 * GG_ERR_UNSUPPORTED; the private-cache batch flags one in the device error
 * word, so the next gg_cache_get_counters returns GG_ERR_UNSUPPORTED;
 * gg_split_accesses rejects one in its access trace: insert barriers into
 * the line records it writes).  Barriers carry no id or count: one global
 * barrier whose count is "every tile with an unfinished trace", released at
 * the quantum boundary after its last arrival.                 */
#define GG_META_BARRIER 0xFFFFFFFFu

/* Per-access result word written by gg_cache_access_batch: one flag per 4-bit
 * field, so result words of up to 15 accesses can be summed field-wise (the
 * replay kernel derives its counters that way).  Where the access was served:
 * L1-D hit = !L1_MISS; L2 hit = L1_MISS && !L2_MISS; directory = L2_MISS.   */
#define GG_RES_L1_MISS         (1u << 0)  /* not an L1-D hit (operationPermissibleinL1Cache, l1:207-243): request to the L2 */
#define GG_RES_L2_MISS         (1u << 4)  /* not an L2 hit either (l2:180-224): SH_REQ / EX_REQ to the home directory */
#define GG_RES_L1_INVAL        (1u << 8)  /* the L1-D held the line without the needed permission: invalidated first (l1:135-137) */
#define GG_RES_L1_EVICT        (1u << 12) /* the L1-D insert evicted a line (insertCacheLineInL1, l2:133-165) */
#define GG_RES_L2_EVICT        (1u << 16) /* the L2 insert evicted a line (l2:74-116) */
#define GG_RES_L2_EVICT_DIRTY  (1u << 20) /* ... in MODIFIED: FLUSH_REP + data (else INV_REP) */
#define GG_RES_L2_EVICT_INV_L1 (1u << 24) /* ... and invalidated its copy in L1-D (invalidateCacheLineInL1, l2:124-131) */
#define GG_RES_UPGRADE         (1u << 28) /* WRITE to a SHARED L2 line: INV_REP + EX_REQ (l2:260-282) */

/* Cache counters, one vector per (tile, level).  Index = what Cache::outputSummary prints. */
enum {
  GG_CC_ACCESSES = 0, GG_CC_MISSES, GG_CC_READ_ACCESSES, GG_CC_READ_MISSES,
  GG_CC_WRITE_ACCESSES, GG_CC_WRITE_MISSES, GG_CC_EVICTIONS, GG_CC_DIRTY_EVICTIONS,
  GG_CC_TAG_READS, GG_CC_TAG_WRITES, GG_CC_DATA_READS, GG_CC_DATA_WRITES,
  GG_NUM_CACHE_COUNTERS
};

/* Network counters per tile (NetworkModel::outputSummary + model event counters). */
enum {
  GG_NC_PACKETS_SENT = 0, GG_NC_FLITS_SENT, GG_NC_BITS_SENT,
  GG_NC_PACKETS_RECEIVED, GG_NC_FLITS_RECEIVED, GG_NC_BITS_RECEIVED,
  GG_NC_TOTAL_LATENCY_PS, GG_NC_TOTAL_CONTENTION_PS,
  /* emesh_hop_counter: updateEventCounters (network_model_emesh_hop_counter.cc:120-127)
   * emesh_hop_by_hop : mesh RouterModel event counters + link traversals    */
  GG_NC_BUFFER_WRITES, GG_NC_BUFFER_READS, GG_NC_SWITCH_ALLOC, GG_NC_CROSSBAR,
  GG_NC_LINK_TRAVERSALS,
  GG_NC_ROUTER_CONTENTION_CYCLES, GG_NC_ROUTER_PACKETS, GG_NC_ANALYTICAL_REQUESTS,
  /* emesh_hop_by_hop with contention: QueueModel utilization counters of the 5
   * mesh output-port queues (queue_model.cc:49-55), + port (SELF, LEFT, RIGHT,
   * DOWN, UP), for RouterModel::getAverageLinkUtilization (router_model.cc:168-182) */
  GG_NC_PORT_UTILIZED_CYCLES,
  GG_NC_PORT_LAST_CYCLES = GG_NC_PORT_UTILIZED_CYCLES + 5,
  /* broadcasts (gg_noc_route_tree): updateSendCounters' broadcast totals
   * (network_model.cc:244-250) and RouterModel::updateEventCounters'
   * Crossbar[2..5] traversals (router_model.cc:126; GG_NC_CROSSBAR = Crossbar[1]) */
  GG_NC_PACKETS_BROADCASTED = GG_NC_PORT_LAST_CYCLES + 5,
  GG_NC_FLITS_BROADCASTED, GG_NC_BITS_BROADCASTED,
  GG_NC_CROSSBAR_MULTI,                 /* + (ports - 2), ports = 2..5 */
  GG_NUM_NET_COUNTERS = GG_NC_CROSSBAR_MULTI + 4
};

/* Queue model types (the type strings of QueueModel::create) and the
 * moving averages of queue_model/basic (MovingAverage::createAvgType,
 * common/misc/moving_average.h).  history_list uses max_list_size and
 * analytical_enabled below (queue_model/history_list, same defaults).    */
enum { GG_QM_HISTORY_TREE = 0, GG_QM_HISTORY_LIST = 1, GG_QM_BASIC = 2 };
enum { GG_MAVG_ARITHMETIC_MEAN = 0, GG_MAVG_MEDIAN = 1, GG_MAVG_NONE = 2 /* moving_avg_enabled = false */,
       GG_MAVG_GEOMETRIC_MEAN = 3 /* not supported: GG_ERR_UNSUPPORTED */ };

typedef struct gg_config {
  uint32_t num_tiles;          /* application tiles (general/total_cores)          */
  uint32_t line_size;          /* bytes, l1_dcache/T1/cache_line_size (64)          */
  uint32_t l1d_size_kb;        /* l1_dcache/T1/cache_size (32)                      */
  uint32_t l1d_assoc;          /* l1_dcache/T1/associativity (4)                    */
  uint32_t l1d_policy;         /* GG_POLICY_*                                        */
  uint32_t l2_size_kb;         /* l2_cache/T1/cache_size (512)                      */
  uint32_t l2_assoc;           /* l2_cache/T1/associativity (8)                     */
  uint32_t l2_policy;
  uint32_t net_model;          /* GG_NET_* for network/memory                        */
  uint32_t flit_width;         /* bits (64)                                          */
  uint32_t router_delay;       /* cycles (1)                                         */
  uint32_t link_delay;         /* cycles (1)                                         */
  uint32_t queue_model_enabled;/* network/emesh_hop_by_hop/queue_model/enabled       */
  uint32_t max_list_size;      /* queue_model/history_tree/max_list_size (100)      */
  uint32_t analytical_enabled; /* queue_model/history_tree/analytical_model_enabled */
  uint32_t total_tiles;        /* app tiles + MCP + spawners (config.cc:77-82); 0 = num_tiles+2 */
  double   frequency_ghz;      /* single DVFS domain (carbon_sim.cfg:147-155)        */
  int32_t  device;             /* HIP device ordinal                                 */
  uint32_t replay_kernel;      /* 0 = single-pass streaming replay where instantiated (else 2),
                                  1 = sharded generic replay, 2 = sharded lean replay */
  /* ---- coherent mode (pr_l1_pr_l2_dram_directory_msi with directory, DRAM, NoC) ---- */
  uint32_t l1d_data_cycles;    /* l1_dcache/T1/data_access_time (1)                 */
  uint32_t l1d_tags_cycles;    /* l1_dcache/T1/tags_access_time (1)                 */
  uint32_t l2_data_cycles;     /* l2_cache/T1/data_access_time (8)                  */
  uint32_t l2_tags_cycles;     /* l2_cache/T1/tags_access_time (3)                  */
  uint32_t dir_assoc;          /* dram_directory/associativity (16)                 */
  uint32_t dir_total_entries;  /* dram_directory/total_entries, 0 = "auto"          */
  uint32_t dir_access_cycles;  /* dram_directory/access_time, 0 = "auto"            */
  uint32_t dram_latency_ns;    /* dram/latency (100)                                */
  float    dram_bandwidth;     /* dram/per_controller_bandwidth, GB/s (5.0)         */
  uint32_t dram_queue_model_enabled; /* dram/queue_model/enabled (history_tree)     */
  uint32_t quantum_ns;         /* clock_skew_management/lax_barrier/quantum (1000)  */
  uint32_t num_shards;         /* logical shards (canonical schedule); 0 = 1 */
  uint32_t shard_begin;        /* shards owned by this context: [shard_begin, shard_end) */
  uint32_t shard_end;          /* 0 = all                                            */
  /* ---- queue models (QueueModel::create, shared_models/queue_model.cc:19-39) ---- */
  uint32_t queue_model_type;   /* network/emesh_hop_by_hop/queue_model/type: GG_QM_* (0 = history_tree) */
  uint32_t dram_queue_model_type; /* dram/queue_model/type: GG_QM_*                 */
  uint32_t basic_moving_avg;   /* queue_model/basic: moving_avg_window_size in bits 0..15
                                  (0 = 64) | GG_MAVG_* << 16 (0 = arithmetic_mean)  */
  uint32_t history_list_no_interleaving; /* queue_model/history_list/interleaving_enabled = false */
  /* ---- miss-type classification (Cache track_miss_types, cache.cc:321-405) ---- */
  uint32_t l1i_track_miss_types; /* l1_icache/T1/track_miss_types (false): the L1-D takes THIS flag
                                    (L1CacheCntlr passes the L1-I one to both, l1_cache_cntlr.cc:69) */
  uint32_t l2_track_miss_types;  /* l2_cache/T1/track_miss_types (false)               */
  uint32_t miss_track_lines;     /* coherent mode, when tracking: address-set capacity per
                                    (tile, cache) in lines, a power of two; 0 = 65536.
                                    The sets keep every line ever fetched, evicted or
                                    invalidated, so size it from the trace's per-tile
                                    footprint; allocated when tracking is on:
                                    tiles x 2 x lines x 8 B (65536: 1 GiB at 1024 tiles,
                                    4 GiB at 4096).  A full table stops the run with
                                    GG_ERR_UNSUPPORTED (no set entry is overwritten). */
  /* ---- caching protocol (caching_protocol/type, carbon_sim.cfg:184) ---- */
  uint32_t protocol;             /* GG_PROTO_*: pr_l1_pr_l2_dram_directory_msi (0) / _mosi (1) /
                                    pr_l1_sh_l2_msi (2) / pr_l1_sh_l2_mesi (3)                */
  uint32_t l1d_track_miss_types; /* l1_dcache/T1/track_miss_types (false): read by the MOSI
                                    protocol only, whose L1CacheCntlr passes the L1-D flag to the
                                    L1-D (…mosi/l1_cache_cntlr.cc:68; MSI passes the L1-I one) */
} gg_config;

/* Caching protocols of the coherent mode (MemoryManager::createMMU,
 * memory_manager.cc:22-60).  pr_l1_sh_l2_msi: private L1s, the L2 a shared
 * slice per tile (home = line % tiles) whose lines hold the full-map
 * directory entries, a DRAM controller per tile reached by DRAM_FETCH /
 * DRAM_STORE messages; the l2_* geometry is one slice's, the dir_* fields are
 * not used.  pr_l1_sh_l2_mesi adds EXCLUSIVE L1 lines: a read of an uncached
 * line is answered SH_REP_EX, the exclusive owner is invalidated (INV_REQ,
 * answered FLUSH_REP when modified) or downgraded (DOWNGRADE_REQ, answered
 * WB_REP when modified, else DOWNGRADE_REP); its own message types count in
 * GG_CT_MSGS_SENT only.  MOSI's DramDirectoryCntlr picks "one sharer"
 * with the directory entry's own drand48 stream (DirectoryEntryFullMap::
 * getOneSharer, directory_entry_full_map.cc:67-74; misc/random.h), which the
 * reference seeds with time(NULL) when the entry is created: the canonical
 * schedule seeds every entry with GG_MOSI_RNG_SEED (one fixed second).      */
enum { GG_PROTO_MSI = 0, GG_PROTO_MOSI = 1, GG_PROTO_SHL2_MSI = 2, GG_PROTO_SHL2_MESI = 3 };
#define GG_MOSI_RNG_SEED 1

/* Miss types (Cache::MissType, cache.h:45-52), counted per (tile, cache). */
enum { GG_MT_COLD = 0, GG_MT_CAPACITY, GG_MT_SHARING, GG_NUM_MISS_TYPES = 3 };

/* Fill cfg with the reference defaults of carbon_sim.cfg for num_tiles tiles. */
void gg_config_default(gg_config* cfg, uint32_t num_tiles);

/* A batch of line accesses in tile-major program order (structure of arrays).
 * Records of tile t are [tile_offsets[t], tile_offsets[t+1]).  addr[i] is the
 * byte address of the accessed line (the low log2(line_size) bits are ignored,
 * as Cache::getTag does, cache.cc:495-498).  Addresses must be < 2^48.        */
typedef struct gg_trace {
  const uint64_t* addr_dev;
  const uint32_t* meta_dev;
  const uint64_t* tile_offsets;   /* host, num_tiles + 1 entries */
  uint64_t        num_records;
} gg_trace;

/* A batch of NoC packets.  Packet k: sender/receiver tile ids, modeled length
 * in bits (NetworkModel::getModeledLength, network_model.cc:185-200) and its
 * send time in picoseconds (NetPacket::time).                                 */
typedef struct gg_packets {
  const uint32_t* src_dev;
  const uint32_t* dst_dev;
  const uint32_t* length_bits_dev;
  const uint64_t* time_ps_dev;
  uint64_t        num_packets;
} gg_packets;

/* Per-packet result: time the packet is handed to the receiving tile
 * (after serialization, network_model.cc:142-150) and the zero-load /
 * contention split (Hop, network_model.cc:556-563).                            */
typedef struct gg_packet_out {
  uint64_t* arrival_ps_dev;
  uint64_t* zero_load_ps_dev;
  uint64_t* contention_ps_dev;
} gg_packet_out;

typedef struct gg_line_info {    /* CacheLineInfo / PrL2CacheLineInfo            */
  uint64_t tag;                  /* line address (addr >> log2 line); ~0 = invalid */
  uint32_t cstate;               /* GG_CSTATE_*                                   */
  uint32_t cached_loc;           /* GG_LOC_* (L2 only)                            */
} gg_line_info;

/* ------------------------------------------------------------------------
 * Coherent mode ("Mode C"): the full pr_l1_pr_l2_dram_directory_msi protocol —
 * L1CacheCntlr / L2CacheCntlr (l1_cache_cntlr.cc, l2_cache_cntlr.cc),
 * DramDirectoryCntlr with DirectoryCache + full-map entries
 * (dram_directory_cntlr.cc, cache/directory_cache.cc,
 * directory_schemes/directory_entry_full_map.cc), DramCntlr + DramPerfModel
 * (dram_cntlr.cc, performance_models/dram_perf_model.cc), the ShmemPerfModel
 * clock (performance_models/shmem_perf_model.cc), the memory network
 * (NetworkModel::routePacket) and the lax-barrier quantum
 * (clock_skew_management_schemes/lax_barrier_sync_*.cc) — driven in the
 * canonical schedule of DESIGN.md §Mode C.
 * ------------------------------------------------------------------------ */

/* ShmemMsg::Type (pr_l1_pr_l2_dram_directory_msi/shmem_msg.h:12-30); MOSI's
 * INV_FLUSH_COMBINED_REQ (…mosi/shmem_msg.h:20, numbered after WB_REQ there)
 * is 13 here so the MSI numbering stays as it is; pr_l1_sh_l2_msi's DRAM
 * messages (…sh_l2_msi/shmem_msg.h:26-30) follow it */
enum {
  GG_MSG_EX_REQ = 1, GG_MSG_SH_REQ, GG_MSG_INV_REQ, GG_MSG_FLUSH_REQ, GG_MSG_WB_REQ,
  GG_MSG_EX_REP, GG_MSG_SH_REP, GG_MSG_UPGRADE_REP, GG_MSG_INV_REP, GG_MSG_FLUSH_REP,
  GG_MSG_WB_REP, GG_MSG_NULLIFY_REQ, GG_MSG_INV_FLUSH_COMBINED_REQ,
  GG_MSG_DRAM_FETCH_REQ, GG_MSG_DRAM_STORE_REQ, GG_MSG_DRAM_FETCH_REP,
  GG_MSG_DOWNGRADE_REQ, GG_MSG_SH_REP_EX, GG_MSG_DOWNGRADE_REP   /* pr_l1_sh_l2_mesi (…sh_l2_mesi/shmem_msg.h:14-39) */
};

/* One ShmemMsg in flight (64 bytes).  The per-sender sequence number keeps
 * the per-channel FIFO order of the reference transports
 * (socktransport.cc:225,366).  A record is either a message for dst's inbox
 * (hop == GG_HOP_NONE) or, under emesh_hop_by_hop with several logical
 * shards, a packet still in the mesh, held at a shard edge: it has left the
 * output port of a router in one shard and continues at router `hop` of
 * another shard after the quantum boundary (arrival_ps = its time at `hop`,
 * contention so far = arrival_ps - send_ps - zero_load_ps).                 */
#define GG_HOP_NONE 0xFFFFFFFFu
typedef struct gg_cmsg {
  uint64_t addr;         /* line byte address                                   */
  uint64_t send_ps;      /* NetPacket::time when sent (MemoryManager::sendMsg)  */
  uint64_t arrival_ps;   /* time handed to the receiver, after the network      */
  uint64_t zero_load_ps; /* zero-load part of the network time so far           */
  uint32_t src, dst;     /* sender / receiver tile                              */
  uint32_t requester;    /* ShmemMsg::_requester                                */
  uint32_t seq;          /* per-sender sequence number                          */
  uint32_t type;         /* GG_MSG_*                                            */
  uint32_t link;         /* backend-private (ignored on import)                 */
  uint32_t hop;          /* GG_HOP_NONE, or the router tile of a held packet    */
  uint32_t single_rx;    /* ShmemMsg::_single_receiver of an INV_FLUSH_COMBINED_REQ
                            (…mosi/shmem_msg.h), else 0                          */
} gg_cmsg;

/* Logical shards: on a full W x H mesh (W = floor(sqrt
 * num_tiles)) the tiles of shard k are the 2-D block the reference gives
 * process k of num_shards under emesh_hop_by_hop
 * (NetworkModelEMeshHopByHop::computeProcessToTileMapping,
 * network_model_emesh_hop_by_hop.cc:367-433); otherwise contiguous tile
 * ranges.  Writes tile_shard[num_tiles]; GG_ERR_INVALID if a shard is empty. */
gg_status gg_shard_map(uint32_t num_tiles, uint32_t num_shards, uint32_t* tile_shard);

/* Per-access output word of the coherent mode: (latency_ps << 2) | level,
 * latency = Core::initiateMemoryAccess final - initial time (core.cc:245-251). */
enum { GG_LVL_L1 = 0, GG_LVL_L2 = 1, GG_LVL_DIR = 2, GG_LVL_SYNC = 3 /* a BARRIER record: latency = sync stall */ };

/* Per-tile statistics of the coherent mode, [tile][GG_NUM_TILE_STATS]. */
enum {
  GG_CT_CLOCK_PS = 0,        /* core clock after the tile's last access / barrier release */
  GG_CT_ACCESSES, GG_CT_L1_HITS, GG_CT_L2_HITS, GG_CT_L2_MISSES, GG_CT_LATENCY_PS,
  GG_CT_DIR_ACCESSES,        /* DirectoryCache::_total_directory_accesses (directory_cache.cc:97-100) */
  GG_CT_DIR_EVICTIONS,       /* _total_evictions                                      */
  GG_CT_DIR_BACK_INVALIDATIONS,
  GG_CT_DRAM_ACCESSES,       /* DramPerfModel::m_num_accesses (dram_perf_model.cc:110)  */
  GG_CT_DRAM_LATENCY_NS,     /* m_total_access_latency                                */
  GG_CT_DRAM_QUEUE_DELAY_NS, /* m_total_queueing_delay                                */
  GG_CT_DRAM_QUEUE_REQUESTS, /* QueueModel::_total_requests of the DRAM queue          */
  GG_CT_DRAM_QUEUE_ANALYTICAL,
  GG_CT_MSGS_SENT,           /* ShmemMsgs sent over the network (self-sends included)  */
  GG_CT_MSGS_RECEIVED,
  GG_CT_SENT_BY_TYPE,        /* + (type - 1), 11 entries                               */
  /* QueueModel utilization counters of the DRAM queue (queue_model.cc:49-55),
   * for DramPerfModel::outputSummary's "Queue Utilization" (dram_perf_model.cc:141-163) */
  GG_CT_DRAM_QUEUE_UTILIZED_NS = GG_CT_SENT_BY_TYPE + 11, /* _total_utilized_cycles */
  GG_CT_DRAM_QUEUE_LAST_NS,                               /* _last_request_time     */
  GG_CT_SENT_INV_FLUSH_COMBINED = 29,                     /* MOSI INV_FLUSH_COMBINED_REQs sent */
  /* pr_l1_sh_l2_msi (no INV_FLUSH_COMBINED_REQ there): its DRAM messages sent */
  GG_CT_SENT_DRAM_FETCH_REQ = 29, GG_CT_SENT_DRAM_STORE_REQ = 30, GG_CT_SENT_DRAM_FETCH_REP = 31,
  GG_NUM_TILE_STATS = 32
};

/* Per-tile protocol event counters of the MOSI controllers, [tile][GG_NUM_PROTO_STATS]
 * (DramDirectoryCntlr::updateShmemReqEventCounters / updateShmemReqLatencyCounters /
 * updateInvalidationEventCounters, …mosi/dram_directory_cntlr.cc:842-1023;
 * L2CacheCntlr::updateInvalidationCounters / updateEvictionCounters,
 * …mosi/l2_cache_cntlr.cc:596-636).  Times in picoseconds.  MSI: zeros.       */
enum {
  GG_PS_EXREQ = 0, GG_PS_EXREQ_MODIFIED, GG_PS_EXREQ_SHARED, GG_PS_EXREQ_UPGRADE, GG_PS_EXREQ_UNCACHED,
  GG_PS_EXREQ_SERIALIZATION_PS, GG_PS_EXREQ_PROCESSING_PS,
  GG_PS_SHREQ, GG_PS_SHREQ_MODIFIED, GG_PS_SHREQ_SHARED, GG_PS_SHREQ_UNCACHED,
  GG_PS_SHREQ_SERIALIZATION_PS, GG_PS_SHREQ_PROCESSING_PS,
  GG_PS_NULLIFY, GG_PS_NULLIFY_MODIFIED, GG_PS_NULLIFY_SHARED, GG_PS_NULLIFY_UNCACHED,
  GG_PS_NULLIFY_SERIALIZATION_PS, GG_PS_NULLIFY_PROCESSING_PS,
  GG_PS_INV_UNICAST, GG_PS_INV_BROADCAST, GG_PS_INV_SHARERS_UNICAST, GG_PS_INV_SHARERS_BROADCAST,
  GG_PS_INV_PROCESSING_UNICAST_PS, GG_PS_INV_PROCESSING_BROADCAST_PS,
  GG_PS_L2_INVALIDATIONS, GG_PS_L2_EVICTIONS, GG_PS_L2_DIRTY_EVICTIONS_EXREQ, GG_PS_L2_CLEAN_EVICTIONS_EXREQ,
  GG_PS_L2_DIRTY_EVICTIONS_SHREQ, GG_PS_L2_CLEAN_EVICTIONS_SHREQ,
  GG_NUM_PROTO_STATS = 32
};

/* Whole-run information, [GG_NUM_RUN_INFO]. */
enum { GG_RI_QUANTA = 0, GG_RI_STEPS, GG_RI_NET_MSGS, GG_RI_SELF_MSGS, GG_RI_BOUNDARY_MSGS,
       GG_RI_FINAL_QUANTUM, GG_NUM_RUN_INFO = 8 };

/* Result of one quantum on the shards a context owns. */
typedef struct gg_coherent_status {
  uint64_t steps;           /* steps run                                                */
  uint64_t boundary_msgs;   /* cross-shard records waiting for the quantum boundary      */
                            /* (messages + held hop-by-hop packets)                      */
  uint64_t min_next_ps;     /* earliest next-access start of a gated owned tile, ~0 if none */
  uint32_t active_tiles;    /* owned tiles whose trace is not finished                  */
  uint32_t blocked_tiles;   /* owned tiles waiting for EX_REP / SH_REP                  */
} gg_coherent_status;

typedef struct gg_ctx gg_ctx;

int         gg_abi_version(void);
const char* gg_last_error(void);

/* Create a context on cfg->device: allocates the device-resident cache state of
 * every tile (reset to the constructor state: all lines invalid, LRU ages =
 * way index, lru_replacement_policy.cc:5-18) and the NoC router state.        */
gg_ctx*   gg_create(const gg_config* cfg, gg_status* status);
void      gg_destroy(gg_ctx* ctx);
gg_status gg_reset(gg_ctx* ctx);

/* Private (decoupled) cache replay of a trace batch, continuing from the
 * context's cache state.  result_dev: one word per record (GG_RES_*), may be
 * NULL.  evicted_dev: L2-evicted line byte address per record or ~0, may be
 * NULL.  Asynchronous on stream (hipStream_t, NULL = default).  Counters
 * accumulate in the context (gg_cache_get_counters).                          */
gg_status gg_cache_access_batch(gg_ctx* ctx, const gg_trace* trace,
                                uint32_t* result_dev, uint64_t* evicted_dev,
                                void* stream);

/* Counters: out has num_tiles * 2 * GG_NUM_CACHE_COUNTERS entries laid out
 * [tile][level][counter].  Synchronizes the context's stream.                */
gg_status gg_cache_get_counters(gg_ctx* ctx, uint64_t* out);

/* The Cache quartet on one tile's device-resident cache (slow path, one line
 * per call; used by the host mirror classes and the parity tests).           */
gg_status gg_cache_get_line_info(gg_ctx* ctx, uint32_t tile, int level,
                                 uint64_t addr, gg_line_info* out);
gg_status gg_cache_set_line_info(gg_ctx* ctx, uint32_t tile, int level,
                                 uint64_t addr, const gg_line_info* in);
gg_status gg_cache_access_line(gg_ctx* ctx, uint32_t tile, int level,
                               uint64_t addr, int is_store);
gg_status gg_cache_insert_line(gg_ctx* ctx, uint32_t tile, int level,
                               uint64_t addr, const gg_line_info* in,
                               int* eviction, uint64_t* evicted_addr,
                               gg_line_info* evicted_info);

/* NoC: route every packet of the batch through the configured EMesh model in
 * the canonical discrete-event order, continuing from the
 * context's router queue state.  Asynchronous on stream.                      */
gg_status gg_noc_route_batch(gg_ctx* ctx, const gg_packets* pk,
                             const gg_packet_out* out, void* stream);
/* NetPacket::BROADCAST (common/network/network.h:54) as a receiver id.     */
#define GG_BROADCAST 0xDEADBABEu
/* NoC with broadcasts: as gg_noc_route_batch, and packets whose dst is
 * GG_BROADCAST take the emesh_hop_by_hop broadcast tree
 * (network_model_emesh_hop_by_hop.cc:163-221: UP / DOWN by the router's row
 * against the sender's, LEFT / RIGHT in the sender's row, SELF at every
 * router; one RouterModel::processPacket per router over the port list,
 * router_model.cc:71-108, contention = the max over its ports) and are
 * received by every tile, the sender included.  emesh_hop_by_hop only (the
 * other models have no broadcast capability: network.cc:187-195 unrolls such
 * a packet into one unicast per tile, which the caller does with
 * gg_noc_route_batch).  out[k] is written for unicast packets; the deliveries
 * of the b-th broadcast packet of the batch (batch order) land in
 * bcast_out[b * num_tiles + tile], num_broadcasts = their count.  One device
 * walk in global (time, packet index) order: the router ports a broadcast
 * serves together couple the X and Y chains that gg_noc_route_batch runs
 * independently.  Asynchronous on stream.                                   */
gg_status gg_noc_route_tree(gg_ctx* ctx, const gg_packets* pk, const gg_packet_out* out,
                            const gg_packet_out* bcast_out, uint64_t num_broadcasts, void* stream);
/* out: num_tiles * GG_NUM_NET_COUNTERS, [tile][counter].                      */
gg_status gg_noc_get_counters(gg_ctx* ctx, uint64_t* out);

/* Stand-alone queue model of cfg.queue_model_type (QueueModel::create(type,
 * min_processing_time), queue_model.cc:19-39: history_tree by default,
 * history_list, basic) over a sequence of (pkt_time, processing_time)
 * requests; writes the queue delays.  Host pointers; used by the known-answer
 * test (tests/unit/history_tree) and the reference-harness fixtures.         */
gg_status gg_queue_delay_batch(gg_ctx* ctx, uint64_t min_processing_time,
                               const uint64_t* pkt_time, const uint64_t* proc_time,
                               uint64_t n, uint64_t* delay_out);

/* Coherent mode.  gg_coherent_begin resets the coherent state and binds a
 * tile-major trace of ALL tiles (meta bits 1..30 = gap cycles before the
 * access); only the owned shards' tiles replay.  access_out_dev receives one
 * word per record (GG_LVL_*), may be NULL.  gg_coherent_quantum runs quantum
 * q (lax barrier at (q+1) * quantum_ns) on the owned shards until no owned
 * tile can progress.  gg_coherent_export moves the cross-shard messages of the
 * quantum into out_dev (device, grouped by destination shard, ascending;
 * counts per shard into per_shard_counts, host, num_shards entries);
 * gg_coherent_import delivers messages for owned tiles (device pointer).
 * gg_coherent_run does the whole run on a context that owns every shard.   */
gg_status gg_coherent_begin(gg_ctx* ctx, const gg_trace* trace, uint64_t* access_out_dev, void* stream);
gg_status gg_coherent_quantum(gg_ctx* ctx, uint64_t q, gg_coherent_status* st);
gg_status gg_coherent_export(gg_ctx* ctx, gg_cmsg* out_dev, uint64_t cap, uint64_t* per_shard_counts);
gg_status gg_coherent_import(gg_ctx* ctx, const gg_cmsg* in_dev, uint64_t n);
gg_status gg_coherent_run(gg_ctx* ctx, const gg_trace* trace, uint64_t* access_out_dev, void* stream);
/* The coherent mode over ranks (one process per GPU), RCCL over xGMI.
 * nccl_comm is an ncclComm_t (RCCL) of W ranks; rank r's context must own
 * logical shards [r*K/W, (r+1)*K/W) (cfg.shard_begin / shard_end, K =
 * num_shards).  gg_round_exchange runs quantum q's steps on the context,
 * sends the held cross-shard records to the ranks that own their shards and
 * receives this rank's (grouped ncclSend / ncclRecv on stream), all-gathers
 * the ranks' status words and imports the records, with one host sync (a
 * rank whose step batch was short repeats the round); *next_q is the quantum
 * every rank runs next and *done 1 when the run is over (GG_ERR_STATE on a
 * deadlock).  It replaces the reference's per-message transport
 * (common/transport/socktransport.cc) plus its lax barrier round
 * (lax_barrier_sync_client.cc:31-69, lax_barrier_sync_server.cc:57-160).
 * gg_coherent_run_ranks = gg_coherent_begin + rounds from quantum 0 until done. */
gg_status gg_round_exchange(gg_ctx* ctx, void* nccl_comm, void* stream, uint64_t q, uint64_t* next_q, int* done);
gg_status gg_coherent_run_ranks(gg_ctx* ctx, void* nccl_comm, const gg_trace* trace, uint64_t* access_out_dev,
                                void* stream);
/* The round of gg_round_exchange split at its transport, for a caller that
 * moves the bytes itself (another transport, or several contexts on one GPU
 * with device copies).  gg_round_exchange is exactly: pack -> transport ->
 * unpack, again while unpack says GG_ROUND_AGAIN, and on GG_ROUND_OVERFLOW a
 * second transport of the remainder -> gg_round_finish.
 *   gg_round_pack: quantum q's steps (a batch sized from the quanta before,
 *     doubled on each repeat) and the tail kernel: the held cross-rank
 *     records into per-peer send slots and this rank's status words; enqueued
 *     on the context's stream (gg_coherent_begin's), not synced.  Fills io.
 *     The checks of world / rank / shard ownership fail before anything is
 *     enqueued (they fail alike on every rank); a failure of the steps or the
 *     tail becomes the error flag of this rank's status words instead, so the
 *     transport still runs and every rank's unpack returns the error.
 *   transport 1: once the context's stream has finished the pack, for every
 *     r != rank: records [0, 1 + slot) of send + r * stride into rank r's
 *     recv + rank * stride; and words_own into words_all + rank *
 *     GG_ROUND_WORDS of every rank (this rank's too: an all-gather).
 *   gg_round_unpack: commit + import on the stream, the gathered words to the
 *     host, one sync; io->state = GG_ROUND_AGAIN (some rank's quantum had not
 *     finished: pack again with the same q), GG_ROUND_OVERFLOW (a slot held
 *     more than `slot` records: send_count[r] / recv_count[r] records are in
 *     send slot r / receive slot r; transport 2 moves records [1 + slot,
 *     1 + send_count[r]) of send slot r into rank r's receive slot `rank`,
 *     then gg_round_finish) or GG_ROUND_DONE (next_q / done as in
 *     gg_round_exchange).  Record 0 of a slot is a header whose addr is the
 *     slot's record count.
 *   A failure unpack or finish meets after the transport (commit / import)
 *   cannot reach the words the peers already hold: the rank decides that
 *   round like its peers (GG_OK, same state) and its next pack raises its
 *   error flag, so every rank's unpack of the next round returns the error
 *   (the failing rank its own message).  If that round ended the run there
 *   is no next round: the failing rank alone returns its error.  A new
 *   gg_coherent_begin drops a round left in progress (after AGAIN or an
 *   error): the next pack starts at step 0 of its quantum.                  */
enum { GG_ROUND_WORDS = 8, GG_ROUND_DONE = 0, GG_ROUND_AGAIN = 1, GG_ROUND_OVERFLOW = 2 };
typedef struct {
  gg_cmsg* send;                 /* device: [world][stride] records, the slots this rank sends */
  gg_cmsg* recv;                 /* device: [world][stride] records, the slots this rank receives */
  uint64_t* words_own;           /* device: [GG_ROUND_WORDS] this rank's status words */
  uint64_t* words_all;           /* device: [world][GG_ROUND_WORDS] every rank's (the all-gather's target) */
  uint64_t stride;               /* records per slot region (1 + capacity) */
  uint64_t slot;                 /* records of transport 1 per slot, header excluded */
  const uint64_t* send_count;    /* host [world]: records in send slot r (GG_ROUND_OVERFLOW) */
  const uint64_t* recv_count;    /* host [world]: records in receive slot r (GG_ROUND_OVERFLOW) */
  uint64_t next_q;               /* GG_ROUND_DONE: the quantum every rank runs next */
  int done;                      /* GG_ROUND_DONE: 1 when the run is over */
  int state;                     /* GG_ROUND_* after unpack / finish */
} gg_round_io;
gg_status gg_round_pack(gg_ctx* ctx, uint32_t world, uint32_t rank, uint64_t q, gg_round_io* io);
gg_status gg_round_unpack(gg_ctx* ctx, gg_round_io* io);
gg_status gg_round_finish(gg_ctx* ctx, gg_round_io* io);
/* tile_stats: [tiles][GG_NUM_TILE_STATS]; cache: [tiles][2][GG_NUM_CACHE_COUNTERS]
 * (either may be NULL); run_info: [GG_NUM_RUN_INFO] (may be NULL).  Tiles a
 * context does not own read 0.  Network counters: gg_noc_get_counters.      */
gg_status gg_coherent_get_stats(gg_ctx* ctx, uint64_t* tile_stats, uint64_t* cache, uint64_t* run_info);
/* The miss types of a coherent run with l1i_track_miss_types / l2_track_miss_types
 * set: out [tiles][2][GG_NUM_MISS_TYPES] (L1-D, L2), zeros for an untracked
 * cache.  Cache::getMissType (cache.cc:363-375) over the evicted /
 * invalidated / fetched address sets that insertCacheLine and
 * setCacheLineInfo keep (cache.cc:131-148, 228-230, 398-404).  The private
 * (Mode P) replay does not track them: gg_cache_access_batch returns
 * GG_ERR_UNSUPPORTED when either flag is set.                                */
gg_status gg_coherent_get_miss_types(gg_ctx* ctx, uint64_t* out);
/* The MOSI event counters of a coherent run: out [tiles][GG_NUM_PROTO_STATS]
 * (zeros under MSI; tiles a context does not own read 0).                   */
gg_status gg_coherent_get_protocol_stats(gg_ctx* ctx, uint64_t* out);

/* The sim.out text of the context's statistics (replaces the per-tile
 * outputSummary chain: TileManager::outputSummary, tile_manager_summary.cc:
 * 60-244 -> Tile / MemoryManager / Cache / DramPerfModel / DirectoryCache /
 * Network summaries).  GG_SUMMARY_BLOCKS: one "Tile t Summary:" block per
 * tile; GG_SUMMARY_TABLE: TileManager's table (one column per tile).  Coherent
 * mode after gg_coherent_run: memory (L1-D, L2, DRAM, directory) and network
 * blocks; private-cache mode: the cache summaries and the network blocks.
 * *needed = the text's bytes + 1; buf (host, cap bytes) receives the
 * NUL-terminated text when it fits, else GG_ERR_RANGE (buf NULL: size query). */
enum { GG_SUMMARY_BLOCKS = 0, GG_SUMMARY_TABLE = 1 };
gg_status gg_dump_summary(gg_ctx* ctx, int format, char* buf, uint64_t cap, uint64_t* needed);

/* Synthetic workload generator (not part of the reference boundary; the
 * reference has no trace capture): fills a tile-major trace of
 * `per_tile` records for tiles [tile_begin, tile_begin + tiles) with the
 * configs[1] generator of DESIGN.md §Workloads — record i of tile t is
 * z = SplitMix64(0x9E3779B97F4A7C15 ^ t) step first+i+1, line = z mod 2^lines_log2
 * at byte base t << base_shift, WRITE iff (z >> 32) % 3 == 0.                */
gg_status gg_gen_uniform_trace(uint64_t* addr_dev, uint32_t* meta_dev, uint32_t tile_begin,
                               uint32_t tiles, uint64_t per_tile, uint64_t first,
                               uint32_t lines_log2, uint32_t base_shift, void* stream);

/* configs[2..4] hotspot generator: record i of tile t,
 * z = SplitMix64(0x9E3779B97F4A7C15 ^ t) step first+i+1; hot iff
 * ((z >> 40) & 0xFF) < hot_frac256 -> line (z & 0xFFFFFFFF) % hot_lines at byte
 * 1 << 44, else line z mod 2^lines_log2 at t << base_shift; WRITE iff
 * ((z >> 32) & 0xFF) % 3 == 0; gap = ctz(((z>>48)&0xFF)|0x100) +
 * ctz(((z>>56)&0xFF)|0x100) core cycles in meta bits 1..30.                 */
/* configs[4] coherent stress trace: record i of tile t
 * is z = SplitMix64(0x9E3779B97F4A7C15 ^ t) step first+i+1; WRITE iff bit 32 of
 * z; with probability pool_frac256/256 (bits 40-47) line
 * g(t) + G * ((z mod 2^32) mod (pool_lines / G)) of the shared pool at byte
 * 2^45, where G = max(1, num_tiles / 64) groups and g(t) the tile's group
 * (lowbias32 hash of t + 0x9E3779B9, mod G), so each pool line has ~64
 * sharers; else line z mod 2^lines_log2 at byte t << base_shift; gap cycles as
 * the hotspot trace.                                                         */
gg_status gg_gen_stress_trace(uint64_t* addr_dev, uint32_t* meta_dev, uint32_t tile_begin, uint32_t tiles,
                              uint64_t per_tile, uint64_t first, uint32_t lines_log2, uint32_t base_shift,
                              uint32_t num_tiles, uint32_t pool_lines, uint32_t pool_frac256, void* stream);
gg_status gg_gen_hotspot_trace(uint64_t* addr_dev, uint32_t* meta_dev, uint32_t tile_begin, uint32_t tiles,
                               uint64_t per_tile, uint64_t first, uint32_t lines_log2, uint32_t base_shift,
                               uint32_t hot_lines, uint32_t hot_frac256, void* stream);

/* Multi-line accesses (replaces the line loop of Core::initiateMemoryAccess,
 * common/tile/core/core.cc:139-266, for the coherent mode).  Input: a
 * tile-major trace of accesses, device arrays addr_dev (byte address),
 * size_dev (bytes), meta_dev (WRITE bit, gap cycles), host tile_offsets
 * [tiles + 1].  Access i becomes the line records first_dev[i] ..
 * first_dev[i+1]-1 (first_dev: device, n + 1 entries): lines begin_aligned ..
 * end_aligned with the zero-size tail skipped (core.cc:167-197); the first
 * keeps the access's WRITE bit and gap, the others are WRITE | GG_META_CONT.
 * A zero-size access makes no line (core.cc:145-155); its gap cycles go to
 * the tile's next access.  line_addr_dev / line_meta_dev (capacity cap) may
 * both be NULL: then only *num_lines and first_dev are produced (size the
 * buffers, call again).  line_tile_offsets (host, may be NULL) receives the
 * line trace's tile offsets.  Synchronous on stream.  Errors: GG_ERR_INVALID
 * (bad arguments, more lines than cap, a carried gap >= 2^30 cycles).       */
gg_status gg_split_accesses(const uint64_t* addr_dev, const uint32_t* size_dev, const uint32_t* meta_dev,
                            const uint64_t* tile_offsets, uint32_t tiles, uint32_t line_size, uint64_t* first_dev,
                            uint64_t* line_addr_dev, uint32_t* line_meta_dev, uint64_t cap, uint64_t* num_lines,
                            uint64_t* line_tile_offsets, void* stream);
/* Per-access results of a coherent run of a split trace (core.cc:239-266):
 * latency_ps_dev[i] = final - initial time = the sum of the access's line
 * latencies (back to back); misses_dev[i] = its lines that did not hit the
 * L1-D on the first attempt (MemoryManager::__coreInitiateMemoryAccess's
 * return, l1_cache_cntlr.cc:100-179).  Either output may be NULL.           */
gg_status gg_combine_accesses(const uint64_t* line_out_dev, const uint64_t* first_dev, uint64_t n,
                              uint64_t* latency_ps_dev, uint32_t* misses_dev, void* stream);

/* Core timing of a trace-driven tile: the simple core model
 * (SimpleCoreModel::handleInstruction, common/tile/core/models/
 * simple_core_model.cc:43-96) over a coherent run's per-access results.  Each
 * access (a record without GG_META_CONT plus the CONT records that follow it)
 * is one instruction: static cost = its gap cycles (execution-unit stall),
 * one memory operand, read or write by the access's WRITE bit, whose latency
 * is the sum of its line latencies (Core::initiateMemoryAccess's final -
 * initial time, core.cc:239-256).  curr_time advances by cost + latency, which
 * is the coherent engine's clock rule, so GG_CORE_TIME_PS equals the run's
 * GG_CT_CLOCK_PS.  A BARRIER record whose access word holds a stall > 0 is
 * the SyncInstruction of sync_client.cc:306-314 (a dynamic instruction:
 * curr_time += stall, core_model.cc:237-240 counters).  No L1-I is modeled
 * (its stall is 0).  The iocoom model is
 * not offered: it needs register operands a memory trace does not carry and
 * would move the issue times the engine replays.
 * Per-tile statistics, [tile][GG_NUM_CORE_STATS]:                            */
enum {
  GG_CORE_INSTRUCTIONS = 0,   /* CoreModel::_instruction_count = data memory accesses  */
  GG_CORE_TIME_PS,            /* _curr_time                                             */
  GG_CORE_MEMORY_STALL_PS,    /* _total_memory_stall_time = total data access latency  */
  GG_CORE_EXECUTION_STALL_PS, /* _total_execution_unit_stall_time                      */
  GG_CORE_L1D_READ_STALL_PS,  /* SimpleCoreModel::_total_l1dcache_read_stall_time      */
  GG_CORE_L1D_WRITE_STALL_PS, /* _total_l1dcache_write_stall_time                      */
  GG_CORE_SYNC_INSTRUCTIONS,  /* _total_sync_instructions: released BARRIER records with a stall */
  GG_CORE_SYNC_STALL_PS,      /* _total_sync_instruction_stall_time                    */
  GG_NUM_CORE_STATS = 8
};
/* Runs the model over the tile-major trace (meta words and tile offsets of
 * `trace`; addresses are not read) and the per-record access words of the
 * coherent run (access_out_dev, (latency_ps << 2) | level), from the model's
 * constructor state; the statistics stay in the context (gg_core_get_stats,
 * gg_dump_summary's "Core Summary" block).  Asynchronous on stream.         */
gg_status gg_core_model_run(gg_ctx* ctx, const gg_trace* trace, const uint64_t* access_out_dev, void* stream);
/* out: num_tiles * GG_NUM_CORE_STATS (host).  Synchronizes.  GG_ERR_STATE if
 * gg_core_model_run has not run on the context.                              */
gg_status gg_core_get_stats(gg_ctx* ctx, uint64_t* out);

/* The iocoom core model (IOCOOMCoreModel, common/tile/core/models/
 * iocoom_core_model.cc; carbon_sim.cfg's default core type): an in-order core
 * with a register scoreboard and out-of-order memory through a load queue
 * and a store buffer.  Its time depends on register dependences, so it runs
 * over an INSTRUCTION stream, one gg_ins per instruction the core model
 * handles (CoreModel::iterate, core_model.cc:290-297), whose memory operands
 * take their DynamicMemoryInfo {address, read, latency} from an ACCESS
 * stream in order (Core::initiateMemoryAccess pushes one per access,
 * core.cc:258-263): per tile, the k-th memory operand of the instruction
 * stream (each instruction's reads, then its writes) is the k-th access.
 * The access stream's latencies are a coherent run's (gg_combine_accesses
 * of its line words, or its access words >> 2 for an unsplit trace): the
 * memory system is timed with the engine's issue times, and the core model
 * retimes the core around them (the reference feeds iocoom's curr_time back
 * as the next access's initial time; a trace carries no instructions between
 * its accesses to do that with).  Barriers likewise: a SYNC instruction
 * costs the stall the coherent engine measured (its release time minus the
 * engine's arrival time), taken as it is.  The reference's SyncClient
 * measures the stall on the core's own clock (sync_client.cc:308-313: time -
 * start_time); iocoom overlaps loads, so its arrival can be earlier and that
 * stall longer, and its clock after a barrier need not land on the common
 * release time.  Not recomputed here (nor in the oracle): parity unpinned.  */
typedef struct {
  uint16_t cost;     /* static cost in core cycles (Instruction::getCost: the
                        [core/static_instruction_costs] of its type, or a
                        branch's resolved cost); unused by a SYNC instruction */
  uint8_t  ops;      /* bits 0-1 memory read operands, bits 2-3 memory write
                        operands, GG_INS_SIMPLE_MOV_LOAD, GG_INS_ATOMIC,
                        GG_INS_FENCE_* in bits 6-7                             */
  uint8_t  regs;     /* bits 0-2 read registers, bits 3-5 write registers
                        (reads + writes <= 6), GG_INS_SYNC                     */
  uint16_t reg[6];   /* the read registers, then the write registers (< 512)  */
} gg_ins;
#define GG_INS_SIMPLE_MOV_LOAD 0x10u   /* Instruction::isSimpleMovMemoryLoad            */
#define GG_INS_ATOMIC          0x20u   /* Instruction::isAtomic (implicit MFENCE)        */
#define GG_INS_FENCE_SHIFT     6       /* 1 LFENCE, 2 SFENCE, 3 MFENCE (INST_*FENCE)    */
#define GG_INS_SYNC            0x80u   /* a SyncInstruction (dynamic): consumes the next
                                          access, which must be a BARRIER record, and
                                          costs its stall (sync_client.cc:306-314); a
                                          released barrier without a stall is no
                                          instruction, as in gg_core_model_run        */
#define GG_IOCOOM_NUM_REGISTERS 512    /* IOCOOMCoreModel::_NUM_REGISTERS               */
typedef struct {
  uint32_t num_load_queue_entries;             /* [core/iocoom] (1..64; default 8)    */
  uint32_t num_store_queue_entries;            /* (1..64; default 8)                   */
  uint32_t speculative_loads_enabled;          /* (default true)                       */
  uint32_t multiple_outstanding_RFOs_enabled;  /* (default true)                       */
} gg_iocoom_params;
/* Per-tile statistics, [tile][GG_NUM_IOCOOM_STATS]: */
enum {
  GG_IOCOOM_INSTRUCTIONS = 0,        /* CoreModel::_instruction_count                        */
  GG_IOCOOM_TIME_PS,                 /* _curr_time                                           */
  GG_IOCOOM_MEMORY_STALL_PS,         /* _total_memory_stall_time                             */
  GG_IOCOOM_EXECUTION_STALL_PS,      /* _total_execution_unit_stall_time                     */
  GG_IOCOOM_SYNC_INSTRUCTIONS,       /* _total_sync_instructions                             */
  GG_IOCOOM_SYNC_STALL_PS,           /* _total_sync_instruction_stall_time                   */
  GG_IOCOOM_LOAD_QUEUE_STALL_PS,     /* IOCOOMCoreModel::_total_load_queue_stall_time        */
  GG_IOCOOM_STORE_QUEUE_STALL_PS,    /* _total_store_queue_stall_time                        */
  GG_IOCOOM_L1I_STALL_PS,            /* _total_l1icache_stall_time (0: no L1-I)              */
  GG_IOCOOM_INTRA_L1D_STALL_PS,      /* _total_intra_ins_l1dcache_stall_time                 */
  GG_IOCOOM_INTER_L1D_STALL_PS,      /* _total_inter_ins_l1dcache_stall_time                 */
  GG_IOCOOM_INTRA_EXEC_STALL_PS,     /* _total_intra_ins_execution_unit_stall_time           */
  GG_IOCOOM_INTER_EXEC_STALL_PS,     /* _total_inter_ins_execution_unit_stall_time           */
  GG_IOCOOM_EXPLICIT_FENCES,         /* lfence + sfence + explicit mfence instructions       */
  GG_IOCOOM_IMPLICIT_MFENCES,        /* atomic instructions                                  */
  GG_IOCOOM_DATA_ACCESSES,           /* memory operands (Core's data memory accesses)        */
  GG_IOCOOM_DATA_LATENCY_PS,         /* their summed latency (Core::incrTotalMemoryAccessLatency) */
  GG_NUM_IOCOOM_STATS = 17
};
/* Runs IOCOOMCoreModel::handleInstruction over each tile's instructions
 * (ins_dev, host ins_tile_offsets[num_tiles + 1]) and accesses (acc_addr_dev
 * u64 address, acc_meta_dev u32 meta word — GG_META_WRITE or GG_META_BARRIER
 * — acc_lat_dev u64 latency in ps or a barrier's stall, host
 * acc_tile_offsets[num_tiles + 1]) from the model's constructor state.  A
 * memory read operand met by a write access (or the reverse), a SYNC met by
 * a non-BARRIER access, a register >= 512, a tile whose instructions leave
 * accesses unconsumed or run out of them, a register time of 2^62 ps or more
 * (the scoreboard keeps the unit in an entry's top two bits): the run's
 * error, reported by gg_iocoom_get_stats (GG_ERR_STATE).  GG_ERR_RANGE up
 * front for a tile of more than 2^31 instructions or accesses.
 * Asynchronous on stream.                                                    */
gg_status gg_iocoom_run(gg_ctx* ctx, const gg_iocoom_params* params, const gg_ins* ins_dev,
                        const uint64_t* ins_tile_offsets, const uint64_t* acc_addr_dev, const uint32_t* acc_meta_dev,
                        const uint64_t* acc_lat_dev, const uint64_t* acc_tile_offsets, void* stream);
/* out: num_tiles * GG_NUM_IOCOOM_STATS (host).  Synchronizes.  GG_ERR_STATE
 * if gg_iocoom_run has not run on the context or its streams disagreed.    */
gg_status gg_iocoom_get_stats(gg_ctx* ctx, uint64_t* out);

/* Device time (ms) of the most recent launch of a named kernel
 * ("cache_hist", "cache_scatter", "cache_replay", "cache_unshard",
 * "noc_hop_counter", ...), measured with HIP
 * events on the stream the kernel ran on; negative if not launched.           */
float     gg_kernel_time_ms(gg_ctx* ctx, const char* kernel);
/* enabled: 0 off; 1 on, coherent-mode launches sampled (an event pair around
 * every 16th launch of each kernel); 2 on, every coherent step / walk launch
 * timed in-kernel (first workgroup start to last workgroup end). */
void      gg_set_timing(gg_ctx* ctx, int enabled);
/* Launches since the last gg_coherent_begin of "coherent_step",
 * "coherent_walk_x", "coherent_walk_y" and their total device time: with
 * timing 1, (mean of the event-timed launches) x launches; with timing 2, the
 * sum of every launch's in-kernel span (s_memrealtime, 100 MHz).           */
gg_status gg_kernel_stats(gg_ctx* ctx, const char* kernel, double* total_ms, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif
