// graphite_host.hpp — C++ host side above the C ABI, mirroring the reference's
// in-process interfaces so a Graphite-style caller reads the same:
//
//   graphite_amd::Cache          Cache::accessCacheLine / insertCacheLine /
//                                getCacheLineInfo / setCacheLineInfo and
//                                outputSummary (common/tile/memory_subsystem/cache/cache.h:87-92,
//                                cache.cc:419-477), one (tile, level) of a context
//   graphite_amd::TraceReplayer  the per-access loop of Core::initiateMemoryAccess
//                                (common/tile/core/core.cc:139-266: line split,
//                                miss count) batched through gg_cache_access_batch
//   graphite_amd::NetworkModel   NetworkModel::routePacket (common/network/network_model.h:188)
//                                + __processReceivedPacket, batched through
//                                gg_noc_route_batch; Hop carries the same fields
//                                (network_model.h:45-63)
//
// Errors: the reference aborts through LOG_ASSERT_ERROR (common/misc/log.h:112-135);
// the mirror throws graphite_amd::Error carrying the ABI status and message.
// Only host memory crosses this header's API; device buffers are internal.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <iomanip>
#include <ostream>
#include <queue>
#include <stdexcept>
#include <algorithm>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/graphite_gpu.h"

namespace graphite_amd {

typedef uint64_t IntPtr;
typedef uint8_t Byte;

struct Error : std::runtime_error {
  gg_status status;
  Error(gg_status s, const std::string& m) : std::runtime_error(m), status(s) {}
};

inline void check(gg_status s, const char* what)
{
  if (s != GG_OK) throw Error(s, std::string(what) + ": " + gg_last_error());
}
inline void hip_check(hipError_t e, const char* what)
{
  if (e != hipSuccess) throw Error(GG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// CacheState::Type values of the MSI protocol (cache_state.h:11-21)
struct CacheState { enum Type { INVALID = 0, SHARED = 1, MODIFIED = 4 }; };
// MemComponent::Type values (mem_component.h:9-18)
struct MemComponent { enum Type { INVALID = 0, L1_DCACHE = 3 }; };

// PrL2CacheLineInfo (pr_l1_pr_l2_dram_directory_msi/cache_line_info.h)
class CacheLineInfo {
 public:
  explicit CacheLineInfo(IntPtr tag = ~(IntPtr)0, CacheState::Type cstate = CacheState::INVALID,
                         MemComponent::Type loc = MemComponent::INVALID)
  { _i.tag = tag; _i.cstate = cstate; _i.cached_loc = loc; }
  bool isValid() const { return _i.tag != ~(IntPtr)0; }
  IntPtr getTag() const { return _i.tag; }
  CacheState::Type getCState() const { return (CacheState::Type)_i.cstate; }
  MemComponent::Type getCachedLoc() const { return (MemComponent::Type)_i.cached_loc; }
  void setTag(IntPtr t) { _i.tag = t; }
  void setCState(CacheState::Type c) { _i.cstate = c; }
  void setCachedLoc(MemComponent::Type l) { _i.cached_loc = l; }
  void invalidate() { _i.tag = ~(IntPtr)0; _i.cstate = CacheState::INVALID; _i.cached_loc = MemComponent::INVALID; }
  gg_line_info* raw() { return &_i; }
 private:
  gg_line_info _i;
};

// RAII owner of one gg_ctx (one per GPU)
class Backend {
 public:
  explicit Backend(const gg_config& cfg) : _cfg(cfg)
  {
    gg_status st = GG_OK;
    _ctx = gg_create(&cfg, &st);
    if (!_ctx) check(st ? st : GG_ERR_INVALID, "gg_create");
  }
  ~Backend() { gg_destroy(_ctx); }
  Backend(const Backend&) = delete;
  Backend& operator=(const Backend&) = delete;
  gg_ctx* ctx() const { return _ctx; }
  const gg_config& config() const { return _cfg; }
  void reset() { check(gg_reset(_ctx), "gg_reset"); }
  std::vector<uint64_t> cacheCounters() const
  {
    std::vector<uint64_t> c((size_t)_cfg.num_tiles * 2 * GG_NUM_CACHE_COUNTERS);
    check(gg_cache_get_counters(_ctx, c.data()), "gg_cache_get_counters");
    return c;
  }
 private:
  gg_config _cfg;
  gg_ctx* _ctx = nullptr;
};

// Cache::outputSummary (cache.cc:419-477) for one cache's counters.  The empty
// write-miss-rate line keeps the reference's 4-space indent (cache.cc:445); the
// asynchronous-communication block is empty in a single DVFS domain.
inline void writeCacheSummary(std::ostream& out, const std::string& name, const uint64_t* c,
                              bool write_back, bool instruction_cache = false, const uint64_t* miss_types = nullptr)
{
  out << "  Cache " << name << ": " << std::endl;
  out << "    Cache Accesses: " << c[GG_CC_ACCESSES] << std::endl;
  out << "    Cache Misses: " << c[GG_CC_MISSES] << std::endl;
  if (c[GG_CC_ACCESSES] > 0)
    out << "    Miss Rate (%): " << 100.0 * c[GG_CC_MISSES] / c[GG_CC_ACCESSES] << std::endl;
  else
    out << "    Miss Rate (%): " << std::endl;
  if (!instruction_cache) {
    out << "      Read Accesses: " << c[GG_CC_READ_ACCESSES] << std::endl;
    out << "      Read Misses: " << c[GG_CC_READ_MISSES] << std::endl;
    if (c[GG_CC_READ_ACCESSES] > 0)
      out << "      Read Miss Rate (%): " << 100.0 * c[GG_CC_READ_MISSES] / c[GG_CC_READ_ACCESSES] << std::endl;
    else
      out << "      Read Miss Rate (%): " << std::endl;
    out << "      Write Accesses: " << c[GG_CC_WRITE_ACCESSES] << std::endl;
    out << "      Write Misses: " << c[GG_CC_WRITE_MISSES] << std::endl;
    if (c[GG_CC_WRITE_ACCESSES] > 0)
      out << "      Write Miss Rate (%): " << 100.0 * c[GG_CC_WRITE_MISSES] / c[GG_CC_WRITE_ACCESSES] << std::endl;
    else
      out << "    Write Miss Rate (%): " << std::endl;
  }
  out << "    Evictions: " << c[GG_CC_EVICTIONS] << std::endl;
  if (write_back) out << "    Dirty Evictions: " << c[GG_CC_DIRTY_EVICTIONS] << std::endl;
  if (miss_types) {                                   // track_miss_types (cache.cc:459-466)
    out << "    Miss Types:" << std::endl;
    out << "      Cold Misses: " << miss_types[GG_MT_COLD] << std::endl;
    out << "      Capacity Misses: " << miss_types[GG_MT_CAPACITY] << std::endl;
    out << "      Sharing Misses: " << miss_types[GG_MT_SHARING] << std::endl;
  }
  out << "    Event Counters:" << std::endl;
  out << "      Tag Array Reads: " << c[GG_CC_TAG_READS] << std::endl;
  out << "      Tag Array Writes: " << c[GG_CC_TAG_WRITES] << std::endl;
  out << "      Data Array Reads: " << c[GG_CC_DATA_READS] << std::endl;
  out << "      Data Array Writes: " << c[GG_CC_DATA_WRITES] << std::endl;
}

// Time::toNanosec / toCycles (misc/time_types.h:104-114)
inline uint64_t psToNanosec(uint64_t ps) { return (uint64_t)ceil(((double)ps) / double(1.0e3)); }
inline uint64_t psToCycles(uint64_t ps, double f) { return (uint64_t)ceil(((double)ps * f) / double(1.0e3)); }

// The core part of a tile's sim.out block for the simple core model over a
// trace (GG_CORE_* statistics of gg_core_model_run): CoreModel::outputSummary
// (core_model.cc:90-115) with the average frequency of the thread-exit
// recomputeAverageFrequency (:183-190), the default one_bit branch predictor's
// block (branch_predictor.cc:66-71: a memory trace has no branches), then
// SimpleCoreModel's breakdown (simple_core_model.cc:29-36) and
// Core::outputSummary's shared-memory block (core.cc:283-310; no L1-I).
// McPATCoreInterface's parameter and micro-op tables (mcpat_core_interface.cc:
// 780-1020) are not written: McPAT is not part of this path.
// CoreModel::outputSummary's lines (core_model.cc:90-115) for a model's
// instruction count, completion time, sync / stall totals and fence counts
inline void writeCoreModelSummary(std::ostream& os, uint64_t n, uint64_t t, uint64_t sync_n, uint64_t mem_ps,
                                  uint64_t ex_ps, uint64_t sync_ps, uint64_t explicit_fences, uint64_t implicit_fences,
                                  double frequency_ghz)
{
  const uint64_t zero = 0;
  const double avg_f = ((double)psToCycles(t, frequency_ghz)) / ((double)psToNanosec(t));
  os << "Core Summary:" << std::endl;
  os << "    Total Instructions: " << n << std::endl;
  os << "    Completion Time (in nanoseconds): " << psToNanosec(t) << std::endl;
  os << "    Average Frequency (in GHz): " << avg_f << std::endl;
  os << "    Synchronization Stalls: " << sync_n << std::endl;
  os << "    Network Recv Stalls: " << zero << std::endl;
  os << "    Stall Time Breakdown (in nanoseconds): " << std::endl;
  os << "      Memory: " << psToNanosec(mem_ps) << std::endl;
  os << "      Execution Unit: " << psToNanosec(ex_ps) << std::endl;
  os << "      Synchronization: " << psToNanosec(sync_ps) << std::endl;
  os << "      Network Recv: " << psToNanosec(0) << std::endl;
  os << "    Branch Predictor Statistics:" << std::endl
     << "      Num Correct: " << zero << std::endl
     << "      Num Incorrect: " << zero << std::endl;
  os << "    Fence Instructions: " << std::endl;
  os << "      Explicit LFENCE, SFENCE, MFENCE: " << explicit_fences << std::endl;
  os << "      Implicit MFENCE: " << implicit_fences << std::endl;
}
// Core::outputSummary's shared-memory block (core.cc:283-310; no L1-I)
inline void writeCoreMemorySummary(std::ostream& os, uint64_t nd, uint64_t data_ps)
{
  const uint64_t zero = 0, ni = 0, data_ns = psToNanosec(data_ps), instr_ns = psToNanosec(0);
  os << "Shared Memory Model Summary: " << std::endl;
  os << "    Total Memory Accesses: " << ni + nd << std::endl;
  os << "    Average Memory Access Latency (in nanoseconds): " << (1.0 * (instr_ns + data_ns) / (ni + nd)) << std::endl;
  os << "    Total Instruction Memory Accesses: " << ni << std::endl;
  os << "    Instruction Buffer Hits: " << zero << std::endl;
  os << "    Average Instruction Memory Access Latency (in nanoseconds): " << 1.0 * instr_ns / ni << std::endl;
  os << "    Total Data Memory Accesses: " << nd << std::endl;
  os << "    Average Data Memory Access Latency (in nanoseconds): " << 1.0 * data_ns / nd << std::endl;
}
inline void writeCoreSummary(std::ostream& os, const uint64_t* core, double frequency_ghz)
{
  const uint64_t n = core[GG_CORE_INSTRUCTIONS];
  writeCoreModelSummary(os, n, core[GG_CORE_TIME_PS], core[GG_CORE_SYNC_INSTRUCTIONS], core[GG_CORE_MEMORY_STALL_PS],
                        core[GG_CORE_EXECUTION_STALL_PS], core[GG_CORE_SYNC_STALL_PS], 0, 0, frequency_ghz);
  os << "    Detailed Stall Time Breakdown (in nanoseconds): " << std::endl;
  os << "      L1-I Cache: " << psToNanosec(0) << std::endl;
  os << "      L1-D Cache: "
     << psToNanosec(core[GG_CORE_L1D_READ_STALL_PS]) + psToNanosec(core[GG_CORE_L1D_WRITE_STALL_PS]) << std::endl;
  // data accesses (Core::_num_data_memory_accesses): the instructions but the sync ones
  writeCoreMemorySummary(os, n - core[GG_CORE_SYNC_INSTRUCTIONS], core[GG_CORE_MEMORY_STALL_PS]);
}
// The iocoom core model's part (GG_IOCOOM_* statistics of gg_iocoom_run):
// CoreModel::outputSummary, IOCOOMCoreModel's detailed breakdown
// (iocoom_core_model.cc:53-64), the shared-memory block.
inline void writeIocoomSummary(std::ostream& os, const uint64_t* io, double frequency_ghz)
{
  writeCoreModelSummary(os, io[GG_IOCOOM_INSTRUCTIONS], io[GG_IOCOOM_TIME_PS], io[GG_IOCOOM_SYNC_INSTRUCTIONS],
                        io[GG_IOCOOM_MEMORY_STALL_PS], io[GG_IOCOOM_EXECUTION_STALL_PS], io[GG_IOCOOM_SYNC_STALL_PS],
                        io[GG_IOCOOM_EXPLICIT_FENCES], io[GG_IOCOOM_IMPLICIT_MFENCES], frequency_ghz);
  os << "    Detailed Stall Time Breakdown (in nanoseconds): " << std::endl;
  os << "      Load Queue: " << psToNanosec(io[GG_IOCOOM_LOAD_QUEUE_STALL_PS]) << std::endl;
  os << "      Store Queue: " << psToNanosec(io[GG_IOCOOM_STORE_QUEUE_STALL_PS]) << std::endl;
  os << "      L1-I Cache: " << psToNanosec(io[GG_IOCOOM_L1I_STALL_PS]) << std::endl;
  os << "      L1-D Cache (Intra-Instruction): " << psToNanosec(io[GG_IOCOOM_INTRA_L1D_STALL_PS]) << std::endl;
  os << "      L1-D Cache (Inter-Instruction): " << psToNanosec(io[GG_IOCOOM_INTER_L1D_STALL_PS]) << std::endl;
  os << "      Execution Unit (Intra-Instruction): " << psToNanosec(io[GG_IOCOOM_INTRA_EXEC_STALL_PS]) << std::endl;
  os << "      Execution Unit (Inter-Instruction): " << psToNanosec(io[GG_IOCOOM_INTER_EXEC_STALL_PS]) << std::endl;
  writeCoreMemorySummary(os, io[GG_IOCOOM_DATA_ACCESSES], io[GG_IOCOOM_DATA_LATENCY_PS]);
}

// NetworkModel::outputSummary (network/network_model.cc:274-316) for one tile's
// GG_NC_* counters, followed for emesh_hop_counter by its event counters
// (network_model_emesh_hop_counter.cc:160-165,226-236).  Time::toCycles /
// toNanosec (misc/time_types.h:104-114) on the picosecond sums; averages are
// float, printed with the default ostream format.  The broadcast lines count
// gg_noc_route_tree's broadcasts (full_map itself never broadcasts).  The
// asynchronous-communication block is empty in a single DVFS domain.
inline void writeNetworkSummary(std::ostream& out, const uint64_t* nc, double frequency_ghz, uint32_t net_model,
                                bool contention_model_enabled = false)
{
  auto to_cycles = [&](uint64_t ps) { return (uint64_t)ceil(((double)ps * frequency_ghz) / double(1.0e3)); };
  auto to_ns = [](uint64_t ps) { return (uint64_t)ceil(((double)ps) / double(1.0e3)); };
  out << "    Total Packets Sent: " << nc[GG_NC_PACKETS_SENT] << std::endl;
  out << "    Total Flits Sent: " << nc[GG_NC_FLITS_SENT] << std::endl;
  out << "    Total Bits Sent: " << nc[GG_NC_BITS_SENT] << std::endl;
  out << "    Total Packets Broadcasted: " << nc[GG_NC_PACKETS_BROADCASTED] << std::endl;
  out << "    Total Flits Broadcasted: " << nc[GG_NC_FLITS_BROADCASTED] << std::endl;
  out << "    Total Bits Broadcasted: " << nc[GG_NC_BITS_BROADCASTED] << std::endl;
  out << "    Total Packets Received: " << nc[GG_NC_PACKETS_RECEIVED] << std::endl;
  out << "    Total Flits Received: " << nc[GG_NC_FLITS_RECEIVED] << std::endl;
  out << "    Total Bits Received: " << nc[GG_NC_BITS_RECEIVED] << std::endl;
  const uint64_t n = nc[GG_NC_PACKETS_RECEIVED];
  if (n > 0) {
    const uint64_t lat = nc[GG_NC_TOTAL_LATENCY_PS], con = nc[GG_NC_TOTAL_CONTENTION_PS];
    out << "    Average Packet Latency (in clock cycles): " << ((float)to_cycles(lat)) / n << std::endl;
    out << "    Average Packet Latency (in nanoseconds): " << ((float)to_ns(lat)) / n << std::endl;
    out << "    Average Contention Delay (in clock cycles): " << ((float)to_cycles(con)) / n << std::endl;
    out << "    Average Contention Delay (in nanoseconds): " << ((float)to_ns(con)) / n << std::endl;
  } else {
    out << "    Average Packet Latency (in clock cycles): 0" << std::endl;
    out << "    Average Packet Latency (in nanoseconds): 0" << std::endl;
    out << "    Average Contention Delay (in clock cycles): 0" << std::endl;
    out << "    Average Contention Delay (in nanoseconds): 0" << std::endl;
  }
  if (net_model == GG_NET_EMESH_HOP_COUNTER) {
    out << "    Event Counters:" << std::endl;
    out << "      Buffer Writes: " << nc[GG_NC_BUFFER_WRITES] << std::endl;
    out << "      Buffer Reads: " << nc[GG_NC_BUFFER_READS] << std::endl;
    out << "      Switch Allocator Traversals: " << nc[GG_NC_SWITCH_ALLOC] << std::endl;
    out << "      Crossbar Traversals: " << nc[GG_NC_CROSSBAR] << std::endl;
    out << "      Link Traversals: " << nc[GG_NC_LINK_TRAVERSALS] << std::endl;
  }
  if (net_model == GG_NET_EMESH_HOP_BY_HOP) {
    // outputEventCountSummary (network_model_emesh_hop_by_hop.cc:436-462):
    // Crossbar[m] = traversals of routings to m output ports (m > 1: broadcast tree)
    out << "    Event Counters:" << std::endl;
    out << "      Buffer Writes: " << nc[GG_NC_BUFFER_WRITES] << std::endl;
    out << "      Buffer Reads: " << nc[GG_NC_BUFFER_READS] << std::endl;
    out << "      Switch Allocator Requests: " << nc[GG_NC_SWITCH_ALLOC] << std::endl;
    for (int i = 1; i <= 5; ++i)
      out << "      Crossbar[" << i << "] Traversals: " << (i == 1 ? nc[GG_NC_CROSSBAR] : nc[GG_NC_CROSSBAR_MULTI + i - 2])
          << std::endl;
    out << "      Link Traversals: " << nc[GG_NC_LINK_TRAVERSALS] << std::endl;
    if (contention_model_enabled) {
      // outputContentionModelsSummary (:464-486) over mesh ports 0..4 with
      // RouterModel::getAverageContentionDelay / getAverageLinkUtilization /
      // getPercentAnalyticalModelsUsed (router_model.cc:145-215), all float
      const uint64_t pk = nc[GG_NC_ROUTER_PACKETS];
      const float avg_delay = pk > 0 ? ((float)nc[GG_NC_ROUTER_CONTENTION_CYCLES]) / pk : 0.0f;
      float util = 0.0f;
      for (int p = 0; p < 5; ++p) {
        const uint64_t last = nc[GG_NC_PORT_LAST_CYCLES + p];
        util += last > 0 ? ((float)nc[GG_NC_PORT_UTILIZED_CYCLES + p]) / last : 0.0f;   // QueueModel::getQueueUtilization
      }
      util = util / 5;
      const float an = pk > 0 ? ((float)nc[GG_NC_ANALYTICAL_REQUESTS] * 100) / pk : 0.0f;
      out << "    Contention Counters:" << std::endl;
      out << "      Average EMesh Router Contention Delay: " << avg_delay << std::endl;
      out << "      Average EMesh Router Link Utilization: " << util << std::endl;
      out << "      Analytical Models Used (%): " << an << std::endl;
    }
  }
}

// DramPerfModel::outputSummary (performance_models/dram_perf_model.cc:131-164)
// for one tile's GG_CT_* stats of the coherent mode.  The averages are double
// sums divided by the access count, printed as float (0 accesses print the
// x86 default NaN, "-nan", as the reference does); the queue block exists for
// history_list / history_tree only and reads QueueModel::getQueueUtilization
// (queue_model.cc:57-62) and the analytical-request fraction, both float.
inline void writeDramSummary(std::ostream& out, const uint64_t* st, bool queue_model_enabled, uint32_t queue_type)
{
  const uint64_t n = st[GG_CT_DRAM_ACCESSES];
  const double lat = (double)st[GG_CT_DRAM_LATENCY_NS], qd = (double)st[GG_CT_DRAM_QUEUE_DELAY_NS];
  out << "Dram Performance Model Summary: " << std::endl;
  out << "    Total Dram Accesses: " << n << std::endl;
  out << "    Average Dram Access Latency (in nanoseconds): " << (float)(lat / n) << std::endl;
  out << "    Average Dram Contention Delay (in nanoseconds): " << (float)(qd / n) << std::endl;
  if (queue_model_enabled && (queue_type == GG_QM_HISTORY_LIST || queue_type == GG_QM_HISTORY_TREE)) {
    const uint64_t total_cycles = st[GG_CT_DRAM_QUEUE_LAST_NS];
    const float util = total_cycles > 0 ? ((float)st[GG_CT_DRAM_QUEUE_UTILIZED_NS]) / total_cycles : 0.0f;
    const float frac = ((float)st[GG_CT_DRAM_QUEUE_ANALYTICAL]) / st[GG_CT_DRAM_QUEUE_REQUESTS];
    out << "    Queue Model:" << std::endl;
    out << "      Queue Utilization(%): " << util * 100 << std::endl;
    out << "      Analytical Model Used(%): " << frac * 100 << std::endl;
  }
}

// DirectoryCache sizing of a coherent configuration (directory_cache.cc:46-59,
// 243-322): auto total entries from the L2 size, full-map entry bytes =
// ceil(application tiles / 8) (DirectoryEntry::getSize, directory_entry.cc:75-92),
// auto access cycles from the directory size.
struct DirectorySizing {
  uint32_t total_entries, size_kb;
  uint64_t access_cycles;
  bool auto_entries, auto_cycles;
};
inline DirectorySizing directorySizing(const gg_config& c)
{
  DirectorySizing d;
  d.auto_entries = c.dir_total_entries == 0;
  d.auto_cycles = c.dir_access_cycles == 0;
  if (d.auto_entries) {
    uint32_t sets = (uint32_t)ceil(2.0 * c.l2_size_kb * 1024 * c.num_tiles / (1.0 * c.line_size * c.dir_assoc * c.num_tiles));
    uint32_t lg = 0;
    while ((1u << lg) < sets) ++lg;
    d.total_entries = (1u << lg) * c.dir_assoc;
  } else d.total_entries = c.dir_total_entries;
  const uint64_t size = (uint64_t)d.total_entries * (uint64_t)ceil(1.0 * c.num_tiles / 8);
  d.size_kb = (uint32_t)ceil(1.0 * size / 1024);
  const uint32_t kb = d.size_kb;
  d.access_cycles = !d.auto_cycles ? c.dir_access_cycles
                  : kb <= 16 ? 1 : kb <= 32 ? 2 : kb <= 64 ? 4 : kb <= 128 ? 6 : kb <= 256 ? 8
                  : kb <= 512 ? 10 : kb <= 1024 ? 13 : kb <= 2048 ? 16 : 20;
  return d;
}

// "Dram Directory Summary:" (MemoryManager::outputSummary, msi/memory_manager.cc:427-428)
// + DirectoryCache::outputSummary (directory_cache.cc:350-369, 385-398).  The
// asynchronous-communication block is empty in a single DVFS domain.
inline void writeDirectorySummary(std::ostream& out, const uint64_t* st, const DirectorySizing& d)
{
  out << "Dram Directory Summary:\n";
  if (d.auto_entries) {
    out << "    Total Entries [auto-generated]: " << d.total_entries << std::endl;
    out << "    Size (in KB) [auto-generated]: " << d.size_kb << std::endl;
  }
  if (d.auto_cycles) out << "    Access Time (in clock cycles) [auto-generated]: " << d.access_cycles << std::endl;
  out << "    Total Accesses: " << st[GG_CT_DIR_ACCESSES] << std::endl;
  out << "    Total Evictions: " << st[GG_CT_DIR_EVICTIONS] << std::endl;
  out << "    Total Back-Invalidations: " << st[GG_CT_DIR_BACK_INVALIDATIONS] << std::endl;
}

// MOSI: L2CacheCntlr::outputSummary (…mosi/l2_cache_cntlr.cc:638-649) for one
// tile's GG_PS_* counters
inline void writeMosiL2CntlrSummary(std::ostream& out, const uint64_t* ps)
{
  out << "    L2 Cache Cntlr: " << std::endl;
  out << "      Total Invalidations: " << ps[GG_PS_L2_INVALIDATIONS] << std::endl;
  out << "      Total Evictions: " << ps[GG_PS_L2_EVICTIONS] << std::endl;
  out << "        Exclusive Request - Dirty Evictions: " << ps[GG_PS_L2_DIRTY_EVICTIONS_EXREQ] << std::endl;
  out << "        Exclusive Request - Clean Evictions: " << ps[GG_PS_L2_CLEAN_EVICTIONS_EXREQ] << std::endl;
  out << "        Shared Request - Dirty Evictions: " << ps[GG_PS_L2_DIRTY_EVICTIONS_SHREQ] << std::endl;
  out << "        Shared Request - Clean Evictions: " << ps[GG_PS_L2_CLEAN_EVICTIONS_SHREQ] << std::endl;
}

// MOSI: DramDirectoryCntlr::outputSummary (…mosi/dram_directory_cntlr.cc:1041-1142).
// The averages are (float) Time::toNanosec() (ceil of ps / 1000, time_types.h:111-114)
// over (float) counts; a block with no requests prints its labels only.
inline void writeMosiDirectoryCntlrSummary(std::ostream& out, const uint64_t* ps)
{
  auto ns = [](uint64_t p) { return (float)(uint64_t)ceil((double)p / 1.0e3); };
  auto avg_ns = [&](uint64_t p, uint64_t n) { return ns(p) / (float)n; };
  const uint64_t ex = ps[GG_PS_EXREQ], sh = ps[GG_PS_SHREQ], nu = ps[GG_PS_NULLIFY];
  out << "Dram Directory Cntlr: " << std::endl;
  out << "    Total Requests: " << ex + sh + nu << std::endl;
  out << "    Exclusive Requests: " << ex << std::endl;
  out << "    Shared Requests: " << sh << std::endl;
  out << "    Nullify Requests: " << nu << std::endl;
  if (ex > 0) {
    out << "    Exclusive Request - MODIFIED State: " << ps[GG_PS_EXREQ_MODIFIED] << std::endl;
    out << "    Exclusive Request - SHARED State: " << ps[GG_PS_EXREQ_SHARED] << std::endl;
    out << "    Exclusive Request - UNCACHED State: " << ps[GG_PS_EXREQ_UNCACHED] << std::endl;
    out << "    Exclusive Request - Upgrade Reply: " << ps[GG_PS_EXREQ_UPGRADE] << std::endl;
    out << "    Average Exclusive Request Serialization Time (in nanoseconds): " << avg_ns(ps[GG_PS_EXREQ_SERIALIZATION_PS], ex) << std::endl;
    out << "    Average Exclusive Request Processing Time (in nanoseconds): " << avg_ns(ps[GG_PS_EXREQ_PROCESSING_PS], ex) << std::endl;
  } else {
    out << "    Exclusive Request - MODIFIED State: " << std::endl;
    out << "    Exclusive Request - SHARED State: " << std::endl;
    out << "    Exclusive Request - UNCACHED State: " << std::endl;
    out << "    Exclusive Request - Upgrade Reply: " << std::endl;
    out << "    Average Exclusive Request Serialization Time (in nanoseconds): " << std::endl;
    out << "    Average Exclusive Request Processing Time (in nanoseconds): " << std::endl;
  }
  if (sh > 0) {
    out << "    Shared Request - MODIFIED State: " << ps[GG_PS_SHREQ_MODIFIED] << std::endl;
    out << "    Shared Request - SHARED State: " << ps[GG_PS_SHREQ_SHARED] << std::endl;
    out << "    Shared Request - UNCACHED State: " << ps[GG_PS_SHREQ_UNCACHED] << std::endl;
    out << "    Average Shared Request Serialization Time (in nanoseconds): " << avg_ns(ps[GG_PS_SHREQ_SERIALIZATION_PS], sh) << std::endl;
    out << "    Average Shared Request Processing Time (in nanoseconds): " << avg_ns(ps[GG_PS_SHREQ_PROCESSING_PS], sh) << std::endl;
  } else {
    out << "    Shared Request - MODIFIED State: " << std::endl;
    out << "    Shared Request - SHARED State: " << std::endl;
    out << "    Shared Request - UNCACHED State: " << std::endl;
    out << "    Average Shared Request Serialization Time (in nanoseconds): " << std::endl;
    out << "    Average Shared Request Processing Time (in nanoseconds): " << std::endl;
  }
  if (nu > 0) {
    out << "    Nullify Request - MODIFIED State: " << ps[GG_PS_NULLIFY_MODIFIED] << std::endl;
    out << "    Nullify Request - SHARED State: " << ps[GG_PS_NULLIFY_SHARED] << std::endl;
    out << "    Nullify Request - UNCACHED State: " << ps[GG_PS_NULLIFY_UNCACHED] << std::endl;
    out << "    Average Nullify Request Serialization Time (in nanoseconds): " << avg_ns(ps[GG_PS_NULLIFY_SERIALIZATION_PS], nu) << std::endl;
    out << "    Average Nullify Request Processing Time (in nanoseconds): " << avg_ns(ps[GG_PS_NULLIFY_PROCESSING_PS], nu) << std::endl;
  } else {
    out << "    Nullify Request - MODIFIED State: " << std::endl;
    out << "    Nullify Request - SHARED State: " << std::endl;
    out << "    Nullify Request - UNCACHED State: " << std::endl;
    out << "    Average Nullify Request Serialization Time (in nanoseconds): " << std::endl;
    out << "    Average Nullify Request Processing Time (in nanoseconds): " << std::endl;
  }
  const uint64_t iu = ps[GG_PS_INV_UNICAST], ib = ps[GG_PS_INV_BROADCAST];
  out << "    Total Invalidation Requests - Unicast Mode: " << iu << std::endl;
  if (iu > 0) {
    out << "    Average Sharers Invalidated - Unicast Mode: " << (float)ps[GG_PS_INV_SHARERS_UNICAST] / (float)iu << std::endl;
    out << "    Average Invalidation Processing Time - Unicast Mode (in nanoseconds): " << avg_ns(ps[GG_PS_INV_PROCESSING_UNICAST_PS], iu) << std::endl;
  } else {
    out << "    Average Sharers Invalidated - Unicast Mode: " << std::endl;
    out << "    Average Invalidation Processing Time - Unicast Mode (in nanoseconds): " << std::endl;
  }
  out << "    Total Invalidation Requests - Broadcast Mode: " << ib << std::endl;
  if (ib > 0) {
    out << "    Average Sharers Invalidated - Broadcast Mode: " << (float)ps[GG_PS_INV_SHARERS_BROADCAST] / (float)ib << std::endl;
    out << "    Average Invalidation Processing Time - Broadcast Mode (in nanoseconds): " << avg_ns(ps[GG_PS_INV_PROCESSING_BROADCAST_PS], ib) << std::endl;
  } else {
    out << "    Average Sharers Invalidated - Broadcast Mode: " << std::endl;
    out << "    Average Invalidation Processing Time - Broadcast Mode (in nanoseconds): " << std::endl;
  }
}

// The memory part of one tile's sim.out block in the coherent mode
// (msi/memory_manager.cc:415-430): Cache Summary (L1-D, L2; no L1-I is
// modeled), then the DRAM and directory summaries (sh_l2: no directory block).  MOSI
// (…mosi/memory_manager.cc:412-436, proto = the tile's GG_PS_* counters): the
// L2 and directory controllers' blocks after the caches, the directory cache
// before the DRAM.
inline void writeMemorySummary(std::ostream& out, const gg_config& c, const uint64_t* tile_stats,
                               const uint64_t* cache_counters, const uint64_t* miss_types = nullptr,
                               const uint64_t* proto = nullptr)
{
  const bool mosi = c.protocol == GG_PROTO_MOSI, shl2 = c.protocol >= GG_PROTO_SHL2_MSI;   // (sh_l2 MSI or MESI)
  const bool l1_mt = (mosi || shl2) ? c.l1d_track_miss_types : c.l1i_track_miss_types;
  out << "Cache Summary:\n";
  // (the L1-D is write-back under pr_l1_sh_l2_msi, …sh_l2_msi/l1_cache_cntlr.cc:57)
  writeCacheSummary(out, "L1-D", cache_counters, shl2, false, miss_types && l1_mt ? miss_types : nullptr);
  writeCacheSummary(out, "L2", cache_counters + GG_NUM_CACHE_COUNTERS, true, false,
                    miss_types && c.l2_track_miss_types ? miss_types + GG_NUM_MISS_TYPES : nullptr);
  if (mosi) {
    static const uint64_t zero_ps[GG_NUM_PROTO_STATS] = {0};
    writeMosiL2CntlrSummary(out, proto ? proto : zero_ps);
    writeMosiDirectoryCntlrSummary(out, proto ? proto : zero_ps);
    writeDirectorySummary(out, tile_stats, directorySizing(c));
    writeDramSummary(out, tile_stats, c.dram_queue_model_enabled != 0, c.dram_queue_model_type);
    return;
  }
  writeDramSummary(out, tile_stats, c.dram_queue_model_enabled != 0, c.dram_queue_model_type);
  // pr_l1_sh_l2_msi (…sh_l2_msi/memory_manager.cc:411-429): the L2 slice is the
  // directory, so no directory-cache block
  if (!shl2) writeDirectorySummary(out, tile_stats, directorySizing(c));
}

// One tile's summary text in the coherent mode: the core part when the core
// model has run (gg_core_model_run), the memory part, then
// Network::outputSummary (network.cc:79-89): the static networks below SYSTEM,
// User (no traffic in a trace-driven run; emesh_hop_counter, carbon_sim.cfg
// [network]) then Memory.  Mode P (no tile statistics): the cache summary only,
// then the networks.
inline void writeTileSummary(std::ostream& os, const gg_config& cfg, const uint64_t* tile_stats,
                             const uint64_t* cache_counters, const uint64_t* net_counters,
                             const uint64_t* core_stats = nullptr, const uint64_t* miss_types = nullptr,
                             const uint64_t* proto = nullptr, const uint64_t* iocoom_stats = nullptr)
{
  static const uint64_t zero_net[GG_NUM_NET_COUNTERS] = {0};
  // Tile::outputSummary (tile.cc:52-69): the tile's core model (iocoom when gg_iocoom_run ran)
  if (iocoom_stats) writeIocoomSummary(os, iocoom_stats, cfg.frequency_ghz);
  else if (core_stats) writeCoreSummary(os, core_stats, cfg.frequency_ghz);
  if (tile_stats) writeMemorySummary(os, cfg, tile_stats, cache_counters, miss_types, proto);
  else {
    os << "Cache Summary:\n";
    writeCacheSummary(os, "L1-D", cache_counters, false);
    writeCacheSummary(os, "L2", cache_counters + GG_NUM_CACHE_COUNTERS, true);
  }
  os << "Network Summary: " << std::endl << "  Network (User): " << std::endl;
  writeNetworkSummary(os, zero_net, cfg.frequency_ghz, GG_NET_EMESH_HOP_COUNTER);
  os << "  Network (Memory): " << std::endl;
  writeNetworkSummary(os, net_counters, cfg.frequency_ghz, cfg.net_model, cfg.queue_model_enabled != 0);
}

// TileManager::outputSummary's table (tile_manager_summary.cc:60-198): every
// tile's summary text ("label: value" lines) becomes one column, the row
// headings are the labels of tile 0's lines, the columns are padded to their
// widest cell and closed by " | ".  Restated with the reference's own string
// scanning (std::string::find, npos wrapping included), so summaries that do
// not follow the "label: value" form come out exactly as the reference lays
// them out.
inline std::string formatTileSummaries(const std::vector<std::string>& summaries)
{
  if (summaries.empty()) return std::string();
  const size_t cols = summaries.size() + 1;
  const size_t rows = (size_t)std::count(summaries[0].begin(), summaries[0].end(), '\n') + 1;   // formatSummaries (:184-187)
  std::vector<std::string> cell(rows * cols);
  auto at = [&](size_t r, size_t c) -> std::string& { return cell[r * cols + c]; };
  {                                                                 // addRowHeadings (:135-151)
    const std::string& sum = summaries[0];
    std::string::size_type pos = 0;
    for (size_t i = 1; i < rows; ++i) {
      const std::string::size_type end = sum.find(':', pos);
      at(i, 0) = sum.substr(pos, end - pos);
      pos = sum.find('\n', pos) + 1;
    }
  }
  for (size_t i = 0; i + 1 < cols; ++i) at(0, i + 1) = "Tile " + std::to_string(i);   // addColHeadings (:153-161)
  for (size_t t = 0; t < summaries.size(); ++t) {                   // addTileSummary (:163-176)
    const std::string& summary = summaries[t];
    std::string::size_type pos = summary.find(':') + 1;
    for (size_t i = 1; i < rows; ++i) {
      const std::string::size_type end = summary.find('\n', pos);
      at(i, t + 1) = summary.substr(pos, end - pos);
      pos = summary.find(':', pos) + 1;
    }
  }
  std::vector<size_t> w(cols, 0);                                   // Table::flatten (:87-115)
  for (size_t r = 0; r < rows; ++r)
    for (size_t c = 0; c < cols; ++c) w[c] = std::max(w[c], at(r, c).length());
  std::ostringstream out;
  for (size_t r = 0; r < rows; ++r) {
    for (size_t c = 0; c < cols; ++c) out << at(r, c) << std::string(w[c] - at(r, c).length(), ' ') << " | ";
    out << '\n';
  }
  return out.str();
}

// One cache (tile, level) of a Backend with the reference Cache API.
class Cache {
 public:
  enum AccessType { LOAD = 0, STORE };
  Cache(Backend& be, uint32_t tile, int level) : _be(be), _tile(tile), _level(level) {}

  void accessCacheLine(IntPtr address, AccessType access_type, Byte* /*buf*/ = nullptr, uint32_t /*num_bytes*/ = 0)
  {
    check(gg_cache_access_line(_be.ctx(), _tile, _level, address, access_type == STORE), "Cache::accessCacheLine");
  }
  void insertCacheLine(IntPtr inserted_address, CacheLineInfo* inserted, Byte* /*fill_buf*/, bool* eviction,
                       IntPtr* evicted_address, CacheLineInfo* evicted, Byte* /*writeback_buf*/)
  {
    int ev = 0;
    check(gg_cache_insert_line(_be.ctx(), _tile, _level, inserted_address, inserted->raw(), &ev, evicted_address,
                               evicted->raw()), "Cache::insertCacheLine");
    *eviction = ev != 0;
  }
  void getCacheLineInfo(IntPtr address, CacheLineInfo* info)
  {
    check(gg_cache_get_line_info(_be.ctx(), _tile, _level, address, info->raw()), "Cache::getCacheLineInfo");
  }
  void setCacheLineInfo(IntPtr address, CacheLineInfo* info)
  {
    check(gg_cache_set_line_info(_be.ctx(), _tile, _level, address, info->raw()), "Cache::setCacheLineInfo");
  }
  void outputSummary(std::ostream& out) const
  {
    std::vector<uint64_t> c = _be.cacheCounters();
    writeCacheSummary(out, _level == GG_L1D ? "L1-D" : "L2",
                      &c[((size_t)_tile * 2 + _level) * GG_NUM_CACHE_COUNTERS], _level == GG_L2);
  }
 private:
  Backend& _be;
  uint32_t _tile;
  int _level;
};

// Device buffer helper
template <class T>
struct DeviceBuffer {
  T* p = nullptr;
  size_t n = 0;
  void resize(size_t want)
  {
    if (want <= n && p) return;
    if (p) hipFree(p);
    hip_check(hipMalloc((void**)&p, sizeof(T) * (want ? want : 1)), "hipMalloc");
    n = want;
  }
  ~DeviceBuffer() { if (p) hipFree(p); }
};

// Core::initiateMemoryAccess line split (core.cc:167-201): the line-aligned
// addresses touched by [address, address + size), zero-size tail skipped.
inline void splitIntoLines(IntPtr address, uint32_t size, uint32_t line, std::vector<IntPtr>& out)
{
  if (size == 0) return;
  const IntPtr begin = address, end = address + size;
  const IntPtr ba = begin - (begin % line), ea = end - (end % line);
  for (IntPtr a = ba; a <= ea; a += line) {
    const uint32_t off = (a == ba) ? (uint32_t)(begin % line) : 0;
    if (a == ea && (uint32_t)(end % line) - off == 0) continue;
    out.push_back(a);
  }
}

// Per-tile line-access trace, replayed in batches through the private-cache
// backend (the batched accessSingleLine of the north star).
class TraceReplayer {
 public:
  explicit TraceReplayer(Backend& be) : _be(be), _lines(be.config().num_tiles), _meta(be.config().num_tiles) {}

  // Core::initiateMemoryAccess(L1_DCACHE, ..., READ/WRITE, address, size): queue its line accesses
  void initiateMemoryAccess(uint32_t tile, bool is_write, IntPtr address, uint32_t size)
  {
    const size_t before = _lines.at(tile).size();
    splitIntoLines(address, size, _be.config().line_size, _lines[tile]);
    _meta[tile].resize(_lines[tile].size(), is_write ? GG_META_WRITE : 0u);
    (void)before;
  }
  void accessSingleLine(uint32_t tile, bool is_write, IntPtr line_address)
  {
    _lines.at(tile).push_back(line_address);
    _meta[tile].push_back(is_write ? GG_META_WRITE : 0u);
  }
  size_t pending() const { size_t n = 0; for (auto& v : _lines) n += v.size(); return n; }

  // Replay everything queued; returns the per-access GG_RES_* words in
  // tile-major order of the queued accesses.
  std::vector<uint32_t> flush(hipStream_t stream = nullptr)
  {
    const uint32_t T = _be.config().num_tiles;
    std::vector<uint64_t> offs(T + 1, 0), addr;
    std::vector<uint32_t> meta;
    for (uint32_t t = 0; t < T; ++t) {
      offs[t + 1] = offs[t] + _lines[t].size();
      addr.insert(addr.end(), _lines[t].begin(), _lines[t].end());
      meta.insert(meta.end(), _meta[t].begin(), _meta[t].end());
      _lines[t].clear();
      _meta[t].clear();
    }
    const size_t n = addr.size();
    std::vector<uint32_t> res(n);
    _addr.resize(n); _m.resize(n); _res.resize(n);
    if (n) {
      hip_check(hipMemcpyAsync(_addr.p, addr.data(), 8 * n, hipMemcpyHostToDevice, stream), "copy addr");
      hip_check(hipMemcpyAsync(_m.p, meta.data(), 4 * n, hipMemcpyHostToDevice, stream), "copy meta");
    }
    gg_trace tr{_addr.p, _m.p, offs.data(), n};
    check(gg_cache_access_batch(_be.ctx(), &tr, _res.p, nullptr, stream), "gg_cache_access_batch");
    if (n) hip_check(hipMemcpyAsync(res.data(), _res.p, 4 * n, hipMemcpyDeviceToHost, stream), "copy result");
    hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    return res;
  }

  // "Cache Summary:" block of every tile (MemoryManager::outputSummary,
  // pr_l1_pr_l2_dram_directory_msi/memory_manager.cc:415-430, L1-D and L2 only)
  void outputSummary(std::ostream& out) const
  {
    std::vector<uint64_t> c = _be.cacheCounters();
    for (uint32_t t = 0; t < _be.config().num_tiles; ++t) {
      out << "Tile " << t << " Cache Summary:" << std::endl;
      writeCacheSummary(out, "L1-D", &c[((size_t)t * 2 + 0) * GG_NUM_CACHE_COUNTERS], false);
      writeCacheSummary(out, "L2", &c[((size_t)t * 2 + 1) * GG_NUM_CACHE_COUNTERS], true);
    }
  }

 private:
  Backend& _be;
  std::vector<std::vector<IntPtr>> _lines;
  std::vector<std::vector<uint32_t>> _meta;
  DeviceBuffer<uint64_t> _addr;
  DeviceBuffer<uint32_t> _m, _res;
};

// NetworkModel::routePacket mirror.  NetPacket/Hop keep the reference fields
// that carry timing (network.h:27-55, network_model.h:45-63).
struct NetPacket {
  uint64_t time_ps = 0;         // NetPacket::time
  uint32_t sender = 0, receiver = 0;
  uint32_t modeled_length_bits = 0;   // NetworkModel::getModeledLength
  uint64_t zero_load_delay_ps = 0, contention_delay_ps = 0;
};
struct Hop {
  uint32_t next_tile_id;
  int32_t next_node_type;       // RECEIVE_TILE
  uint64_t time_ps, zero_load_delay_ps, contention_delay_ps;
};
enum { RECEIVE_TILE = 2 };

// QueueModel::create (shared_models/queue_model.cc:19-39): the type string of
// network/emesh_hop_by_hop/queue_model/type or dram/queue_model/type ->
// gg_config.queue_model_type / dram_queue_model_type.  Unknown types are an
// error, as LOG_PRINT_ERROR("Unrecognized Queue Model Type") in the reference.
inline uint32_t queueModelType(const std::string& type)
{
  if (type == "history_tree") return GG_QM_HISTORY_TREE;
  if (type == "history_list") return GG_QM_HISTORY_LIST;
  if (type == "basic") return GG_QM_BASIC;
  throw std::invalid_argument("Unrecognized Queue Model Type(" + type + ")");
}
// MovingAverage::createAvgType (common/misc/moving_average.h) for
// queue_model/basic: packs moving_avg_{enabled,type,window_size} into
// gg_config.basic_moving_avg.
inline uint32_t basicMovingAverage(bool enabled, const std::string& type, uint32_t window)
{
  uint32_t avg;
  if (!enabled) avg = GG_MAVG_NONE;
  else if (type == "arithmetic_mean") avg = GG_MAVG_ARITHMETIC_MEAN;
  else if (type == "median") avg = GG_MAVG_MEDIAN;
  else if (type == "geometric_mean") avg = GG_MAVG_GEOMETRIC_MEAN;   // rejected by gg_create
  else throw std::invalid_argument("Unsupported Average Type: " + type);
  if (window == 0 || window > 0xFFFF) throw std::invalid_argument("moving_avg_window_size");
  return window | (avg << 16);
}

// The configured queue model (cfg.queue_model_type) over a sequence of
// requests from its constructor state: computeQueueDelay per request.
class QueueModel {
 public:
  QueueModel(Backend& be, uint64_t min_processing_time) : _be(be), _min(min_processing_time) {}
  std::vector<uint64_t> computeQueueDelays(const std::vector<uint64_t>& pkt_time, const std::vector<uint64_t>& proc_time)
  {
    if (pkt_time.size() != proc_time.size()) throw std::invalid_argument("computeQueueDelays: size mismatch");
    std::vector<uint64_t> d(pkt_time.size());
    check(gg_queue_delay_batch(_be.ctx(), _min, pkt_time.data(), proc_time.data(), pkt_time.size(), d.data()),
          "gg_queue_delay_batch");
    return d;
  }
 private:
  Backend& _be;
  uint64_t _min;
};

class NetworkModel {
 public:
  explicit NetworkModel(Backend& be) : _be(be) {}
  // Routes every packet of the batch to its receiver (all hops, in the
  // canonical order of DESIGN.md §NoC) and returns one RECEIVE_TILE hop per
  // packet (per tile for a broadcast: the application tiles, then the system
  // tiles), after the receiver's serialization delay.
  void routePackets(const std::vector<NetPacket>& pkts, std::vector<Hop>& hops, hipStream_t stream = nullptr)
  {
    const gg_config& cfg = _be.config();
    const size_t T = cfg.num_tiles, TT = cfg.total_tiles ? cfg.total_tiles : cfg.num_tiles + 2;
    const bool any_bcast = std::any_of(pkts.begin(), pkts.end(), [](const NetPacket& p) { return p.receiver == GG_BROADCAST; });
    if (any_bcast && cfg.net_model != GG_NET_EMESH_HOP_BY_HOP) {
      // no broadcast capability: Network::netSend sends one packet per tile
      // (network.cc:187-195); a receiver that is a system tile (MCP, thread
      // spawners) gets a zero-latency hop (processCornerCases, network_model.cc:440-443)
      std::vector<NetPacket> ex;
      for (const NetPacket& p : pkts) {
        if (p.receiver != GG_BROADCAST) { ex.push_back(p); continue; }
        for (size_t c = 0; c < T; ++c) { NetPacket q = p; q.receiver = (uint32_t)c; ex.push_back(q); }
      }
      std::vector<Hop> h;
      routePackets(ex, h, stream);
      hops.clear();
      size_t i = 0;
      for (const NetPacket& p : pkts) {
        if (p.receiver != GG_BROADCAST) { hops.push_back(h[i++]); continue; }
        for (size_t c = 0; c < T; ++c) hops.push_back(h[i++]);
        for (size_t c = T; c < TT; ++c) hops.push_back(Hop{(uint32_t)c, RECEIVE_TILE, p.time_ps, 0, 0});
      }
      return;
    }
    const size_t n = pkts.size();
    std::vector<uint32_t> src(n), dst(n), len(n);
    std::vector<uint64_t> t(n), arr(n), zl(n), ct(n);
    for (size_t k = 0; k < n; ++k) {
      src[k] = pkts[k].sender; dst[k] = pkts[k].receiver;
      len[k] = pkts[k].modeled_length_bits; t[k] = pkts[k].time_ps;
    }
    _s.resize(n); _d.resize(n); _l.resize(n); _t.resize(n); _a.resize(n); _z.resize(n); _c.resize(n);
    if (n) {
      hip_check(hipMemcpyAsync(_s.p, src.data(), 4 * n, hipMemcpyHostToDevice, stream), "copy");
      hip_check(hipMemcpyAsync(_d.p, dst.data(), 4 * n, hipMemcpyHostToDevice, stream), "copy");
      hip_check(hipMemcpyAsync(_l.p, len.data(), 4 * n, hipMemcpyHostToDevice, stream), "copy");
      hip_check(hipMemcpyAsync(_t.p, t.data(), 8 * n, hipMemcpyHostToDevice, stream), "copy");
    }
    gg_packets pk{_s.p, _d.p, _l.p, _t.p, n};
    gg_packet_out out{_a.p, _z.p, _c.p};
    // broadcasts (receiver NetPacket::BROADCAST): the hop-by-hop broadcast tree,
    // one RECEIVE_TILE hop per tile (network_model_emesh_hop_by_hop.cc:163-221)
    const size_t nb = (size_t)std::count(dst.begin(), dst.end(), GG_BROADCAST);
    std::vector<uint64_t> barr(nb * T), bzl(nb * T), bct(nb * T);
    if (nb) {
      _ba.resize(nb * T); _bz.resize(nb * T); _bc.resize(nb * T);
      gg_packet_out bout{_ba.p, _bz.p, _bc.p};
      check(gg_noc_route_tree(_be.ctx(), &pk, &out, &bout, nb, stream), "gg_noc_route_tree");
      hip_check(hipMemcpyAsync(barr.data(), _ba.p, 8 * nb * T, hipMemcpyDeviceToHost, stream), "copy");
      hip_check(hipMemcpyAsync(bzl.data(), _bz.p, 8 * nb * T, hipMemcpyDeviceToHost, stream), "copy");
      hip_check(hipMemcpyAsync(bct.data(), _bc.p, 8 * nb * T, hipMemcpyDeviceToHost, stream), "copy");
    } else {
      check(gg_noc_route_batch(_be.ctx(), &pk, &out, stream), "gg_noc_route_batch");
    }
    if (n) {
      hip_check(hipMemcpyAsync(arr.data(), _a.p, 8 * n, hipMemcpyDeviceToHost, stream), "copy");
      hip_check(hipMemcpyAsync(zl.data(), _z.p, 8 * n, hipMemcpyDeviceToHost, stream), "copy");
      hip_check(hipMemcpyAsync(ct.data(), _c.p, 8 * n, hipMemcpyDeviceToHost, stream), "copy");
    }
    hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    hops.clear();
    hops.reserve(n + nb * (T ? T - 1 : 0));
    size_t b = 0;
    for (size_t k = 0; k < n; ++k) {
      if (dst[k] != GG_BROADCAST) { hops.push_back(Hop{dst[k], RECEIVE_TILE, arr[k], zl[k], ct[k]}); continue; }
      for (size_t c = 0; c < T; ++c) {
        const size_t o = b * T + c;
        hops.push_back(Hop{(uint32_t)c, RECEIVE_TILE, barr[o], bzl[o], bct[o]});
      }
      // the system tiles: zero-latency hops pushed by processCornerCases (network_model.cc:451-458)
      for (size_t c = T; c < TT; ++c) hops.push_back(Hop{(uint32_t)c, RECEIVE_TILE, t[k], 0, 0});
      ++b;
    }
  }
  // The single-packet form of the reference: pushes the packet's delivery hop
  // (a broadcast: one per tile, in tile order).
  void routePacket(const NetPacket& pkt, std::queue<Hop>& next_hops)
  {
    std::vector<Hop> h;
    routePackets(std::vector<NetPacket>(1, pkt), h);
    for (const Hop& x : h) next_hops.push(x);
  }
 private:
  Backend& _be;
  DeviceBuffer<uint32_t> _s, _d, _l;
  DeviceBuffer<uint64_t> _t, _a, _z, _c, _ba, _bz, _bc;
};

}  // namespace graphite_amd
