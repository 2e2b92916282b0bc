// coh_harness.cc — the REFERENCE's own MSI protocol controllers, compiled from
// the sources where they lie under /root/reference (oracle/ref/Makefile),
// driven in the canonical coherent schedule of DESIGN.md §Mode C, writing the
// golden fixtures tests/golden/coh_*.  TEST INFRASTRUCTURE ONLY: never shipped,
// never linked into graphite_amd/.
//
// Reference code exercised verbatim, its own assert() calls active (only
// log.h's LOG_* are compiled out: the logging back end needs Boost, absent
// from this image; oracle/ref/assert_prelude.h):
//   L1CacheCntlr          pr_l1_pr_l2_dram_directory_msi/l1_cache_cntlr.cc
//   L2CacheCntlr          pr_l1_pr_l2_dram_directory_msi/l2_cache_cntlr.cc
//   DramDirectoryCntlr    pr_l1_pr_l2_dram_directory_msi/dram_directory_cntlr.cc
//   ShmemMsg / ShmemReq   pr_l1_pr_l2_dram_directory_msi/shmem_msg.cc, shmem_req.cc
//   PrL1/PrL2CacheLineInfo, CacheSet, LRU / round-robin policies, CacheState
//   DirectoryEntry(FullMap), BitVector, AddressHomeLookup, CachePerfModel(Parallel)
//   IntervalTree + QueueModelMG1 (under the DRAM queue, ref_htree.h)
//
// Glue restated here, statement by statement with the file:line it follows,
// because its reference translation units include Boost (config.hpp) or
// McPAT/DSENT headers the image lacks: Cache (cache.cc), DirectoryCache
// (directory_cache.cc), Directory (directory.cc), DramCntlr + DramPerfModel
// (dram_cntlr.cc, dram_perf_model.cc), ShmemPerfModel (shmem_perf_model.cc),
// the MemoryManager plumbing (memory_manager.cc, …msi/memory_manager.cc), Tile,
// Config/DVFSManager lookups (single 1 GHz domain: synchronization delays 0,
// dvfs_manager.cc:497-500) and the emesh_hop_counter / magic latency
// (network_model_emesh_hop_counter.cc:143-157, network_model.cc:142-150).
// The schedule (steps, inbox order, quanta) is the canonical one; app threads
// are ucontext coroutines so processMemOpFromCore can block in
// waitForSimThread exactly where the reference does.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <stdint.h>
#include <string>
#include <vector>
#include <map>
#include <algorithm>
#include <ucontext.h>

#include "tile.h"
#include "config.h"
#include "dvfs_manager.h"
#include "shmem_perf_model.h"
#include "cache.h"
#include "cache_set.h"
#include "cache_hash_fn.h"
#include "cache_line_info.h"
#include "cache_replacement_policy.h"
#include "directory_cache.h"
#include "directory.h"
#include "directory_entry.h"
#include "directory_entry_limitless.h"
#include "network.h"
#ifdef GG_PROTO_MOSI
// pr_l1_pr_l2_dram_directory_mosi (coh_harness_mosi): the protocol's event
// counters are private members of DramDirectoryCntlr / L2CacheCntlr; the
// harness reads them after the run (access widened for this translation unit
// only: the reference objects are compiled as they are)
#include <fstream>
#include <iostream>
#include <sstream>
#define private public
#define protected public
#include "pr_l1_pr_l2_dram_directory_mosi/memory_manager.h"
#undef private
#undef protected
#elif defined(GG_PROTO_SHL2) && defined(GG_SHL2_MESI)
// pr_l1_sh_l2_mesi (coh_harness_shl2_mesi): the shared-L2 organisation with
// EXCLUSIVE lines (SH_REP_EX, DOWNGRADE_REQ / _REP); the same glue as MSI's
#include "pr_l1_sh_l2_mesi/memory_manager.h"
#include "pr_l1_sh_l2_mesi/l2_cache_hash_fn.h"
#include "pr_l1_sh_l2_mesi/l2_directory_cfg.h"
#elif defined(GG_PROTO_SHL2)
// pr_l1_sh_l2_msi (coh_harness_shl2): private L1s, the L2 a shared slice per
// tile holding each line's directory entry, a DRAM controller per tile
#include "pr_l1_sh_l2_msi/memory_manager.h"
#include "pr_l1_sh_l2_msi/l2_cache_hash_fn.h"
#include "pr_l1_sh_l2_msi/l2_directory_cfg.h"
#else
#include "pr_l1_pr_l2_dram_directory_msi/memory_manager.h"
#endif
#include "ref_htree.h"

using namespace std;
#ifdef GG_PROTO_MOSI
namespace MSI = PrL1PrL2DramDirectoryMOSI;     // (the glue below is written once for both protocols)
// DirectoryEntryFullMap::getOneSharer draws from a drand48 stream the entry
// seeds with time(NULL) (misc/random.h:14-18): the canonical schedule fixes
// that seed (GG_MOSI_RNG_SEED, include/graphite_gpu.h), so every entry starts
// from the same drand48 state, as entries created in the same second do
extern "C" time_t time(time_t* t) { if (t) *t = (time_t)1; return (time_t)1; }
#elif defined(GG_PROTO_SHL2) && defined(GG_SHL2_MESI)
namespace MSI = PrL1ShL2MESI;
#elif defined(GG_PROTO_SHL2)
namespace MSI = PrL1ShL2MSI;
#else
namespace MSI = PrL1PrL2DramDirectoryMSI;
#endif

// message types in the backend's numbering (GG_MSG_*, include/graphite_gpu.h):
// the MSI enum is that numbering; MOSI's inserts INV_FLUSH_COMBINED_REQ after WB_REQ
static UInt32 gg_type(UInt32 t)
{
#ifdef GG_PROTO_MOSI
  switch (t) {
  case MSI::ShmemMsg::EX_REQ: return 1; case MSI::ShmemMsg::SH_REQ: return 2; case MSI::ShmemMsg::INV_REQ: return 3;
  case MSI::ShmemMsg::FLUSH_REQ: return 4; case MSI::ShmemMsg::WB_REQ: return 5; case MSI::ShmemMsg::EX_REP: return 6;
  case MSI::ShmemMsg::SH_REP: return 7; case MSI::ShmemMsg::UPGRADE_REP: return 8; case MSI::ShmemMsg::INV_REP: return 9;
  case MSI::ShmemMsg::FLUSH_REP: return 10; case MSI::ShmemMsg::WB_REP: return 11; case MSI::ShmemMsg::NULLIFY_REQ: return 12;
  case MSI::ShmemMsg::INV_FLUSH_COMBINED_REQ: return 13;
  default: CHECK(0); return 0;
  }
#elif defined(GG_PROTO_SHL2) && defined(GG_SHL2_MESI)
  // MESI inserts DOWNGRADE_REQ, SH_REP_EX and DOWNGRADE_REP: they follow the DRAM messages here
  switch (t) {
  case MSI::ShmemMsg::EX_REQ: return 1; case MSI::ShmemMsg::SH_REQ: return 2; case MSI::ShmemMsg::INV_REQ: return 3;
  case MSI::ShmemMsg::FLUSH_REQ: return 4; case MSI::ShmemMsg::WB_REQ: return 5; case MSI::ShmemMsg::EX_REP: return 6;
  case MSI::ShmemMsg::SH_REP: return 7; case MSI::ShmemMsg::UPGRADE_REP: return 8; case MSI::ShmemMsg::INV_REP: return 9;
  case MSI::ShmemMsg::FLUSH_REP: return 10; case MSI::ShmemMsg::WB_REP: return 11; case MSI::ShmemMsg::NULLIFY_REQ: return 12;
  case MSI::ShmemMsg::DRAM_FETCH_REQ: return 14; case MSI::ShmemMsg::DRAM_STORE_REQ: return 15;
  case MSI::ShmemMsg::DRAM_FETCH_REP: return 16; case MSI::ShmemMsg::DOWNGRADE_REQ: return 17;
  case MSI::ShmemMsg::SH_REP_EX: return 18; case MSI::ShmemMsg::DOWNGRADE_REP: return 19;
  default: CHECK(0); return 0;
  }
#elif defined(GG_PROTO_SHL2)
  // EX_REQ .. WB_REP share the numbering; the DRAM messages follow the MOSI type
  switch (t) {
  case MSI::ShmemMsg::DRAM_FETCH_REQ: return 14; case MSI::ShmemMsg::DRAM_STORE_REQ: return 15;
  case MSI::ShmemMsg::DRAM_FETCH_REP: return 16; case MSI::ShmemMsg::NULLIFY_REQ: return 12;
  default: CHECK(t >= 1 && t <= 11); return t;
  }
#else
  return t;
#endif
}

// ===========================================================================
// harness configuration and per-tile harness state
// ===========================================================================
struct HCfg {
  UInt32 T, K, net;           // tiles, logical shards, 0 magic / 1 hop counter
  UInt32 dir_entries;         // 0 = auto
  UInt32 dir_assoc;
  UInt64 quantum_ps;
  UInt32 l2_assoc;            // l2_cache/T1/associativity (carbon_sim.cfg:233: 8; configs[4]: 16)
  UInt32 workload;            // 0 hotspot (configs[2..3]), 1 stress (configs[4])
};
static HCfg H;

enum { NC_PS = 0, NC_PR, NC_LAT, NC_N };        // packets sent, received, total latency (ps)
enum { S_CLOCK = 0, S_ACC, S_L1H, S_L2H, S_MISS, S_LAT, S_DACC, S_DEV, S_DBI, S_DRAM, S_DRAMLAT, S_DRAMQD,
       S_DRAMQR, S_DRAMQA, S_SENT, S_RECV, S_BYTYPE, S_DRAMQU = S_BYTYPE + 11, S_DRAMQL, S_SENT_IFC = 29, S_N = 32 };

struct HMsg {
  UInt32 src, dst, seq, type;
  UInt64 send, arrival;
  vector<Byte> buf;           // ShmemMsg::makeMsgBuf()
};

struct HTile {
  Tile* tile;
  MSI::MemoryManager* mm;
  UInt64 rec, rec_end, clk;
  bool blocked, resumed_by_handler;
  UInt64 pend_start;
  UInt32 seq;
  vector<HMsg> inbox;
  UInt64 st[S_N];
  UInt64 net[NC_N];
  ucontext_t app_ctx;
  ucontext_t* ret_ctx;
  vector<char> stack;
};
static vector<HTile> g_t;
static vector<HMsg> g_step, g_bnd;
static const UInt64* g_addr; static const UInt32* g_meta; static UInt64* g_out;
static UInt64 g_barrier;
static UInt32 g_cur;          // tile whose code is running

// Logical shards = the process -> tile mapping NetworkModelEMeshHopByHop::
// computeProcessToTileMapping gives K processes (network_model_emesh_hop_by_hop.cc:
// 367-433; its translation unit pulls DSENT / Berkeley-DB headers through
// router_model.h, so it is restated here): 2-D blocks of the W x H mesh, or
// contiguous tile ranges when the tile count is not a full mesh.
static vector<UInt32> g_shard;
static void build_shard_map()
{
  const SInt32 T = (SInt32)H.T, K = (SInt32)H.K;
  g_shard.assign(T, 0);
  const SInt32 W = (SInt32)floor(sqrt(T)), Hh = (SInt32)ceil(1.0 * T / W);
  if (W * Hh != T) { for (SInt32 t = 0; t < T; ++t) g_shard[t] = (UInt32)(((UInt64)t * K) / T); return; }
  const SInt32 pw = (SInt32)floor(sqrt(K)), ph = (SInt32)floor(1.0 * K / pw);
  const SInt32 hl = (SInt32)((1.0 * Hh * pw * ph) / K);
  for (SInt32 i = 0; i < pw; i++)
    for (SInt32 j = 0; j < ph; j++) {
      SInt32 sx = W / pw, sy = hl / ph;
      const SInt32 bx = i * sx, by = j * sy;
      if (i == pw - 1) sx = W - (pw - 1) * sx;
      if (j == ph - 1) sy = hl - (ph - 1) * sy;
      for (SInt32 ii = 0; ii < sx; ii++)
        for (SInt32 jj = 0; jj < sy; jj++) g_shard[(bx + ii) + (by + jj) * W] = (UInt32)(i + j * pw);
    }
  const SInt32 left = K - pw * ph;
  for (SInt32 i = pw * ph; i < K; i++) {
    SInt32 sx = W / left;
    const SInt32 sy = Hh - hl, bx = (i - pw * ph) * sx, by = hl;
    if (i == K - 1) sx = W - (left - 1) * sx;
    for (SInt32 ii = 0; ii < sx; ii++)
      for (SInt32 jj = 0; jj < sy; jj++) g_shard[(bx + ii) + (by + jj) * W] = (UInt32)i;
  }
}
static UInt32 shard_of(UInt32 t) { return g_shard[t]; }
static int tile_of(MemoryManager* mm) { return mm->getTile()->getId(); }

// ===========================================================================
// Config / DVFSManager lookups (misc/config.cc, system/dvfs_manager.cc)
// ===========================================================================
static double g_config_storage[64];
Config* Config::getSingleton() { return (Config*)g_config_storage; }
bool Config::isApplicationTile(tile_id_t t) { return t >= 0 && t < (tile_id_t)H.T; }   // config.cc
UInt32 Config::getTotalTiles() { return H.T + 2; }           // app + MCP + 1 process (config.cc:77-82)
UInt32 Config::getApplicationTiles() { return H.T; }
UInt32 DVFSManager::getSynchronizationDelay() { return 0; }  // one DVFS domain (dvfs_manager.cc:497-500)
module_t DVFSManager::convertToModule(MemComponent::Type c)   // dvfs_manager.cc:503-518
{
  switch (c) {
  case MemComponent::L1_ICACHE: return L1_ICACHE;
  case MemComponent::L1_DCACHE: return L1_DCACHE;
  case MemComponent::L2_CACHE: return L2_CACHE;
  case MemComponent::DRAM_DIRECTORY: return DIRECTORY;
  default: return INVALID_MODULE;
  }
}
// pr_l1_*_cache_line_info.cc of the other protocols are compiled; Limitless needs config.hpp
// (only full_map directories are built here: the limitless entry points trap)
DirectoryEntryLimitless::DirectoryEntryLimitless(SInt32 a, SInt32 b) : DirectoryEntryLimited(a) { (void)b; CHECK(0); }
DirectoryEntryLimitless::~DirectoryEntryLimitless() {}
bool DirectoryEntryLimitless::hasSharer(tile_id_t) { CHECK(0); return false; }
bool DirectoryEntryLimitless::addSharer(tile_id_t) { CHECK(0); return false; }
void DirectoryEntryLimitless::removeSharer(tile_id_t, bool) { CHECK(0); }
bool DirectoryEntryLimitless::getSharersList(vector<tile_id_t>&) { CHECK(0); return false; }
SInt32 DirectoryEntryLimitless::getNumSharers() { CHECK(0); return 0; }
UInt32 DirectoryEntryLimitless::getLatency() { CHECK(0); return 0; }

// ===========================================================================
// ShmemPerfModel (performance_models/shmem_perf_model.cc:7-45)
// ===========================================================================
ShmemPerfModel::ShmemPerfModel() : _curr_time(0), _enabled(false) {}
ShmemPerfModel::~ShmemPerfModel() {}
void ShmemPerfModel::setCurrTime(const Time& t) { _curr_time = t; }
Time ShmemPerfModel::getCurrTime() { return _curr_time; }
void ShmemPerfModel::updateCurrTime(const Time& t) { if (_curr_time < t) _curr_time = t; }
void ShmemPerfModel::incrCurrTime(const Time& t) { if (_enabled) _curr_time += t; }

// ===========================================================================
// Cache (cache/cache.cc) — counters kept beside the object
// ===========================================================================
enum { CC_ACC = 0, CC_MISS, CC_RACC, CC_RMISS, CC_WACC, CC_WMISS, CC_EV, CC_DEV, CC_TR, CC_TW, CC_DR, CC_DW, CC_N };
static map<const Cache*, vector<UInt64> > g_cc;
static UInt64* ccount(const Cache* c) { vector<UInt64>& v = g_cc[c]; if (v.empty()) v.resize(CC_N, 0); return &v[0]; }

Cache::Cache(string name, CachingProtocolType cpt, CacheCategory cat, SInt32 level, WritePolicy wp, UInt32 size,
             UInt32 assoc, UInt32 line, UInt32 banks, CacheReplacementPolicy* rp, CacheHashFn* hf, UInt32 data_lat,
             UInt32 tags_lat, string perf_model_type, bool track, ShmemPerfModel* spm)
  : _enabled(false), _name(name), _cache_category(cat), _write_policy(wp), _cache_size(k_KILO * size),
    _associativity(assoc), _line_size(line), _num_banks(banks), _replacement_policy(rp), _hash_fn(hf),
    _track_miss_types(track), _mcpat_cache_interface(NULL)            // cache.cc:15-42
{
  (void)spm;
  _num_sets = _cache_size / (_associativity * _line_size);            // :44
  _log_line_size = floorLog2(_line_size);
  _sets = new CacheSet*[_num_sets];
  for (UInt32 i = 0; i < _num_sets; i++) _sets[i] = new CacheSet(i, cpt, level, _replacement_policy, _associativity, _line_size);
  _frequency = 1.0; _voltage = 1.0;                                    // initializeDVFS: the 1 GHz domain
  _perf_model = CachePerfModel::create(perf_model_type, data_lat, tags_lat, _frequency);
  ccount(this);
}
Cache::~Cache() { for (UInt32 i = 0; i < _num_sets; i++) delete _sets[i]; delete[] _sets; delete _perf_model; }
IntPtr Cache::getTag(IntPtr a) const { return a >> _log_line_size; }                       // :495-498
CacheSet* Cache::getSet(IntPtr a) const { return _sets[_hash_fn->compute(a)]; }            // :500-505
UInt32 Cache::getLineOffset(IntPtr a) const { return a & (_line_size - 1); }               // :507-511
IntPtr Cache::getAddressFromTag(IntPtr tag) const { return tag << _log_line_size; }        // :513-517
Time Cache::getSynchronizationDelay(module_t) { return Time(0); }

void Cache::accessCacheLine(IntPtr address, AccessType access_type, Byte* buf, UInt32 num_bytes)   // :84-112
{
  CacheSet* set = getSet(address);
  UInt32 line_index = -1;
  CacheLineInfo* li = set->find(getTag(address), &line_index);
  CHECK(li);
  if (access_type == LOAD) set->read_line(line_index, getLineOffset(address), buf, num_bytes);
  else set->write_line(line_index, getLineOffset(address), buf, num_bytes);
  if (_enabled) ccount(this)[access_type == LOAD ? CC_DR : CC_DW]++;
}
void Cache::insertCacheLine(IntPtr a, CacheLineInfo* in, Byte* fill, bool* ev, IntPtr* ev_addr, CacheLineInfo* ev_info,
                            Byte* wb)                                                          // :114-184
{
  CacheSet* set = getSet(a);
  set->insert(in, fill, ev, ev_info, wb);
  *ev_addr = getAddressFromTag(ev_info->getTag());
  if (_enabled) {
    UInt64* c = ccount(this);
    if (*ev) {
      CHECK(ev_info->getCState() != CacheState::INVALID);
      c[CC_TR]++; c[CC_DR]++; c[CC_EV]++;
      if (_write_policy == WRITE_BACK && CacheState(ev_info->getCState()).dirty()) c[CC_DEV]++;
    } else {
      c[CC_TR]++;
    }
    c[CC_TW]++; c[CC_DW]++;
  }
}
CacheLineInfo* Cache::getCacheLineInfo(IntPtr a) { return getSet(a)->find(getTag(a)); }     // :207-215
void Cache::getCacheLineInfo(IntPtr a, CacheLineInfo* out)                                  // :187-205
{
  CacheLineInfo* li = getCacheLineInfo(a);
  if (li) out->assign(li);
  if (_enabled) ccount(this)[CC_TR]++;
}
void Cache::setCacheLineInfo(IntPtr a, CacheLineInfo* in)                                   // :218-241
{
  CacheLineInfo* li = getCacheLineInfo(a);
  CHECK(li);
  li->assign(in);
  if (_enabled) ccount(this)[CC_TW]++;
}
Cache::MissType Cache::updateMissCounters(IntPtr, Core::mem_op_t op, bool miss)              // :321-360
{
  if (_enabled) {
    UInt64* c = ccount(this);
    c[CC_ACC]++;
    bool rd = (op == Core::READ) || (op == Core::READ_EX);
    c[rd ? CC_RACC : CC_WACC]++;
    if (miss) { c[CC_MISS]++; c[rd ? CC_RMISS : CC_WMISS]++; }
  }
  return INVALID_MISS_TYPE;
}

// ===========================================================================
// Directory (directory_schemes/directory.cc:6-45)
// ===========================================================================
Directory::Directory(CachingProtocolType cpt, DirectoryType dt, SInt32 total, SInt32 hw, SInt32 num)
  : _total_entries(total), _directory_type(dt)
{
  _directory_entry_list.resize(_total_entries);
  for (SInt32 i = 0; i < _total_entries; i++) _directory_entry_list[i] = DirectoryEntry::create(cpt, dt, hw, num);
}
Directory::~Directory() { for (SInt32 i = 0; i < _total_entries; i++) delete _directory_entry_list[i]; }
DirectoryEntry* Directory::getDirectoryEntry(SInt32 n) { return _directory_entry_list[n]; }
void Directory::setDirectoryEntry(SInt32 n, DirectoryEntry* e) { _directory_entry_list[n] = e; }
void Directory::updateSharerStats(SInt32, SInt32) {}

// ===========================================================================
// DirectoryCache (cache/directory_cache.cc) — counters kept beside the object
// ===========================================================================
enum { DC_ACC = 0, DC_EV, DC_BI, DC_N };
static map<const DirectoryCache*, vector<UInt64> > g_dc;
static UInt64* dcount(const DirectoryCache* d) { vector<UInt64>& v = g_dc[d]; if (v.empty()) v.resize(DC_N, 0); return &v[0]; }

DirectoryCache::DirectoryCache(Tile* tile, CachingProtocolType cpt, string dts, string tes, UInt32 assoc, UInt32 line,
                               UInt32 hw, UInt32 num, UInt32 slices, string acs, ShmemPerfModel* spm)   // :10-81
  : _tile(tile), _caching_protocol_type(cpt), _max_hw_sharers(hw), _max_num_sharers(num), _total_entries_str(tes),
    _associativity(assoc), _cache_line_size(line), _num_directory_slices(slices), _directory_access_cycles_str(acs),
    _mcpat_cache_interface(NULL), _enabled(false), _module(DIRECTORY), _shmem_perf_model(spm)
{
  _directory_type = DirectoryEntry::parseDirectoryType(dts);
  _total_entries = computeDirectoryTotalEntries();
  _num_sets = _total_entries / _associativity;
  _directory = new Directory(cpt, _directory_type, _total_entries, hw, num);
  UInt32 max_application_sharers = Config::getSingleton()->getApplicationTiles();
  UInt32 entry_size = ceil(1.0 * DirectoryEntry::getSize(_directory_type, hw, max_application_sharers) / 8);
  _directory_size = _total_entries * entry_size;
  _frequency = 1.0; _voltage = 1.0;
  _directory_access_cycles = computeDirectoryAccessCycles();
  _directory_access_latency = Time(Latency(_directory_access_cycles, _frequency));
  _synchronization_delay = Time(Latency(DVFSManager::getSynchronizationDelay(), _frequency));
  _log_num_sets = floorLog2(_num_sets);
  _log_cache_line_size = floorLog2(_cache_line_size);
  _log_num_directory_slices = ceilLog2(_num_directory_slices);
  dcount(this);
}
DirectoryCache::~DirectoryCache() { delete _directory; }
Time DirectoryCache::getSynchronizationDelay(module_t) { return Time(0); }
ShmemPerfModel* DirectoryCache::getShmemPerfModel() { return _tile->getMemoryManager()->getShmemPerfModel(); }
void DirectoryCache::updateCounters() { dcount(this)[DC_ACC]++; }                          // :92-95
UInt32 DirectoryCache::computeDirectoryTotalEntries()                                        // :243-268
{
  if (_total_entries_str == "auto") {
    UInt32 max_L2_cache_size = 512;                                    // l2_cache/T1/cache_size
    UInt32 num_sets = (UInt32)ceil(2.0 * max_L2_cache_size * 1024 * Config::getSingleton()->getApplicationTiles() /
                                   (_cache_line_size * _associativity * _num_directory_slices));
    num_sets = 1 << ceilLog2(num_sets);
    return num_sets * _associativity;
  }
  return (UInt32)atoi(_total_entries_str.c_str());
}
UInt64 DirectoryCache::computeDirectoryAccessCycles()                                        // :292-322
{
  if (_directory_access_cycles_str == "auto") {
    UInt32 kb = (UInt32)ceil(1.0 * _directory_size / 1024);
    if (kb <= 16) return 1; else if (kb <= 32) return 2; else if (kb <= 64) return 4; else if (kb <= 128) return 6;
    else if (kb <= 256) return 8; else if (kb <= 512) return 10; else if (kb <= 1024) return 13;
    else if (kb <= 2048) return 16; else return 20;
  }
  return (UInt64)atoll(_directory_access_cycles_str.c_str());
}
IntPtr DirectoryCache::computeSetIndex(IntPtr address)                                       // :332-348
{
  IntPtr set = 0;
  for (UInt32 i = _log_cache_line_size + _log_num_directory_slices; (i + _log_num_sets) <= (sizeof(IntPtr) * 8);
       i += _log_num_sets)
    set = set ^ getBits<IntPtr>(address, i + _log_num_sets, i);
  return (UInt32)set;
}
void DirectoryCache::splitAddress(IntPtr a, IntPtr& tag, UInt32& set_index)                  // :233-241
{
  tag = a >> _log_cache_line_size;
  set_index = computeSetIndex(a);
}
DirectoryEntry* DirectoryCache::getDirectoryEntry(IntPtr address)                            // :102-145
{
  if (_enabled) { getShmemPerfModel()->incrCurrTime(_directory_access_latency); updateCounters(); }
  IntPtr tag; UInt32 set_index;
  splitAddress(address, tag, set_index);
  for (UInt32 i = 0; i < _associativity; i++) {
    DirectoryEntry* e = _directory->getDirectoryEntry(set_index * _associativity + i);
    if (e->getAddress() == address) {
      if (getShmemPerfModel()) getShmemPerfModel()->incrCurrTime(Latency(e->getLatency(), _frequency));
      return e;
    }
  }
  for (UInt32 i = 0; i < _associativity; i++) {
    DirectoryEntry* e = _directory->getDirectoryEntry(set_index * _associativity + i);
    if (e->getAddress() == INVALID_ADDRESS) { e->setAddress(address); return e; }
  }
  for (vector<DirectoryEntry*>::iterator it = _replaced_directory_entry_list.begin();
       it != _replaced_directory_entry_list.end(); it++)
    if ((*it)->getAddress() == address) return *it;
  return NULL;
}
void DirectoryCache::getReplacementCandidates(IntPtr address, vector<DirectoryEntry*>& list)  // :147-161
{
  CHECK(getDirectoryEntry(address) == NULL);   // the reference build keeps this assert (no NDEBUG): one access
  IntPtr tag; UInt32 set_index;
  splitAddress(address, tag, set_index);
  for (UInt32 i = 0; i < _associativity; i++) list.push_back(_directory->getDirectoryEntry(set_index * _associativity + i));
}
DirectoryEntry* DirectoryCache::replaceDirectoryEntry(IntPtr replaced_address, IntPtr address)   // :163-213
{
  IntPtr tag; UInt32 set_index;
  splitAddress(replaced_address, tag, set_index);
  DirectoryEntry* replaced = NULL;
  DirectoryEntry* ne = DirectoryEntry::create(_caching_protocol_type, _directory_type, _max_hw_sharers, _max_num_sharers);
  ne->setAddress(address);
  for (UInt32 i = 0; i < _associativity; i++) {
    DirectoryEntry* e = _directory->getDirectoryEntry(set_index * _associativity + i);
    if (e->getAddress() == replaced_address) {
      replaced = e;
      _directory->setDirectoryEntry(set_index * _associativity + i, ne);
      break;
    }
  }
  CHECK(replaced);
  _replaced_directory_entry_list.push_back(replaced);
  if (_enabled) {
    getShmemPerfModel()->incrCurrTime(_directory_access_latency);
    updateCounters();
    dcount(this)[DC_EV]++;
    if (replaced->getDirectoryBlockInfo()->getDState() != DirectoryState::UNCACHED) dcount(this)[DC_BI]++;
  }
  return ne;
}
void DirectoryCache::invalidateDirectoryEntry(IntPtr address)                                 // :215-231
{
  for (vector<DirectoryEntry*>::iterator it = _replaced_directory_entry_list.begin();
       it != _replaced_directory_entry_list.end(); it++) {
    if ((*it)->getAddress() == address) { delete (*it); _replaced_directory_entry_list.erase(it); return; }
  }
  CHECK(0);
}

// ===========================================================================
// DramCntlr + DramPerfModel (dram_cntlr.cc:37-74, dram_perf_model.cc:20-116)
// ===========================================================================
struct HDram { RefHistoryTree* q; bool enabled; UInt64 n, lat, qd, qreq; };
static map<const DramCntlr*, HDram> g_dram;
DramCntlr::DramCntlr(Tile* tile, float cost, float bw, bool qm, string qtype, UInt32 line)
  : _tile(tile), _dram_perf_model(NULL), _dram_access_count(NULL), _cache_line_size(line)
{
  CHECK(qtype == "history_tree");
  HDram d;
  UInt64 min_proc = (UInt64)((float)line / bw) + 1;                   // dram_perf_model.cc:48
  d.q = qm ? new RefHistoryTree(min_proc, 100, true) : NULL;          // queue_model/history_tree defaults
  d.enabled = false; d.n = d.lat = d.qd = d.qreq = 0;
  g_dram[this] = d;
  (void)cost;
}
DramCntlr::~DramCntlr() {}
ShmemPerfModel* DramCntlr::getShmemPerfModel() { return _tile->getMemoryManager()->getShmemPerfModel(); }
static UInt64 g_dram_cost = 100; static float g_dram_bw = 5.0f;
Latency DramCntlr::runDramPerfModel()                                  // dram_cntlr.cc:66-71 + getAccessLatency
{
  HDram& d = g_dram[this];
  Time pkt_time = getShmemPerfModel()->getCurrTime();
  UInt64 pkt_time_ns = (UInt64)ceil(pkt_time.getTime() / 1000.0);
  if (!d.enabled) return Latency(0, DRAM_FREQUENCY);
  UInt64 processing_time = (UInt64)((float)_cache_line_size / g_dram_bw) + 1;
  UInt64 queue_delay = 0;
  if (d.q) { queue_delay = d.q->delay(pkt_time_ns, processing_time); d.qreq++; }
  UInt64 access_latency = queue_delay + processing_time + (UInt64)(float)g_dram_cost;
  d.n++; d.lat += access_latency; d.qd += queue_delay;
  return Latency(access_latency, DRAM_FREQUENCY);
}
void DramCntlr::getDataFromDram(IntPtr address, Byte* data_buf, bool modeled)   // :37-55
{
  if (_data_map[address] == NULL) { _data_map[address] = new Byte[_cache_line_size]; memset(_data_map[address], 0, _cache_line_size); }
  memcpy(data_buf, _data_map[address], _cache_line_size);
  Latency l = modeled ? runDramPerfModel() : Latency(0, DRAM_FREQUENCY);
  getShmemPerfModel()->incrCurrTime(l);
}
void DramCntlr::putDataToDram(IntPtr address, Byte* data_buf, bool modeled)     // :57-64
{
  CHECK(_data_map[address] != NULL);
  memcpy(_data_map[address], data_buf, _cache_line_size);
  if (modeled) (void)runDramPerfModel();
}

// ===========================================================================
// NetPacket (network/network.cc:645-656)
// ===========================================================================
NetPacket::NetPacket() : time(0), type(INVALID_PACKET_TYPE), sender(INVALID_CORE_ID), receiver(INVALID_CORE_ID),
  node_type(0 /* NetworkModel::SEND_TILE, network_model.h */), length(0), data(0), zero_load_delay(0), contention_delay(0) {}

// ===========================================================================
// MemoryManager (memory_manager.cc) and the MSI MemoryManager (…msi/memory_manager.cc)
// ===========================================================================
#ifdef GG_PROTO_MOSI
CachingProtocolType MemoryManager::_caching_protocol_type = PR_L1_PR_L2_DRAM_DIRECTORY_MOSI;
ofstream MSI::MemoryManager::_cache_line_replication_file;
#elif defined(GG_PROTO_SHL2) && defined(GG_SHL2_MESI)
CachingProtocolType MemoryManager::_caching_protocol_type = PR_L1_SH_L2_MESI;
#elif defined(GG_PROTO_SHL2)
CachingProtocolType MemoryManager::_caching_protocol_type = PR_L1_SH_L2_MSI;
#else
CachingProtocolType MemoryManager::_caching_protocol_type = PR_L1_PR_L2_DRAM_DIRECTORY_MSI;
#endif
MemoryManager::MemoryManager(Tile* tile) : _tile(tile), _network(NULL), _enabled(false)
{
  _shmem_perf_model = new ShmemPerfModel();
}
MemoryManager::~MemoryManager() { delete _shmem_perf_model; }
void MemoryManager::enableModels() { _enabled = true; _shmem_perf_model->enable(); }
void MemoryManager::disableModels() { _enabled = false; _shmem_perf_model->disable(); }
void MemoryManager::outputSummary(std::ostream&, const Time&) {}
// memory_manager.cc:78-99 (the per-tile lock is implicit: one coroutine runs at a time)
bool MemoryManager::__coreInitiateMemoryAccess(MemComponent::Type mc, Core::lock_signal_t ls, Core::mem_op_t op,
                                               IntPtr address, UInt32 offset, Byte* buf, UInt32 len, Time& curr_time,
                                               bool modeled)
{
  _shmem_perf_model->setCurrTime(curr_time);
  bool ret = coreInitiateMemoryAccess(mc, ls, op, address, offset, buf, len, modeled);
  curr_time = _shmem_perf_model->getCurrTime();
  return ret;
}
// memory_manager.cc:102-120
void MemoryManager::__handleMsgFromNetwork(NetPacket& packet)
{
  _shmem_perf_model->setCurrTime(packet.time);
  handleMsgFromNetwork(packet);
}

// APP / SIM thread hand-over (memory_manager.cc:128-151) as coroutine switches
static void app_yield(HTile& T) { ucontext_t* r = T.ret_ctx; swapcontext(&T.app_ctx, r); }
void MemoryManager::waitForSimThread()       // the app blocks until its reply has been handled
{
  HTile& T = g_t[tile_of(this)];
  T.blocked = true;
  app_yield(T);
}
void MemoryManager::wakeUpAppThread()        // the reply handler hands control to the app ...
{
  HTile& T = g_t[tile_of(this)];
  ucontext_t here;
  T.ret_ctx = &here;
  T.resumed_by_handler = true;
  swapcontext(&here, &T.app_ctx);
}
void MemoryManager::waitForAppThread() {}    // ... which returns once its access has completed
void MemoryManager::wakeUpSimThread() {}

#ifdef GG_PROTO_SHL2
// carbon_sim.cfg defaults (l1_icache/T1 :208-217, l1_dcache/T1 :219-228,
// l2_cache/T1 :230-239, l2_directory :260-263, dram :265-273); the
// constructor body follows …sh_l2_msi/memory_manager.cc:116-185 (the config
// reads are Boost's, so the values are given here)
MSI::MemoryManager::MemoryManager(Tile* tile) : ::MemoryManager(tile), _dram_cntlr(NULL), _dram_cntlr_present(false)
{
  _cache_line_size = 64;
  vector<tile_id_t> ctrl;
  for (UInt32 i = 0; i < H.T; ++i) ctrl.push_back(i);
  _dram_home_lookup = new AddressHomeLookup(ceilLog2(64), ctrl, 64);
  _L2_cache_home_lookup = new AddressHomeLookup(ceilLog2(64), ctrl, 64);
  _dram_cntlr_present = true;
  _dram_cntlr = new DramCntlr(this, (float)g_dram_cost, g_dram_bw, true, "history_tree", 64);
  L2DirectoryCfg::setDirectoryType(DirectoryEntry::parseDirectoryType("full_map"));
  L2DirectoryCfg::setMaxHWSharers(64);
  L2DirectoryCfg::setMaxNumSharers(Config::getSingleton()->getTotalTiles());
  _L1_cache_cntlr = new L1CacheCntlr(this, _L2_cache_home_lookup, 64, 16, 4, 1, "lru", 1, 1, "parallel", false,
                                     32, 4, 1, "lru", 1, 1, "parallel", false);
  _L2_cache_cntlr = new L2CacheCntlr(this, _dram_home_lookup, 64, 512, H.l2_assoc, 1, "lru", 8, 3, "parallel", false);
}
MSI::MemoryManager::~MemoryManager() {}
void MSI::MemoryManager::enableModels()                                    // …sh_l2_msi/memory_manager.cc:378-393
{
  getL1ICache()->enable(); getL1DCache()->enable(); getL2Cache()->enable();
  _L2_cache_cntlr->enable();
  g_dram[_dram_cntlr].enabled = true;
  ::MemoryManager::enableModels();
}
void MSI::MemoryManager::disableModels() { ::MemoryManager::disableModels(); }
void MSI::MemoryManager::outputSummary(std::ostream&, const Time&) {}
void MSI::MemoryManager::computeEnergy(const Time&) {}
double MSI::MemoryManager::getDynamicEnergy() { return 0; }
double MSI::MemoryManager::getLeakageEnergy() { return 0; }
int MSI::MemoryManager::getDVFS(module_t, double&, double&) { return -1; }
int MSI::MemoryManager::setDVFS(module_t, double, voltage_option_t, const Time&) { return -1; }
bool MSI::MemoryManager::coreInitiateMemoryAccess(MemComponent::Type mc, Core::lock_signal_t ls, Core::mem_op_t op,
                                                  IntPtr address, UInt32 offset, Byte* buf, UInt32 len, bool modeled)
{                                                                           // …sh_l2_msi/memory_manager.cc:202-213
  return _L1_cache_cntlr->processMemOpFromCore(mc, ls, op, address, offset, buf, len, modeled);
}
void MSI::MemoryManager::handleMsgFromNetwork(NetPacket& packet)           // …sh_l2_msi/memory_manager.cc:215-294
{
  core_id_t sender = packet.sender;
  ShmemMsg* shmem_msg = ShmemMsg::getShmemMsg((Byte*)packet.data);
  const MemComponent::Type snd = shmem_msg->getSenderMemComponent();
  switch (shmem_msg->getReceiverMemComponent()) {
  case MemComponent::L1_ICACHE:
  case MemComponent::L1_DCACHE:
    if (snd == MemComponent::CORE) { CHECK(sender.tile_id == getTile()->getId()); _L1_cache_cntlr->handleMsgFromCore(shmem_msg); }
    else { CHECK(snd == MemComponent::L2_CACHE); _L1_cache_cntlr->handleMsgFromL2Cache(sender.tile_id, shmem_msg); }
    break;
  case MemComponent::L2_CACHE:
    if (snd == MemComponent::L1_ICACHE || snd == MemComponent::L1_DCACHE) _L2_cache_cntlr->handleMsgFromL1Cache(sender.tile_id, shmem_msg);
    else { CHECK(snd == MemComponent::DRAM_CNTLR); _L2_cache_cntlr->handleMsgFromDram(sender.tile_id, shmem_msg); }
    break;
  case MemComponent::DRAM_CNTLR:
    CHECK(_dram_cntlr_present && snd == MemComponent::L2_CACHE);
    _dram_cntlr->handleMsgFromL2Cache(sender.tile_id, shmem_msg);
    break;
  default: CHECK(0);
  }
  if (shmem_msg->getDataLength() > 0) delete[] shmem_msg->getDataBuf();
  delete shmem_msg;
}
// L2CacheHashFn (…sh_l2_msi/l2_cache_hash_fn.cc: its translation unit includes
// simulator.h, which needs Boost): the XOR fold of the address' set-index fields
MSI::L2CacheHashFn::L2CacheHashFn(UInt32 cache_size, UInt32 associativity, UInt32 cache_line_size)
  : CacheHashFn(cache_size, associativity, cache_line_size)                  // :8-13
{
  _log_num_application_tiles = floorLog2(Config::getSingleton()->getApplicationTiles());
  _log_num_sets = floorLog2(_num_sets);
}
MSI::L2CacheHashFn::~L2CacheHashFn() {}
UInt32 MSI::L2CacheHashFn::compute(IntPtr address)                               // :18-34
{
  if (_log_num_sets == 0) return 0;
  IntPtr set = 0;
  for (UInt32 i = _log_cache_line_size; (i + _log_num_sets) <= (sizeof(IntPtr) * 8); i += _log_num_sets)
    set = set ^ getBits<IntPtr>(address, i + _log_num_sets, i);
  return (UInt32)set;
}
#else
MSI::MemoryManager::MemoryManager(Tile* tile) : ::MemoryManager(tile), _dram_directory_cntlr(NULL), _dram_cntlr(NULL),
                                                _dram_cntlr_present(false)
{
  // carbon_sim.cfg defaults (l1_icache/T1 :208-217, l1_dcache/T1 :219-228, l2_cache/T1 :230-239,
  // dram_directory :253-258, dram :265-273)
  _cache_line_size = 64;
  vector<tile_id_t> ctrl;
  for (UInt32 i = 0; i < H.T; ++i) ctrl.push_back(i);
  _dram_cntlr_present = true;
  _dram_cntlr = new DramCntlr(tile, (float)g_dram_cost, g_dram_bw, true, "history_tree", 64);
  char ent[32], acc[8] = "auto";
  if (H.dir_entries) snprintf(ent, sizeof(ent), "%u", H.dir_entries); else snprintf(ent, sizeof(ent), "auto");
#ifdef GG_PROTO_MOSI
  _dram_directory_cntlr = new DramDirectoryCntlr(this, _dram_cntlr, ent, H.dir_assoc, 64,
                                                 Config::getSingleton()->getTotalTiles(), 64, "full_map", H.T, acc);
#else
  _dram_directory_cntlr = new DramDirectoryCntlr(this, _dram_cntlr, ent, H.dir_assoc, 64,
                                                 Config::getSingleton()->getTotalTiles(), 64, "full_map", acc, H.T);
#endif
  _dram_directory_home_lookup = new AddressHomeLookup(ceilLog2(64), ctrl, 64);
  _L1_cache_cntlr = new L1CacheCntlr(this, 64, 16, 4, 1, "lru", 1, 1, "parallel", false,
                                     32, 4, 1, "lru", 1, 1, "parallel", false);
  _L2_cache_cntlr = new L2CacheCntlr(this, _L1_cache_cntlr, _dram_directory_home_lookup, 64, 512, H.l2_assoc, 1, "lru",
                                     8, 3, "parallel", false);
  _L1_cache_cntlr->setL2CacheCntlr(_L2_cache_cntlr);
}
MSI::MemoryManager::~MemoryManager() {}
void MSI::MemoryManager::enableModels()                                    // …msi/memory_manager.cc:382-396
{                                                                           // (…mosi/memory_manager.cc:373-390)
  getL1ICache()->enable(); getL1DCache()->enable(); getL2Cache()->enable();
#ifdef GG_PROTO_MOSI
  _L2_cache_cntlr->enable();
  _dram_directory_cntlr->enable();
#endif
  _dram_directory_cntlr->getDramDirectoryCache()->enable();
  g_dram[_dram_cntlr].enabled = true;
  ::MemoryManager::enableModels();
}
void MSI::MemoryManager::disableModels() { ::MemoryManager::disableModels(); }
void MSI::MemoryManager::outputSummary(std::ostream&, const Time&) {}
void MSI::MemoryManager::computeEnergy(const Time&) {}
double MSI::MemoryManager::getDynamicEnergy() { return 0; }
double MSI::MemoryManager::getLeakageEnergy() { return 0; }
int MSI::MemoryManager::getDVFS(module_t, double&, double&) { return -1; }
int MSI::MemoryManager::setDVFS(module_t, double, voltage_option_t, const Time&) { return -1; }
bool MSI::MemoryManager::coreInitiateMemoryAccess(MemComponent::Type mc, Core::lock_signal_t ls, Core::mem_op_t op,
                                                  IntPtr address, UInt32 offset, Byte* buf, UInt32 len, bool modeled)
{                                                                           // …msi/memory_manager.cc:224-235
  return _L1_cache_cntlr->processMemOpFromCore(mc, ls, op, address, offset, buf, len, modeled);
}
void MSI::MemoryManager::handleMsgFromNetwork(NetPacket& packet)           // …msi/memory_manager.cc:237-304
{
  core_id_t sender = packet.sender;
  ShmemMsg* shmem_msg = ShmemMsg::getShmemMsg((Byte*)packet.data);
  switch (shmem_msg->getReceiverMemComponent()) {
  case MemComponent::L2_CACHE:
    if (shmem_msg->getSenderMemComponent() == MemComponent::DRAM_DIRECTORY)
      _L2_cache_cntlr->handleMsgFromDramDirectory(sender.tile_id, shmem_msg);
    else { CHECK(sender.tile_id == getTile()->getId()); _L2_cache_cntlr->handleMsgFromL1Cache(shmem_msg); }
    break;
  case MemComponent::DRAM_DIRECTORY:
    CHECK(shmem_msg->getSenderMemComponent() == MemComponent::L2_CACHE);
    _dram_directory_cntlr->handleMsgFromL2Cache(sender.tile_id, shmem_msg);
    break;
  default: CHECK(0);
  }
  if (shmem_msg->getDataLength() > 0) delete[] shmem_msg->getDataBuf();
  delete shmem_msg;
}
#endif
// the MSI incrCurrTime (…msi/memory_manager.cc:356-380)
void MSI::MemoryManager::incrCurrTime(MemComponent::Type mc, CachePerfModel::AccessType at)
{
  switch (mc) {
  case MemComponent::L1_ICACHE: getShmemPerfModel()->incrCurrTime(_L1_cache_cntlr->getL1ICache()->getPerfModel()->getLatency(at)); break;
  case MemComponent::L1_DCACHE: getShmemPerfModel()->incrCurrTime(_L1_cache_cntlr->getL1DCache()->getPerfModel()->getLatency(at)); break;
  case MemComponent::L2_CACHE: getShmemPerfModel()->incrCurrTime(_L2_cache_cntlr->getL2Cache()->getPerfModel()->getLatency(at)); break;
  case MemComponent::INVALID: break;
  default: CHECK(0);
  }
}
// sendMsg (…msi/memory_manager.cc:306-332) into the canonical schedule
void MSI::MemoryManager::sendMsg(tile_id_t receiver, ShmemMsg& msg)
{
  const UInt32 src = getTile()->getId();
  Time t = getShmemPerfModel()->getCurrTime();
  Byte* buf = msg.makeMsgBuf();
#ifdef GG_PROTO_SHL2
  // the core -> L1 request of a miss (…sh_l2_msi/l1_cache_cntlr.cc:131-136) is handled at once
  const bool at_once = (UInt32)receiver == src && msg.getSenderMemComponent() == MemComponent::CORE;
#else
  const bool at_once = (UInt32)receiver == src && msg.getReceiverMemComponent() == MemComponent::L2_CACHE &&
      (msg.getSenderMemComponent() == MemComponent::L1_DCACHE || msg.getSenderMemComponent() == MemComponent::L1_ICACHE);
#endif
  if (at_once) {
    // the L1 -> L2 request of a miss is handled at once
    NetPacket p; p.time = t; p.sender = Tile::getMainCoreId(src); p.receiver = p.sender;
    p.length = msg.getMsgLen(); p.data = buf;
    __handleMsgFromNetwork(p);
    delete[] buf;
    return;
  }
  HTile& S = g_t[src];
  HMsg m;
  m.src = src; m.dst = (UInt32)receiver; m.seq = S.seq++; m.type = gg_type(msg.getType());
  m.send = t.getTime(); m.arrival = m.send;
  m.buf.assign(buf, buf + msg.getMsgLen());
  delete[] buf;
  g_step.push_back(m);
  S.st[S_SENT]++;
  if (m.type == 13) S.st[S_SENT_IFC]++;                                      // INV_FLUSH_COMBINED_REQ (MOSI)
  else if (m.type >= 14 && m.type <= 16) S.st[S_SENT_IFC + m.type - 14]++;  // DRAM_FETCH_REQ / STORE_REQ / FETCH_REP (sh_l2)
  else if (m.type >= 17) {}                                                 // MESI's own types: msgs_sent only
  else S.st[S_BYTYPE + m.type - 1]++;
}
void MSI::MemoryManager::broadcastMsg(ShmemMsg&) { CHECK(0); }   // full_map never broadcasts

Tile::Tile(tile_id_t id) : _id(id), _network(NULL), _core(NULL), _memory_manager(NULL), _dvfs_manager(NULL),
                           _tile_energy_monitor(NULL), _remote_query_helper(NULL)
{
  _memory_manager = new MSI::MemoryManager(this);
}
Tile::~Tile() { delete _memory_manager; }

// ===========================================================================
// the canonical schedule
// ===========================================================================
static UInt32 modeled_bits(UInt32 type)        // network_model.cc:185-200 + shmem_msg.cc:100-125 (…mosi/shmem_msg.cc:122-151)
{
  UInt32 idb = H.T > 1 ? ceilLog2(H.T) : 0;
  bool data = type == 6 || type == 7 || type == 10 || type == 11 || type == 15 || type == 16 || type == 18;   // EX_REP, SH_REP, FLUSH_REP, WB_REP, DRAM_STORE_REQ, DRAM_FETCH_REP, SH_REP_EX (DOWNGRADE_REP: no data buffer)
  return 2 * idb + 4 + 48 + (data ? 512 : 0) + (type == 13 ? idb : 0);   // INV_FLUSH_COMBINED_REQ: + single receiver
}
static UInt64 lat_ps(UInt64 cycles) { return (UInt64)ceil(((double)1000 * cycles) / 1.0); }
// emesh_hop_counter (network_model_emesh_hop_counter.cc:143-157) / magic + serialization (network_model.cc:142-150)
static void route(HMsg& m)
{
  if (m.src == m.dst) return;
  UInt32 bits = modeled_bits(m.type);
  UInt64 zl;
  if (H.net == 0) {
    zl = lat_ps(1);
  } else {
    UInt32 w = (UInt32)floor(sqrt((double)H.T));
    int hops = abs((int)(m.src % w) - (int)(m.dst % w)) + abs((int)(m.src / w) - (int)(m.dst / w));
    UInt64 nf = (bits % 64 == 0) ? bits / 64 : bits / 64 + 1;
    zl = lat_ps((UInt64)hops * 2) + lat_ps(nf);
  }
  m.arrival = m.send + zl;
  g_t[m.src].net[NC_PS]++;
  g_t[m.dst].net[NC_PR]++;
  g_t[m.dst].net[NC_LAT] += zl;
}

static void deliver(HTile& D, const HMsg& m)
{
  NetPacket p;
  p.time = Time(m.arrival); p.sender = Tile::getMainCoreId(m.src); p.receiver = Tile::getMainCoreId(m.dst);
  p.length = m.buf.size(); p.data = &m.buf[0];
  D.st[S_RECV]++;
  D.mm->__handleMsgFromNetwork(p);
}

static bool chan_lt(const HMsg& a, const HMsg& b) { return a.src < b.src || (a.src == b.src && a.seq < b.seq); }

static void drain_inbox(UInt32 t)
{
  HTile& T = g_t[t];
  vector<HMsg> in;
  in.swap(T.inbox);
  sort(in.begin(), in.end(), chan_lt);
  vector<bool> used(in.size(), false);
  for (size_t k = 0; k < in.size(); ++k) {
    size_t best = (size_t)-1; UInt32 prev = (UInt32)-1;
    for (size_t i = 0; i < in.size(); ++i) {
      if (used[i]) continue;
      if (in[i].src == prev) continue;
      prev = in[i].src;
      if (best == (size_t)-1 || in[i].arrival < in[best].arrival ||
          (in[i].arrival == in[best].arrival && in[i].src < in[best].src)) best = i;
    }
    used[best] = true;
    g_cur = t;
    deliver(T, in[best]);
  }
}

// the app coroutine: Core::initiateMemoryAccess per trace record (core.cc:139-266)
static void app_main(int t)
{
  HTile& T = g_t[t];
  Byte data[8];
  memset(data, 0, sizeof(data));
  for (;;) {
    while (!T.blocked && T.rec < T.rec_end) {
      UInt32 meta = g_meta[T.rec];
      UInt64 s = T.clk + (UInt64)((meta & 0x7FFFFFFFu) >> 1) * lat_ps(1);
      if (s >= g_barrier) break;
      IntPtr addr = g_addr[T.rec] & ~(IntPtr)63;
      Core::mem_op_t op = (meta & 1) ? Core::WRITE : Core::READ;
      T.resumed_by_handler = false;
      Time curr(s);
      bool l1hit = T.mm->__coreInitiateMemoryAccess(MemComponent::L1_DCACHE, Core::NONE, op, addr, 0, data, 8, curr, true);
      UInt64 start = T.blocked ? T.pend_start : s;
      UInt32 level = l1hit ? 0 : (T.resumed_by_handler ? 2 : 1);
      UInt64 lat = curr.getTime() - s;
      if (g_out) g_out[T.rec] = (lat << 2) | level;
      T.st[S_ACC]++; T.st[S_LAT] += lat;
      T.st[level == 0 ? S_L1H : level == 1 ? S_L2H : S_MISS]++;
      T.clk = curr.getTime(); T.st[S_CLOCK] = T.clk;
      T.rec++;
      T.blocked = false;
      (void)start;
      if (T.resumed_by_handler) { T.resumed_by_handler = false; app_yield(T); }
    }
    app_yield(T);
  }
}
static void app_entry(int t) { app_main(t); }

static void run_app(UInt32 t)
{
  HTile& T = g_t[t];
  if (T.blocked || T.rec >= T.rec_end) return;
  ucontext_t here;
  T.ret_ctx = &here;
  g_cur = t;
  swapcontext(&here, &T.app_ctx);
}

static int run_all(UInt64* quanta_out, UInt64* steps_out)
{
  UInt64 q = 0, quanta = 0, steps = 0;
  for (;;) {
    g_barrier = (q + 1) * H.quantum_ps;
    for (;;) {
      for (UInt32 t = 0; t < H.T; ++t) { drain_inbox(t); run_app(t); }
      ++steps;
      if (g_step.empty()) break;
      vector<HMsg> msgs;
      msgs.swap(g_step);
      for (size_t i = 0; i < msgs.size(); ++i) {
        route(msgs[i]);
        if (shard_of(msgs[i].src) == shard_of(msgs[i].dst)) g_t[msgs[i].dst].inbox.push_back(msgs[i]);
        else g_bnd.push_back(msgs[i]);
      }
    }
    ++quanta;
    size_t nb = g_bnd.size();
    for (size_t i = 0; i < nb; ++i) g_t[g_bnd[i].dst].inbox.push_back(g_bnd[i]);
    g_bnd.clear();
    UInt64 active = 0, blocked = 0, mn = ~0ull;
    for (UInt32 t = 0; t < H.T; ++t) {
      HTile& T = g_t[t];
      if (T.rec >= T.rec_end) continue;
      active++;
      if (T.blocked) { blocked++; continue; }
      UInt64 s = T.clk + (UInt64)((g_meta[T.rec] & 0x7FFFFFFFu) >> 1) * lat_ps(1);
      mn = min(mn, s);
    }
    if (active == 0 && nb == 0) break;
    if (nb == 0 && blocked == 0) q = max(q + 1, mn / H.quantum_ps);
    else if (nb == 0) { fprintf(stderr, "coh_harness: deadlock\n"); return 1; }
    else q = q + 1;
  }
  *quanta_out = quanta; *steps_out = steps;
  return 0;
}

// ===========================================================================
// the configs[2..4] hotspot generator (oracle_gen_hotspot)
// ===========================================================================
static UInt64 splitmix_at(UInt64 seed, UInt64 i)
{
  UInt64 z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void gen_hotspot(UInt32 tile, UInt64 n, UInt32 hot_lines, UInt64* addr, UInt32* meta)
{
  const UInt64 seed = 0x9E3779B97F4A7C15ull ^ (UInt64)tile;
  for (UInt64 k = 0; k < n; ++k) {
    UInt64 z = splitmix_at(seed, k);
    bool hot = hot_lines && (((z >> 40) & 0xFF) < 51);
    addr[k] = hot ? (1ull << 44) + ((z & 0xFFFFFFFFull) % hot_lines) * 64ull : ((UInt64)tile << 26) + ((z & 0x7FFF) << 6);
    UInt32 gap = (UInt32)__builtin_ctz((UInt32)(((z >> 48) & 0xFF) | 0x100)) +
                 (UInt32)__builtin_ctz((UInt32)(((z >> 56) & 0xFF) | 0x100));
    meta[k] = ((((z >> 32) & 0xFF) % 3) == 0 ? 1u : 0u) | (gap << 1);
  }
}

// the configs[4] stress generator (oracle_gen_stress):
// WRITE p = 1/2; 77/256 of the records to a 4096-line pool at byte 2^45, pool
// line L shared by the tiles of group L mod groups (T/64 groups by a 32-bit
// hash of the tile), the rest private as the hotspot generator
static UInt32 stress_group(UInt32 t, UInt32 groups)
{
  UInt32 x = t + 0x9E3779B9u;
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x % groups;
}
static void gen_stress(UInt32 tile, UInt64 n, UInt32 num_tiles, UInt64* addr, UInt32* meta)
{
  const UInt64 seed = 0x9E3779B97F4A7C15ull ^ (UInt64)tile;
  const UInt32 pool_lines = 4096, groups = num_tiles >= 128 ? num_tiles / 64 : 1;
  const UInt32 per_group = pool_lines / groups ? pool_lines / groups : 1;
  for (UInt64 k = 0; k < n; ++k) {
    UInt64 z = splitmix_at(seed, k);
    bool pool = ((z >> 40) & 0xFF) < 77;
    addr[k] = pool ? (1ull << 45) + (UInt64)(stress_group(tile, groups) + groups * ((UInt32)(z & 0xFFFFFFFFull) % per_group)) * 64ull
                   : ((UInt64)tile << 26) + ((z & 0x7FFF) << 6);
    UInt32 gap = (UInt32)__builtin_ctz((UInt32)(((z >> 48) & 0xFF) | 0x100)) +
                 (UInt32)__builtin_ctz((UInt32)(((z >> 56) & 0xFF) | 0x100));
    meta[k] = (UInt32)((z >> 32) & 1u) | (gap << 1);
  }
}

// ===========================================================================
// fixtures
// ===========================================================================
static string g_dir;
static void write_bin(const string& name, const void* p, size_t bytes)
{
  string path = g_dir + "/" + name;
  FILE* f = fopen(path.c_str(), "wb");
  CHECK(f);
  CHECK(fwrite(p, 1, bytes, f) == bytes);
  fclose(f);
}

// a captured trace (workload 2): tile-major records and tile offsets, raw
// little-endian files <prefix>.addr (u64), .meta (u32), .offs (u64, T + 1)
struct RawTrace { vector<UInt64> addr, offs; vector<UInt32> meta; };
template <class V> static void read_raw(const string& path, V& v)
{
  FILE* f = fopen(path.c_str(), "rb");
  CHECK(f);
  fseek(f, 0, SEEK_END);
  const long bytes = ftell(f);
  fseek(f, 0, SEEK_SET);
  v.resize((size_t)bytes / sizeof(v[0]));
  CHECK(fread(&v[0], sizeof(v[0]), v.size(), f) == v.size());
  fclose(f);
}

static void run_case(FILE* man, bool first, const char* name, UInt32 T, UInt32 N, UInt32 hot, UInt32 K, UInt32 net,
                     UInt32 dir_entries, UInt32 dir_assoc, UInt32 l2_assoc = 8, UInt32 workload = 0,
                     const RawTrace* raw = NULL)
{
  H.T = T; H.K = K; H.net = net; H.dir_entries = dir_entries; H.dir_assoc = dir_assoc; H.quantum_ps = 1000000;
  H.l2_assoc = l2_assoc; H.workload = workload;
  build_shard_map();
  g_t.clear(); g_t.resize(T); g_step.clear(); g_bnd.clear(); g_cc.clear(); g_dc.clear(); g_dram.clear();
  vector<UInt64> offs(T + 1);
  for (UInt32 t = 0; t <= T; ++t) offs[t] = raw ? raw->offs[t] : (UInt64)t * N;
  const size_t nrec = (size_t)offs[T];
  vector<UInt64> addr(nrec); vector<UInt32> meta(nrec); vector<UInt64> out(nrec, 0);
  if (raw) {
    CHECK(raw->offs.size() == T + 1 && raw->addr.size() == nrec && raw->meta.size() == nrec);
    addr = raw->addr; meta = raw->meta;
  }
  for (UInt32 t = 0; t < T && !raw; ++t) {
    if (workload == 1) gen_stress(t, N, T, &addr[(size_t)t * N], &meta[(size_t)t * N]);
    else gen_hotspot(t, N, hot, &addr[(size_t)t * N], &meta[(size_t)t * N]);
  }
  g_addr = nrec ? &addr[0] : NULL; g_meta = nrec ? &meta[0] : NULL; g_out = nrec ? &out[0] : NULL;
  for (UInt32 t = 0; t < T; ++t) {
    HTile& X = g_t[t];
    X.tile = new Tile(t);
    X.mm = (MSI::MemoryManager*)X.tile->getMemoryManager();
    X.mm->enableModels();                                  // synthetic_memory.cc:96
    X.rec = offs[t]; X.rec_end = offs[t + 1]; X.clk = 0; X.blocked = false; X.resumed_by_handler = false;
    X.pend_start = 0; X.seq = 0;
    memset(X.st, 0, sizeof(X.st)); memset(X.net, 0, sizeof(X.net));
    X.stack.resize(T > 256 ? 1 << 18 : 1 << 20);
    getcontext(&X.app_ctx);
    X.app_ctx.uc_stack.ss_sp = &X.stack[0];
    X.app_ctx.uc_stack.ss_size = X.stack.size();
    X.app_ctx.uc_link = NULL;
    makecontext(&X.app_ctx, (void (*)())app_entry, 1, (int)t);
  }
  UInt64 quanta = 0, steps = 0;
  CHECK(run_all(&quanta, &steps) == 0);
  vector<UInt64> st((size_t)T * S_N, 0), cc((size_t)T * 2 * CC_N, 0);
  for (UInt32 t = 0; t < T; ++t) {
    HTile& X = g_t[t];
    UInt64* s = &st[(size_t)t * S_N];
    memcpy(s, X.st, sizeof(X.st));
#ifndef GG_PROTO_SHL2                                        // (sh_l2: the directory lives in the L2 lines)
    DirectoryCache* dc = X.mm->getDramDirectoryCache();
    s[S_DACC] = dcount(dc)[DC_ACC]; s[S_DEV] = dcount(dc)[DC_EV]; s[S_DBI] = dcount(dc)[DC_BI];
#endif
    HDram& d = g_dram[X.mm->getDramCntlr()];
    s[S_DRAM] = d.n; s[S_DRAMLAT] = d.lat; s[S_DRAMQD] = d.qd; s[S_DRAMQR] = d.qreq;
    s[S_DRAMQA] = d.q ? d.q->analytical_requests : 0;
    s[S_DRAMQU] = d.q ? d.q->util : 0; s[S_DRAMQL] = d.q ? d.q->last_req : 0;
    memcpy(&cc[((size_t)t * 2 + 0) * CC_N], ccount(X.mm->getL1DCache()), sizeof(UInt64) * CC_N);
    memcpy(&cc[((size_t)t * 2 + 1) * CC_N], ccount(X.mm->getL2Cache()), sizeof(UInt64) * CC_N);
  }
  vector<UInt64> nc((size_t)T * 3);
  for (UInt32 t = 0; t < T; ++t) { nc[t * 3] = g_t[t].net[NC_PS]; nc[t * 3 + 1] = g_t[t].net[NC_PR]; nc[t * 3 + 2] = g_t[t].net[NC_LAT]; }
  string n = name;
  write_bin("coh_" + n + "_out.u64", &out[0], out.size() * 8);
  write_bin("coh_" + n + "_stats.u64", &st[0], st.size() * 8);
  write_bin("coh_" + n + "_cache.u64", &cc[0], cc.size() * 8);
  write_bin("coh_" + n + "_net.u64", &nc[0], nc.size() * 8);
#ifdef GG_PROTO_MOSI
  {
    // the MOSI controllers' event counters [T][32] (GG_PS_*, include/graphite_gpu.h)
    // and their outputSummary text (l2_cache_cntlr.cc:638-649,
    // dram_directory_cntlr.cc:1041-1142), one "Tile t:" block per tile
    vector<UInt64> ps((size_t)T * 32, 0);
    string txt;
    for (UInt32 t = 0; t < T; ++t) {
      MSI::DramDirectoryCntlr* d = g_t[t].mm->_dram_directory_cntlr;
      MSI::L2CacheCntlr* l2 = g_t[t].mm->_L2_cache_cntlr;
      UInt64* v = &ps[(size_t)t * 32];
      v[0] = d->_total_exreq; v[1] = d->_total_exreq_in_modified_state; v[2] = d->_total_exreq_in_shared_state;
      v[3] = d->_total_exreq_with_upgrade_replies; v[4] = d->_total_exreq_in_uncached_state;
      v[5] = d->_total_exreq_serialization_time.getTime(); v[6] = d->_total_exreq_processing_time.getTime();
      v[7] = d->_total_shreq; v[8] = d->_total_shreq_in_modified_state; v[9] = d->_total_shreq_in_shared_state;
      v[10] = d->_total_shreq_in_uncached_state;
      v[11] = d->_total_shreq_serialization_time.getTime(); v[12] = d->_total_shreq_processing_time.getTime();
      v[13] = d->_total_nullifyreq; v[14] = d->_total_nullifyreq_in_modified_state; v[15] = d->_total_nullifyreq_in_shared_state;
      v[16] = d->_total_nullifyreq_in_uncached_state;
      v[17] = d->_total_nullifyreq_serialization_time.getTime(); v[18] = d->_total_nullifyreq_processing_time.getTime();
      v[19] = d->_total_invalidations_unicast_mode; v[20] = d->_total_invalidations_broadcast_mode;
      v[21] = d->_total_sharers_invalidated_unicast_mode; v[22] = d->_total_sharers_invalidated_broadcast_mode;
      v[23] = d->_total_invalidation_processing_time_unicast_mode.getTime();
      v[24] = d->_total_invalidation_processing_time_broadcast_mode.getTime();
      v[25] = l2->_total_invalidations; v[26] = l2->_total_evictions;
      v[27] = l2->_total_dirty_evictions_exreq; v[28] = l2->_total_clean_evictions_exreq;
      v[29] = l2->_total_dirty_evictions_shreq; v[30] = l2->_total_clean_evictions_shreq;
      std::ostringstream os;
      os << "Tile " << t << ":\n";
      l2->outputSummary(os);
      d->outputSummary(os);
      txt += os.str();
    }
    write_bin("coh_" + n + "_proto.u64", &ps[0], ps.size() * 8);
    write_bin("coh_" + n + "_summary.txt", txt.data(), txt.size());
  }
#endif
  fprintf(man, "%s  \"%s\": {\"tiles\": %u, \"per_tile\": %u, \"hot_lines\": %u, \"num_shards\": %u, \"net\": %u, "
          "\"dir_entries\": %u, \"dir_assoc\": %u, \"l2_assoc\": %u, \"workload\": \"%s\", \"records\": %llu, "
          "\"quanta\": %llu, \"steps\": %llu}",
          first ? "" : ",\n", name, T, N, hot, K, net, dir_entries, dir_assoc, l2_assoc,
          workload == 2 ? "fft_real_p16_m10" : workload ? "stress" : "hotspot", (unsigned long long)nrec,
          (unsigned long long)quanta, (unsigned long long)steps);
  printf("  coh %-10s tiles %u x %u: %llu quanta, %llu steps\n", name, T, N, (unsigned long long)quanta,
         (unsigned long long)steps);
  for (UInt32 t = 0; t < T; ++t) delete g_t[t].tile;
}

int main(int argc, char** argv)
{
  g_dir = argc > 1 ? argv[1] : ".";
#if defined(GG_PROTO_SHL2)
  // pr_l1_sh_l2_msi: the hotspot / stress shapes of the MSI fixtures (shared
  // L2 slices: remote L2 hits, DRAM fetches and stores through the DRAM
  // controller, L2 evictions with NULLIFY of their sharers, upgrade replies)
  // and the reference's FFT
#ifdef GG_SHL2_MESI
  const string pre = "mesi_";                                   // pr_l1_sh_l2_mesi
#else
  const string pre = "shl2_";
#endif
  string mp = g_dir + "/coh_" + pre + "manifest.json";
  FILE* man = fopen(mp.c_str(), "w");
  CHECK(man);
  fprintf(man, "{\n");
#define N(x) (pre + x).c_str()
  run_case(man, true, N("private16"), 16, 1500, 0, 1, 1, 0, 16);
  run_case(man, false, N("hot16"), 16, 1500, 64, 1, 1, 0, 16);
  run_case(man, false, N("hot16magic"), 16, 1000, 8, 1, 0, 0, 16);
  run_case(man, false, N("shard64"), 64, 400, 32, 8, 1, 0, 16);
  run_case(man, false, N("shard256"), 256, 150, 64, 8, 1, 0, 16);
  run_case(man, false, N("stress256w16"), 256, 96, 0, 8, 1, 0, 16, 16, 1);
  run_case(man, false, N("shard1024"), 1024, 24, 256, 8, 1, 0, 16);
  // L2 slice evictions (2-way slices; a 1-way slice whose one line waits on a
  // request has no replacement candidate, l2_cache_replacement_policy.cc:55-66):
  // NULLIFY of sharers and owners, DRAM stores
  run_case(man, false, N("evict16"), 16, 12000, 64, 1, 1, 0, 16, 2);
  run_case(man, false, N("evict16s4"), 16, 12000, 64, 4, 1, 0, 16, 2);
  if (argc > 2) {
    RawTrace fft;
    read_raw(string(argv[2]) + ".addr", fft.addr);
    read_raw(string(argv[2]) + ".meta", fft.meta);
    read_raw(string(argv[2]) + ".offs", fft.offs);
    run_case(man, false, N("fft10"), 16, 0, 0, 1, 1, 0, 16, 8, 2, &fft);
  }
#undef N
  fprintf(man, "\n}\n");
  fclose(man);
  return 0;
#elif defined(GG_PROTO_MOSI)
  // pr_l1_pr_l2_dram_directory_mosi: the hotspot / stress shapes of the MSI
  // fixtures (OWNED lines, upgrade replies, combined invalidate-flush, the
  // directory's cached data, NULLIFY of OWNED entries) and the reference's FFT
  string mp = g_dir + "/coh_mosi_manifest.json";
  FILE* man = fopen(mp.c_str(), "w");
  CHECK(man);
  fprintf(man, "{\n");
  run_case(man, true, "mosi_hot16", 16, 1500, 64, 1, 1, 0, 16);
  run_case(man, false, "mosi_hot16magic", 16, 1000, 8, 1, 0, 0, 16);
  run_case(man, false, "mosi_dir16", 16, 1000, 32, 1, 1, 64, 4);
  run_case(man, false, "mosi_shard64", 64, 400, 32, 8, 1, 0, 16);
  run_case(man, false, "mosi_shard256", 256, 150, 64, 8, 1, 0, 16);
  run_case(man, false, "mosi_stress256w16", 256, 96, 0, 8, 1, 0, 16, 16, 1);
  run_case(man, false, "mosi_shard1024", 1024, 24, 256, 8, 1, 0, 16);
  // L2 evictions (private footprints past the 8192-line L2): FLUSH_REP of
  // MODIFIED / OWNED lines, INV_REP of SHARED ones, "just an eviction" writes
  run_case(man, false, "mosi_evict16", 16, 12000, 64, 1, 1, 0, 16);
  run_case(man, false, "mosi_evict16s4", 16, 12000, 64, 4, 1, 0, 16);
  if (argc > 2) {
    RawTrace fft;
    read_raw(string(argv[2]) + ".addr", fft.addr);
    read_raw(string(argv[2]) + ".meta", fft.meta);
    read_raw(string(argv[2]) + ".offs", fft.offs);
    run_case(man, false, "mosi_fft10", 16, 0, 0, 1, 1, 0, 16, 8, 2, &fft);
  }
  fprintf(man, "\n}\n");
  fclose(man);
  return 0;
#else
  string mp = g_dir + "/coh_manifest.json";
  FILE* man = fopen(mp.c_str(), "w");
  CHECK(man);
  fprintf(man, "{\n");
  run_case(man, true, "private16", 16, 1500, 0, 1, 1, 0, 16);
  run_case(man, false, "hot16", 16, 1500, 64, 1, 1, 0, 16);
  run_case(man, false, "hot16magic", 16, 1000, 8, 1, 0, 0, 16);
  run_case(man, false, "dir16", 16, 1000, 32, 1, 1, 64, 4);
  run_case(man, false, "shard64", 64, 400, 32, 8, 1, 0, 16);
  run_case(man, false, "hot256", 256, 120, 64, 1, 1, 0, 16);
  run_case(man, false, "shard256", 256, 150, 64, 8, 1, 0, 16);
  // configs[4] shape: 16-way L2 (512 sets), the stress generator (50/50 R/W,
  // 4096-line pool, ~64 sharers per pool line), 8 logical shards
  run_case(man, false, "stress256w16", 256, 96, 0, 8, 1, 0, 16, 16, 1);
  // configs[3] scale: 1024 tiles x 8 logical shards, 256 hot lines, reduced length
  run_case(man, false, "shard1024", 1024, 24, 256, 8, 1, 0, 16);
  // L2 evictions (private footprints past the 8192-line L2)
  run_case(man, false, "evict16", 16, 12000, 64, 1, 1, 0, 16);
  run_case(man, false, "evict16s4", 16, 12000, 64, 4, 1, 0, 16);
  // configs[0]: the reference's own fft.C (-p16 -m10) as captured by
  // tools/fft_trace (tests/golden/fft_real_p16_m10.npz, accesses only: the
  // BARRIER release is restated, not the reference's SyncServer), 16 tiles,
  // emesh_hop_counter; exported to raw files by make_golden.sh
  if (argc > 2) {
    RawTrace fft;
    read_raw(string(argv[2]) + ".addr", fft.addr);
    read_raw(string(argv[2]) + ".meta", fft.meta);
    read_raw(string(argv[2]) + ".offs", fft.offs);
    run_case(man, false, "fft10", 16, 0, 0, 1, 1, 0, 16, 8, 2, &fft);
  }
  fprintf(man, "\n}\n");
  fclose(man);
  return 0;
#endif
}
