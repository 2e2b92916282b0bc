// ref_harness.cc — drives the REFERENCE's own classes, compiled from the
// sources where they lie under /root/reference (see oracle/ref/Makefile), and
// writes golden fixtures for tests/golden/.
//
// TEST INFRASTRUCTURE ONLY: never shipped, never linked into graphite_amd/.
//
// Reference code exercised verbatim, its own assert() calls active (only
// log.h's LOG_* are compiled out, because the logging back end
// common/misc/log.cc needs Boost, which this image lacks;
// oracle/ref/assert_prelude.h):
//   CacheSet                      common/tile/memory_subsystem/cache/cache_set.cc
//   LRUReplacementPolicy          .../cache/lru_replacement_policy.cc
//   RoundRobinReplacementPolicy   .../cache/round_robin_replacement_policy.cc
//   CacheReplacementPolicy        .../cache/cache_replacement_policy.cc
//   CacheLineInfo, PrL2CacheLineInfo .../cache/cache_line_info.cc,
//                                 .../pr_l1_pr_l2_dram_directory_msi/cache_line_info.cc
//   IntervalTree                  common/misc/interval_tree.cc
//   QueueModelMG1                 common/shared_models/queue_models/queue_model_m_g_1.cc
//
// The thin glue the reference keeps in files that cannot be compiled here
// (Cache in cache.cc, the L1/L2 controllers, QueueModelHistoryTree) is
// restated below on top of those classes, statement by statement, with the
// file:line it follows; it is a second, independent restatement next to
// oracle/gg_oracle.c, so the two cross-check each other.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdint.h>
#include <string>
#include <vector>
#include <utility>

#include "cache_set.h"
#include "cache_line_info.h"
#include "cache_replacement_policy.h"
#include "cache_state.h"
#include "pr_l1_pr_l2_dram_directory_msi/cache_line_info.h"
#include "interval_tree.h"
#include "queue_model_m_g_1.h"

using namespace std;

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "ref_harness: check failed %s:%d: %s\n", __FILE__, __LINE__, #c); exit(2); } } while (0)

// --------------------------------------------------------------------------
// Cache glue (common/tile/memory_subsystem/cache/cache.cc)
// --------------------------------------------------------------------------
enum { TAG_R = 0, TAG_W, DATA_R, DATA_W };
enum { C_ACC = 0, C_MISS, C_RACC, C_RMISS, C_WACC, C_WMISS, C_EV, C_DEV, C_TR, C_TW, C_DR, C_DW, C_N };

struct RefCache {
  UInt32 num_sets, assoc, log_line;
  bool write_back;
  CacheReplacementPolicy* policy;
  vector<CacheSet*> sets;
  UInt64 c[C_N];
  SInt32 level;

  RefCache(UInt32 size_kb, UInt32 a, UInt32 line, const string& pol, SInt32 lvl, bool wb)
      : assoc(a), write_back(wb), level(lvl) {
    num_sets = size_kb * 1024 / (a * line);                          // cache.cc:44
    log_line = 0; while ((1u << log_line) < line) ++log_line;         // floorLog2
    policy = CacheReplacementPolicy::create(pol, size_kb, a, line);   // cache_replacement_policy.cc:16-31
    for (UInt32 i = 0; i < num_sets; ++i)
      sets.push_back(new CacheSet(i, PR_L1_PR_L2_DRAM_DIRECTORY_MSI, lvl, policy, a, line));
    memset(c, 0, sizeof(c));
  }
  ~RefCache() { for (size_t i = 0; i < sets.size(); ++i) delete sets[i]; delete policy; }

  CacheSet* getSet(IntPtr addr) const { return sets[(addr >> log_line) & (num_sets - 1)]; }  // cache_hash_fn.h:17
  IntPtr getTag(IntPtr addr) const { return addr >> log_line; }                             // cache.cc:495

  // Cache::accessCacheLine (cache.cc:84-112)
  bool accessCacheLine(IntPtr addr, bool store) {
    CacheSet* s = getSet(addr);
    UInt32 idx = (UInt32)-1;
    CacheLineInfo* li = s->find(getTag(addr), &idx);
    if (!li) return false;
    if (!store) s->read_line(idx, 0, NULL, 0); else s->write_line(idx, 0, NULL, 0);
    c[store ? C_DW : C_DR]++;
    return true;
  }
  // Cache::insertCacheLine (cache.cc:114-184)
  void insertCacheLine(IntPtr addr, CacheLineInfo* in, bool* ev, IntPtr* ev_addr, CacheLineInfo* ev_info) {
    CacheSet* s = getSet(addr);
    s->insert(in, NULL, ev, ev_info, NULL);
    *ev_addr = ev_info->getTag() << log_line;
    if (*ev) {
      CHECK(ev_info->getCState() != CacheState::INVALID);
      c[C_TR]++; c[C_DR]++; c[C_EV]++;
      if (write_back && CacheState(ev_info->getCState()).dirty()) c[C_DEV]++;
    } else {
      c[C_TR]++;
    }
    c[C_TW]++; c[C_DW]++;
  }
  // Cache::getCacheLineInfo (cache.cc:187-215)
  void getCacheLineInfo(IntPtr addr, CacheLineInfo* out) {
    CacheLineInfo* li = getSet(addr)->find(getTag(addr));
    if (li) out->assign(li);
    c[C_TR]++;
  }
  // Cache::setCacheLineInfo (cache.cc:218-241)
  bool setCacheLineInfo(IntPtr addr, CacheLineInfo* in) {
    CacheLineInfo* li = getSet(addr)->find(getTag(addr));
    if (!li) return false;
    li->assign(in);
    c[C_TW]++;
    return true;
  }
  // Cache::updateMissCounters (cache.cc:321-360)
  void updateMissCounters(bool write, bool miss) {
    c[C_ACC]++;
    if (!write) c[C_RACC]++; else c[C_WACC]++;
    if (miss) { c[C_MISS]++; if (!write) c[C_RMISS]++; else c[C_WMISS]++; }
  }
};

typedef PrL1PrL2DramDirectoryMSI::PrL2CacheLineInfo L2Info;
typedef PrL1PrL2DramDirectoryMSI::PrL1CacheLineInfo L1Info;
static UInt64 loc_of(L1Info*) { return 0; }
static UInt64 loc_of(L2Info* i) { return (UInt64)i->getCachedLoc(); }
static void set_loc(L1Info*, UInt32) {}
static void set_loc(L2Info* i, UInt32 loc) { if (loc) i->setForcedCachedLoc(MemComponent::L1_DCACHE); }

// --------------------------------------------------------------------------
// Private-mode L1/L2 controllers (pr_l1_pr_l2_dram_directory_msi/)
// --------------------------------------------------------------------------
enum { R_L1 = 0, R_L2 = 1, R_DIR = 2, R_UPG = 4, R_L1EV = 8, R_L2EV = 16, R_L2DIRTY = 32, R_L2INV = 64 };

struct RefTile {
  RefCache l1, l2;
  RefTile(UInt32 l1kb, UInt32 l1a, const string& l1p, UInt32 l2kb, UInt32 l2a, const string& l2p)
      : l1(l1kb, l1a, 64, l1p, PrL1PrL2DramDirectoryMSI::L1, false),
        l2(l2kb, l2a, 64, l2p, PrL1PrL2DramDirectoryMSI::L2, true) {}

  // L1CacheCntlr::invalidateCacheLine (l1_cache_cntlr.cc:293-305)
  bool l1Invalidate(IntPtr a) {
    L1Info info;
    l1.getCacheLineInfo(a, &info);
    if (info.isValid()) { info.invalidate(); CHECK(l1.setCacheLineInfo(a, &info)); return true; }
    return false;
  }
  // L1CacheCntlr::accessCache (l1_cache_cntlr.cc:182-205)
  void l1Access(IntPtr a, bool w) {
    CHECK(l1.accessCacheLine(a, w));
    if (w) CHECK(l2.accessCacheLine(a, true));        // L2CacheCntlr::writeCacheLine
  }
  // L2CacheCntlr::insertCacheLineInL1 (l2_cache_cntlr.cc:133-165)
  void insertInL1(IntPtr a, CacheState::Type cs, UInt32* res) {
    L1Info in; in.setTag(l1.getTag(a)); in.setCState(cs);
    L1Info ev_info; bool ev = false; IntPtr ev_addr = 0;
    l1.insertCacheLine(a, &in, &ev, &ev_addr, &ev_info);
    if (ev) {
      *res |= R_L1EV;
      L2Info l2i;
      l2.getCacheLineInfo(ev_addr, &l2i);
      CHECK(l2i.getCachedLoc() == MemComponent::L1_DCACHE);   // LOG_ASSERT_ERROR (l2:152-157)
      l2i.clearCachedLoc(MemComponent::L1_DCACHE);
      CHECK(l2.setCacheLineInfo(ev_addr, &l2i));
    }
  }
  // L2CacheCntlr::insertCacheLine (l2_cache_cntlr.cc:74-116)
  void l2Insert(IntPtr a, CacheState::Type cs, UInt32* res, IntPtr* evicted) {
    L2Info in; in.setTag(l2.getTag(a)); in.setCState(cs); in.setCachedLoc(MemComponent::L1_DCACHE);
    L2Info ev_info; bool ev = false; IntPtr ev_addr = 0;
    l2.insertCacheLine(a, &in, &ev, &ev_addr, &ev_info);
    if (ev) {
      *res |= R_L2EV; *evicted = ev_addr;
      if (ev_info.getCachedLoc() != MemComponent::INVALID)
        if (l1Invalidate(ev_addr)) *res |= R_L2INV;
      if (ev_info.getCState() == CacheState::MODIFIED) *res |= R_L2DIRTY;
      else CHECK(ev_info.getCState() == CacheState::SHARED);
    }
  }
  // L1CacheCntlr::processMemOpFromCore (l1_cache_cntlr.cc:89-180), directory granting
  UInt32 access(IntPtr a, bool w, IntPtr* evicted) {
    UInt32 res = 0; *evicted = ~(IntPtr)0;
    for (int access_num = 1; access_num <= 2; ++access_num) {
      L1Info info;
      l1.getCacheLineInfo(a, &info);
      bool hit = w ? CacheState(info.getCState()).writable() : CacheState(info.getCState()).readable();
      if (access_num == 1) l1.updateMissCounters(w, !hit);
      if (hit) { l1Access(a, w); return res; }
      CHECK(access_num == 1);
      l1Invalidate(a);
      // L2CacheCntlr::processShmemRequestFromL1Cache (l2:180-224)
      L2Info l2i;
      l2.getCacheLineInfo(a, &l2i);
      CacheState::Type cs = l2i.getCState();
      bool l2hit = w ? CacheState(cs).writable() : CacheState(cs).readable();
      l2.updateMissCounters(w, !l2hit);
      if (l2hit) {
        res |= R_L2;
        CHECK(l2.accessCacheLine(a, false));
        insertInL1(a, cs, &res);
        if (l2i.getCachedLoc() != MemComponent::INVALID) {
          CHECK(l2i.getCachedLoc() != MemComponent::L1_DCACHE);
          CHECK(cs == CacheState::SHARED);
          l2i.setForcedCachedLoc(MemComponent::L1_DCACHE);
        } else {
          l2i.setCachedLoc(MemComponent::L1_DCACHE);
        }
        CHECK(l2.setCacheLineInfo(a, &l2i));
        l1Access(a, w);
        return res;
      }
      res |= R_DIR;
      CacheState::Type ns;
      if (w) {   // processExReqFromL1Cache (l2:260-282)
        L2Info x;
        l2.getCacheLineInfo(a, &x);
        CHECK(x.getCState() == CacheState::INVALID || x.getCState() == CacheState::SHARED);
        if (x.getCState() == CacheState::SHARED) {
          x.invalidate(); CHECK(l2.setCacheLineInfo(a, &x)); res |= R_UPG;
        }
        ns = CacheState::MODIFIED;
      } else {
        ns = CacheState::SHARED;
      }
      l2Insert(a, ns, &res, evicted);     // insertCacheLineInHierarchy (l2:167-178)
      insertInL1(a, ns, &res);
    }
    return res;
  }
};

#include "ref_htree.h"

// --------------------------------------------------------------------------
// fixture writing
// --------------------------------------------------------------------------
static string g_dir;
static FILE* g_manifest;
static bool g_first = true;

static void write_bin(const string& name, const void* p, size_t bytes) {
  string path = g_dir + "/" + name;
  FILE* f = fopen(path.c_str(), "wb");
  CHECK(f);
  CHECK(fwrite(p, 1, bytes, f) == bytes);
  fclose(f);
}
static void manifest(const string& entry) {
  fprintf(g_manifest, "%s  %s", g_first ? "" : ",\n", entry.c_str());
  g_first = false;
}

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint64_t sm_at(uint64_t seed, uint64_t i) { return mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ull); }

// The known-answer test of the reference (tests/unit/history_tree/history_tree.cc:9-20)
static const UInt64 kKat[10][3] = {
  {10, 10, 0}, {21, 10, 0}, {32, 10, 0}, {43, 10, 0}, {0, 1, 0},
  {0, 10, 53}, {45, 10, 18}, {60, 4, 13}, {70, 8, 7}, {75, 10, 10}};

static void gen_htree(const char* name, uint64_t seed, int n, UInt64 span, UInt64 maxp, int max_size, bool an,
                      UInt64 gap = 0) {
  RefHistoryTree h(1, max_size, an);
  vector<UInt64> rows;
  UInt64 base = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t z = sm_at(seed, (uint64_t)i);
    // mostly increasing arrival times with out-of-order stragglers
    base += gap + (z & 7);
    UInt64 t = ((z >> 8) % 4 == 0 && base > span) ? base - ((z >> 16) % span) : base;
    UInt64 p = 1 + ((z >> 32) % maxp);
    UInt64 d = h.delay(t, p);
    rows.push_back(t); rows.push_back(p); rows.push_back(d);
  }
  char file[256]; snprintf(file, sizeof file, "%s.u64", name);
  write_bin(file, rows.data(), rows.size() * 8);
  char m[512];
  snprintf(m, sizeof m, "\"%s\": {\"file\": \"%s\", \"kind\": \"htree\", \"rows\": %d, \"cols\": [\"pkt_time\", \"proc_time\", \"delay\"], "
           "\"max_list_size\": %d, \"analytical\": %s, \"analytical_requests\": %llu}",
           name, file, n, max_size, an ? "true" : "false", (unsigned long long)h.analytical_requests);
  manifest(m);
}

// The same arrival process through the other two queue models of
// QueueModel::create (queue_model.cc:19-39).  kind "qlist": history_list
// (aux = no-interleaving flag), "qbasic": basic (aux = GG basic_moving_avg).
static void gen_qlist(const char* name, uint64_t seed, int n, UInt64 span, UInt64 maxp, int max_size, bool an, bool il) {
  RefHistoryList h(1, (UInt32)max_size, an, il);
  vector<UInt64> rows;
  UInt64 base = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t z = sm_at(seed, (uint64_t)i);
    base += (z & 7);
    UInt64 t = ((z >> 8) % 4 == 0 && base > span) ? base - ((z >> 16) % span) : base;
    UInt64 p = 1 + ((z >> 32) % maxp);
    rows.push_back(t); rows.push_back(p); rows.push_back(h.delay(t, p));
  }
  char file[256]; snprintf(file, sizeof file, "%s.u64", name);
  write_bin(file, rows.data(), rows.size() * 8);
  char m[512];
  snprintf(m, sizeof m, "\"%s\": {\"file\": \"%s\", \"kind\": \"qlist\", \"rows\": %d, \"cols\": [\"pkt_time\", \"proc_time\", \"delay\"], "
           "\"max_list_size\": %d, \"analytical\": %s, \"aux\": %d, \"analytical_requests\": %llu}",
           name, file, n, max_size, an ? "true" : "false", il ? 0 : 1, (unsigned long long)h.analytical_requests);
  manifest(m);
}
static void gen_qbasic(const char* name, uint64_t seed, int n, UInt64 span, UInt64 maxp, const char* avg, int gg_avg, UInt32 window) {
  RefBasic h(avg, window);
  vector<UInt64> rows;
  UInt64 base = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t z = sm_at(seed, (uint64_t)i);
    base += (z & 7);
    UInt64 t = ((z >> 8) % 4 == 0 && base > span) ? base - ((z >> 16) % span) : base;
    UInt64 p = 1 + ((z >> 32) % maxp);
    rows.push_back(t); rows.push_back(p); rows.push_back(h.delay(t, p));
  }
  char file[256]; snprintf(file, sizeof file, "%s.u64", name);
  write_bin(file, rows.data(), rows.size() * 8);
  char m[512];
  snprintf(m, sizeof m, "\"%s\": {\"file\": \"%s\", \"kind\": \"qbasic\", \"rows\": %d, \"cols\": [\"pkt_time\", \"proc_time\", \"delay\"], "
           "\"aux\": %u}", name, file, n, (unsigned)(window | ((UInt32)gg_avg << 16)));
  manifest(m);
}

// Random quartet-op sequences on one RefCache.  op codes: 0 get, 1 set, 2 access(load), 3 access(store), 4 insert
// Info is PrL1CacheLineInfo for L1 and PrL2CacheLineInfo for L2 (their assign() must see matching types).
template <class Info>
static void quartet_op(RefCache& c, int level, UInt32 op, UInt64 addr, CacheState::Type ins, UInt32 loc, UInt64* r) {
  UInt64 ok = 1, otag = ~0ull, ost = 0, oloc = 0, ev = 0, evaddr = 0;
  if (op == 0) {
    Info out;
    c.getCacheLineInfo(addr, &out);
    otag = out.getTag(); ost = out.getCState(); oloc = loc_of(&out);
  } else if (op == 1) {
    Info in; in.setTag(c.getTag(addr)); in.setCState(ins); set_loc(&in, level ? loc : 0);
    if (ins == CacheState::INVALID) in.invalidate();
    ok = c.setCacheLineInfo(addr, &in) ? 1 : 0;
  } else if (op == 2 || op == 3) {
    ok = c.accessCacheLine(addr, op == 3) ? 1 : 0;
  } else {
    // insert only lines that are not present (the controllers never insert a present line)
    if (c.getSet(addr)->find(c.getTag(addr))) { ok = 0; }
    else {
      Info in; in.setTag(c.getTag(addr)); in.setCState(ins); set_loc(&in, level ? loc : 0);
      Info evi; bool e = false; IntPtr ea = 0;
      c.insertCacheLine(addr, &in, &e, &ea, &evi);
      ev = e; evaddr = ea; otag = evi.getTag(); ost = evi.getCState(); oloc = loc_of(&evi);
    }
  }
  r[0] = op; r[1] = addr; r[2] = (UInt64)ins; r[3] = level ? loc : 0; r[4] = ok;
  r[5] = otag; r[6] = ost; r[7] = oloc; r[8] = ev; r[9] = evaddr;
}

static void gen_quartet(const char* name, uint64_t seed, int n, UInt32 kb, UInt32 a, const string& pol, int level) {
  RefCache c(kb, a, 64, pol, level == 0 ? PrL1PrL2DramDirectoryMSI::L1 : PrL1PrL2DramDirectoryMSI::L2, level == 1);
  // address pool: 3x the capacity in lines, so sets fill up and evict
  UInt32 lines = c.num_sets * a * 3;
  vector<UInt64> rows;   // op, addr, in_state, in_loc, out_ok, out_tag, out_state, out_loc, eviction, ev_addr
  for (int i = 0; i < n; ++i) {
    uint64_t z = sm_at(seed, (uint64_t)i);
    UInt64 addr = ((z >> 8) % lines) * 64 + 0x10000000ull;
    UInt32 op = (UInt32)(z % 5);
    UInt32 st_pick = (UInt32)((z >> 40) % 3);
    CacheState::Type ins = st_pick == 0 ? CacheState::INVALID : (st_pick == 1 ? CacheState::SHARED : CacheState::MODIFIED);
    UInt32 loc = ((z >> 44) & 1) ? MemComponent::L1_DCACHE : MemComponent::INVALID;
    if (op == 4 && ins == CacheState::INVALID) ins = CacheState::SHARED;
    UInt64 r[10];
    if (level == 0) quartet_op<L1Info>(c, level, op, addr, ins, loc, r);
    else quartet_op<L2Info>(c, level, op, addr, ins, loc, r);
    rows.insert(rows.end(), r, r + 10);
  }
  char file[256]; snprintf(file, sizeof file, "%s.u64", name);
  write_bin(file, rows.data(), rows.size() * 8);
  char m[1024];
  snprintf(m, sizeof m, "\"%s\": {\"file\": \"%s\", \"kind\": \"quartet\", \"rows\": %d, \"level\": %d, \"size_kb\": %u, "
           "\"assoc\": %u, \"policy\": \"%s\", \"cols\": [\"op\", \"addr\", \"in_state\", \"in_loc\", \"ok\", \"out_tag\", "
           "\"out_state\", \"out_loc\", \"eviction\", \"evicted_addr\"], \"counters\": [",
           name, file, n, level, kb, a, pol.c_str());
  string s(m);
  for (int k = 0; k < C_N; ++k) { char b[32]; snprintf(b, sizeof b, "%s%llu", k ? ", " : "", (unsigned long long)c.c[k]); s += b; }
  s += "]}";
  manifest(s);
}

// Private-mode replay fixtures.  gen: 0 = uniform over 2^lines_log2 lines at tile<<26
// (WRITE iff (z>>32)%3==0), 1 = small hot set (64 lines) + stride sweep to force
// upgrades/evictions.
static void gen_modep(const char* name, int gen, uint32_t tiles, uint32_t per_tile, uint32_t lines_log2,
                      UInt32 l1kb, UInt32 l1a, const string& l1p, UInt32 l2kb, UInt32 l2a, const string& l2p) {
  vector<uint8_t> res; vector<UInt64> evicted_sum(tiles, 0); vector<UInt64> counters;
  vector<UInt64> addr_hash(tiles, 0);
  for (uint32_t t = 0; t < tiles; ++t) {
    RefTile T(l1kb, l1a, l1p, l2kb, l2a, l2p);
    uint64_t seed = 0x9E3779B97F4A7C15ull ^ (uint64_t)t;
    for (uint32_t i = 0; i < per_tile; ++i) {
      uint64_t z = sm_at(seed, i);
      UInt64 a; bool w;
      if (gen == 0) {
        a = ((UInt64)t << 26) + ((z & ((1ull << lines_log2) - 1)) << 6);
        w = ((z >> 32) % 3) == 0;
      } else {
        UInt32 sel = (UInt32)((z >> 60) & 3);
        if (sel == 0) a = ((UInt64)t << 26) + (((z >> 8) & 63) << 6);                   // hot lines
        else if (sel == 1) a = ((UInt64)t << 26) + ((((UInt64)i * 17) & ((1ull << lines_log2) - 1)) << 6);  // stride
        else a = ((UInt64)t << 26) + ((z & ((1ull << lines_log2) - 1)) << 6);
        w = ((z >> 32) & 1) == 0;
      }
      addr_hash[t] = mix64(addr_hash[t] ^ a ^ (w ? 1ull : 0ull));
      IntPtr ev = 0;
      UInt32 r = T.access(a, w, &ev);
      res.push_back((uint8_t)r);
      if (r & R_L2EV) evicted_sum[t] += ev;
    }
    for (int k = 0; k < C_N; ++k) counters.push_back(T.l1.c[k]);
    for (int k = 0; k < C_N; ++k) counters.push_back(T.l2.c[k]);
  }
  char f1[256], f2[256];
  snprintf(f1, sizeof f1, "%s_result.u8", name);
  snprintf(f2, sizeof f2, "%s_counters.u64", name);
  write_bin(f1, res.data(), res.size());
  write_bin(f2, counters.data(), counters.size() * 8);
  char m[1024];
  snprintf(m, sizeof m, "\"%s\": {\"kind\": \"modep\", \"gen\": %d, \"tiles\": %u, \"per_tile\": %u, \"lines_log2\": %u, "
           "\"l1d_size_kb\": %u, \"l1d_assoc\": %u, \"l1d_policy\": \"%s\", \"l2_size_kb\": %u, \"l2_assoc\": %u, "
           "\"l2_policy\": \"%s\", \"result_file\": \"%s\", \"counters_file\": \"%s\", \"evicted_sum\": [",
           name, gen, tiles, per_tile, lines_log2, l1kb, l1a, l1p.c_str(), l2kb, l2a, l2p.c_str(), f1, f2);
  string s(m);
  for (uint32_t t = 0; t < tiles; ++t) { char b[32]; snprintf(b, sizeof b, "%s%llu", t ? ", " : "", (unsigned long long)evicted_sum[t]); s += b; }
  s += "], \"trace_hash\": [";
  for (uint32_t t = 0; t < tiles; ++t) { char b[32]; snprintf(b, sizeof b, "%s%llu", t ? ", " : "", (unsigned long long)addr_hash[t]); s += b; }
  s += "]}";
  manifest(s);
}

int main(int argc, char** argv) {
  CHECK(argc == 2);
  g_dir = argv[1];
  g_manifest = fopen((g_dir + "/manifest.json").c_str(), "w");
  CHECK(g_manifest);
  fprintf(g_manifest, "{\n");

  // 1. the reference KAT, run through the reference IntervalTree/MG1 + restated glue
  {
    RefHistoryTree h(1, 100, true);
    for (int i = 0; i < 10; ++i) CHECK(h.delay(kKat[i][0], kKat[i][1]) == kKat[i][2]);
    manifest("\"htree_kat\": {\"kind\": \"htree_kat\", \"source\": \"tests/unit/history_tree/history_tree.cc:9-20\", "
             "\"rows\": [[10,10,0],[21,10,0],[32,10,0],[43,10,0],[0,1,0],[0,10,53],[45,10,18],[60,4,13],[70,8,7],[75,10,10]]}");
  }
  // 2. randomized history-tree sequences (exercise pruning at max_list_size and M/G/1)
  gen_htree("htree_rand_a", 1, 4000, 64, 9, 100, true);
  gen_htree("htree_rand_b", 2, 4000, 300, 3, 100, true);
  gen_htree("htree_rand_c", 3, 3000, 40, 12, 16, true);
  gen_htree("htree_rand_noan", 4, 3000, 64, 9, 100, false);
  // sparse arrivals grow the history to max_list_size, so the oldest free
  // intervals are pruned and stragglers behind them take the M/G/1 branch
  // (queue_model_history_tree.cc:52-64)
  gen_htree("htree_analytical", 13, 4000, 4000, 9, 16, true, 12);
  gen_htree("htree_analytical8", 14, 4000, 2000, 9, 8, true, 12);
  // 2b. history_list and basic queue models on the same arrival process
  gen_qlist("qlist_rand_a", 1, 4000, 64, 9, 100, true, true);
  gen_qlist("qlist_rand_b", 2, 4000, 300, 3, 100, true, true);
  gen_qlist("qlist_rand_c", 3, 3000, 40, 12, 16, true, true);
  gen_qlist("qlist_noil", 5, 3000, 64, 9, 100, true, false);
  gen_qlist("qlist_noan", 4, 3000, 64, 9, 24, false, true);
  gen_qlist("qlist_small", 10, 3000, 300, 2, 3, true, true);
  gen_qbasic("qbasic_mean", 6, 3000, 64, 9, "arithmetic_mean", 0, 64);
  gen_qbasic("qbasic_mean7", 7, 3000, 300, 12, "arithmetic_mean", 0, 7);
  gen_qbasic("qbasic_median", 8, 3000, 64, 9, "median", 1, 16);
  gen_qbasic("qbasic_none", 9, 3000, 64, 9, "", 2, 64);
  // 3. Cache quartet sequences, L1 (write-through) and L2 (write-back), LRU and round robin
  gen_quartet("quartet_l1_lru", 11, 3000, 2, 4, "lru", 0);
  gen_quartet("quartet_l2_lru", 12, 3000, 4, 8, "lru", 1);
  gen_quartet("quartet_l1_rr", 13, 3000, 2, 4, "round_robin", 0);
  gen_quartet("quartet_l2_rr", 14, 3000, 4, 8, "round_robin", 1);
  // 4. private-mode replays: reference geometry, 16-way L2 (config 5), small caches, RR
  gen_modep("modep_cfg2", 0, 4, 60000, 15, 32, 4, "lru", 512, 8, "lru");
  gen_modep("modep_cfg5", 0, 2, 60000, 15, 32, 4, "lru", 512, 16, "lru");
  gen_modep("modep_mixed", 1, 3, 50000, 13, 32, 4, "lru", 512, 8, "lru");
  gen_modep("modep_small", 1, 3, 40000, 11, 4, 2, "lru", 16, 4, "lru");
  gen_modep("modep_rr", 1, 2, 40000, 12, 8, 4, "round_robin", 64, 8, "round_robin");

  fprintf(g_manifest, "\n}\n");
  fclose(g_manifest);
  printf("ref_harness: fixtures written to %s\n", g_dir.c_str());
  return 0;
}
