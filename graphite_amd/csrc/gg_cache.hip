// gg_cache.hip — private L1-D/L2 cache replay on MI355X (gfx950).
//
// Path: for every line access of a tile, L1CacheCntlr::processMemOpFromCore
// (pr_l1_pr_l2_dram_directory_msi/l1_cache_cntlr.cc:89-180) with the private
// L2CacheCntlr (l2_cache_cntlr.cc:74-527) and the directory granting each
// request (dram_directory_cntlr.cc:238-380 on an UNCACHED entry), on top of
// Cache::{access,insert}CacheLine / {get,set}CacheLineInfo (cache.cc:84-241),
// CacheSet (cache_set.cc:31-103) and LRU / round-robin replacement
// (lru_replacement_policy.cc:5-50, round_robin_replacement_policy.cc:4-27).
//
// Decomposition (DESIGN.md §Cache kernels): one *unit* = (tile, L1-D set).
// Every L2 set of a tile nests inside one L1-D set when L2 sets >= L1-D sets
// (cache_hash_fn.h:17-18), and every L1<->L2 interaction of an access stays in
// the accessed line's sets, so units evolve independently.  A unit is one
// lane: its L1-D set lives in VGPRs, its S2 L2 sets (S2*A2 = 64 lines for the
// reference geometries) live in LDS laid out [line][lane] (conflict-free
// ds_read_b32), and its records arrive through a stable per-tile partition of
// the program-order trace (k_shard_*).
#include "gg_internal.h"

#include <algorithm>
#include <cstring>

namespace {

constexpr uint32_t kChunk = 4096;        // records per shard chunk (one wave)
constexpr uint64_t kB7 = 0x8080808080808080ull;
constexpr uint64_t k7F = 0x7F7F7F7F7F7F7F7Full;
constexpr uint64_t k1F = 0x1F1F1F1F1F1F1F1Full;
constexpr uint64_t k01 = 0x0101010101010101ull;

// cache-counter indices
enum { ACC = GG_CC_ACCESSES, MISS = GG_CC_MISSES, RACC = GG_CC_READ_ACCESSES, RMISS = GG_CC_READ_MISSES,
       WACC = GG_CC_WRITE_ACCESSES, WMISS = GG_CC_WRITE_MISSES, EV = GG_CC_EVICTIONS,
       DEV = GG_CC_DIRTY_EVICTIONS, TR = GG_CC_TAG_READS, TW = GG_CC_TAG_WRITES,
       DR = GG_CC_DATA_READS, DW = GG_CC_DATA_WRITES, NC = GG_NUM_CACHE_COUNTERS };

// ---------------------------------------------------------------------------
// SWAR helpers on packed meta words (8 ways per u64, one byte per way)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ages_of(uint64_t m) { return (m >> 3) & k1F; }
// bit 7 of byte i set iff byte i of x == 0 (exact, no borrow leakage)
__device__ __forceinline__ uint64_t zero_bytes(uint64_t x) { return ~(((x & k7F) + k7F) | x | k7F); }

// LRUReplacementPolicy::update (lru_replacement_policy.cc:40-50) on one meta
// word: every age below `acc` is incremented, then the accessed way's age := 0.
// Bytes beyond the associativity carry age 31 and never move.
__device__ __forceinline__ uint64_t lru_bump(uint64_t m, uint32_t acc)
{
  uint64_t x = (ages_of(m) | kB7) - (k01 * acc);   // bit 7 set iff age >= acc
  uint64_t lt = (~x) & kB7;                         // ages < acc
  return m + ((lt >> 7) << 3);
}
__device__ __forceinline__ uint64_t clear_age(uint64_t m, uint32_t byte) { return m & ~(0xF8ull << (8 * byte)); }

// Byte w of a register-resident meta array; the word is picked with selects
// (no runtime register indexing, which would spill to scratch).
template <int MW>
__device__ __forceinline__ uint32_t meta_byte_t(const uint64_t* mw, uint32_t w)
{
  uint64_t v = mw[0];
#pragma unroll
  for (int k = 1; k < MW; ++k) if ((w >> 3) == (uint32_t)k) v = mw[k];
  return (uint32_t)(v >> (8 * (w & 7))) & 0xFFu;
}
template <int MW>
__device__ __forceinline__ void meta_set_byte_t(uint64_t* mw, uint32_t w, uint32_t b)
{
  const uint32_t sh = 8 * (w & 7);
#pragma unroll
  for (int k = 0; k < MW; ++k)
    if ((w >> 3) == (uint32_t)k) mw[k] = (mw[k] & ~(0xFFull << sh)) | ((uint64_t)(b & 0xFFu) << sh);
}
__device__ __forceinline__ uint32_t meta_byte(const uint64_t* mw, uint32_t w) { return meta_byte_t<1>(mw, w); }
__device__ __forceinline__ void meta_set_byte(uint64_t* mw, uint32_t w, uint32_t b) { meta_set_byte_t<1>(mw, w, b); }

template <int MW>
__device__ __forceinline__ void lru_update(uint64_t* mw, uint32_t way)
{
  const uint32_t acc = GG_M_AGE(meta_byte_t<MW>(mw, way));
#pragma unroll
  for (int k = 0; k < MW; ++k) {
    mw[k] = lru_bump(mw[k], acc);
    if ((way >> 3) == (uint32_t)k) mw[k] = clear_age(mw[k], way & 7);
  }
}

// LRUReplacementPolicy::getReplacementWay (lru_replacement_policy.cc:23-38):
// first invalid way, else the (last) way whose age == assoc-1; -1 if none.
template <int A, int MW>
__device__ __forceinline__ int lru_victim(uint32_t inv_mask, const uint64_t* mw)
{
  if (inv_mask) return __builtin_ctz(inv_mask);
  int way = -1;
#pragma unroll
  for (int k = 0; k < MW; ++k) {
    uint64_t z = zero_bytes(ages_of(mw[k]) ^ (k01 * (uint64_t)(A - 1)));
    if (z) way = k * 8 + (63 - __builtin_clzll(z)) / 8;
  }
  return way;
}

__device__ __forceinline__ uint32_t ms_to_cstate(uint32_t st) { return st == GG_MS_M ? GG_CSTATE_MODIFIED : (st == GG_MS_S ? GG_CSTATE_SHARED : GG_CSTATE_INVALID); }

// ---------------------------------------------------------------------------
// Storage views of the L2 sets of one unit: LDS (replay) or HBM (quartet).
// ---------------------------------------------------------------------------
template <int A2>
struct L2Lds {
  static constexpr int MW = (A2 + 7) / 8;
  uint32_t* T;   // [s*A2 + w][64]
  uint64_t* M;   // [(s*64 + lane)*MW + k]
  uint8_t*  R;   // [s][64]
  uint32_t lane;
  __device__ uint32_t tag(uint32_t s, uint32_t w) const { return T[(s * A2 + w) * GG_WAVE + lane]; }
  __device__ void set_tag(uint32_t s, uint32_t w, uint32_t v) { T[(s * A2 + w) * GG_WAVE + lane] = v; }
  __device__ uint64_t meta(uint32_t s, uint32_t k) const { return M[(s * GG_WAVE + lane) * MW + k]; }
  __device__ void set_meta(uint32_t s, uint32_t k, uint64_t v) { M[(s * GG_WAVE + lane) * MW + k] = v; }
  __device__ uint32_t rr(uint32_t s) const { return R[s * GG_WAVE + lane]; }
  __device__ void set_rr(uint32_t s, uint32_t v) { R[s * GG_WAVE + lane] = (uint8_t)v; }
};

template <int A2>
struct L2Hbm {
  static constexpr int MW = (A2 + 7) / 8;
  gg_cache_state cs; uint64_t units, u;
  __device__ uint32_t tag(uint32_t s, uint32_t w) const { return cs.l2_tag[(uint64_t)(s * A2 + w) * units + u]; }
  __device__ void set_tag(uint32_t s, uint32_t w, uint32_t v) { cs.l2_tag[(uint64_t)(s * A2 + w) * units + u] = v; }
  __device__ uint64_t meta(uint32_t s, uint32_t k) const { return cs.l2_meta[(uint64_t)(s * MW + k) * units + u]; }
  __device__ void set_meta(uint32_t s, uint32_t k, uint64_t v) { cs.l2_meta[(uint64_t)(s * MW + k) * units + u] = v; }
  __device__ uint32_t rr(uint32_t s) const { return cs.l2_rr[(uint64_t)s * units + u]; }
  __device__ void set_rr(uint32_t s, uint32_t v) { cs.l2_rr[(uint64_t)s * units + u] = (uint8_t)v; }
};

// ---------------------------------------------------------------------------
// One unit (tile, L1-D set): L1-D set in registers + its L2 sets in a store.
// ---------------------------------------------------------------------------
template <int A1, int A2, class Store>
struct Unit {
  static constexpr int MW = (A2 + 7) / 8;
  uint64_t t1[A1];        // L1-D line numbers (~0 = invalid)
  uint64_t m1;            // L1-D meta bytes
  uint32_t rr1;           // L1-D round-robin index
  uint32_t c1[NC], c2[NC];
  uint32_t err;
  Store st;
  uint32_t l1set, log_u1, s2, log_l2, pol1, pol2;

  // ---- L1-D (Cache "L1-D", WRITE_THROUGH: l1_cache_cntlr.cc:55-71) ----
  __device__ int l1_find(uint64_t line) const
  {
    int w1 = -1;   // CacheSet::find scans high -> low; tags are unique
#pragma unroll
    for (int w = 0; w < A1; ++w) if (t1[w] == line) w1 = w;
    return w1;
  }
  __device__ void l1_policy_update(uint32_t way) { if (pol1 == GG_POLICY_LRU) lru_update<1>(&m1, way); }

  // L1CacheCntlr::invalidateCacheLine (l1_cache_cntlr.cc:293-305)
  __device__ bool l1_invalidate(uint64_t line)
  {
    c1[TR]++;
    const int w = l1_find(line);
    if (w < 0) return false;
#pragma unroll
    for (int k = 0; k < A1; ++k) if (k == w) t1[k] = GG_L1_INV_TAG;
    uint64_t mw = m1; meta_set_byte(&mw, (uint32_t)w, meta_byte(&mw, (uint32_t)w) & ~7u); m1 = mw;
    c1[TW]++;
    return true;
  }

  // ---- L2 (Cache "L2", WRITE_BACK) ----
  __device__ uint32_t l2_set_of(uint64_t line) const { return (uint32_t)(line >> log_u1) & (s2 - 1); }
  __device__ uint32_t l2_tag_of(uint64_t line) const { return (uint32_t)(line >> log_l2); }
  __device__ uint64_t l2_line_of(uint32_t s, uint32_t tag) const
  {
    return ((uint64_t)tag << log_l2) | ((uint64_t)s << log_u1) | l1set;
  }
  __device__ int l2_find(uint32_t s, uint32_t tag) const
  {
    int w2 = -1;
#pragma unroll
    for (int w = 0; w < A2; ++w) if (st.tag(s, w) == tag) w2 = w;
    return w2;
  }
  __device__ void l2_policy_update(uint32_t s, uint32_t way)
  {
    if (pol2 != GG_POLICY_LRU) return;
    uint64_t mw[MW];
#pragma unroll
    for (int k = 0; k < MW; ++k) mw[k] = st.meta(s, k);
    lru_update<MW>(mw, way);
#pragma unroll
    for (int k = 0; k < MW; ++k) st.set_meta(s, k, mw[k]);
  }
  // Cache::accessCacheLine on L2 (cache.cc:84-112)
  __device__ void l2_access(uint64_t line, bool store)
  {
    const uint32_t s = l2_set_of(line);
    const int w = l2_find(s, l2_tag_of(line));
    if (w < 0) { err |= GG_DERR_STATE; return; }
    l2_policy_update(s, (uint32_t)w);
    c2[DW] += store ? 1u : 0u; c2[DR] += store ? 0u : 1u;
  }
  __device__ void l2_set_meta_byte(uint32_t s, uint32_t w, uint32_t b)
  {
    uint64_t v = st.meta(s, w >> 3);
    const uint32_t sh = 8 * (w & 7);
    v = (v & ~(0xFFull << sh)) | ((uint64_t)b << sh);
    st.set_meta(s, w >> 3, v);
  }
  __device__ uint32_t l2_meta_byte(uint32_t s, uint32_t w) const { return (uint32_t)(st.meta(s, w >> 3) >> (8 * (w & 7))) & 0xFFu; }

  // L2CacheCntlr::insertCacheLineInL1 (l2_cache_cntlr.cc:133-165)
  __device__ void insert_in_l1(uint64_t line, uint32_t ms, uint32_t& res, int& way_out)
  {
    int v;
    if (pol1 == GG_POLICY_LRU) {
      uint32_t inv = 0;
#pragma unroll
      for (int w = 0; w < A1; ++w) inv |= (t1[w] == GG_L1_INV_TAG ? 1u : 0u) << w;
      v = lru_victim<A1, 1>(inv, &m1);
    } else {
      v = (int)rr1;
      rr1 = (rr1 == 0) ? (A1 - 1) : (rr1 - 1);
    }
    if (v < 0) { err |= GG_DERR_STATE; v = 0; }
    uint64_t ev_line = GG_L1_INV_TAG;
#pragma unroll
    for (int w = 0; w < A1; ++w) if (w == v) { ev_line = t1[w]; t1[w] = line; }
    uint64_t mw = m1;
    const uint32_t old = meta_byte(&mw, (uint32_t)v);
    meta_set_byte(&mw, (uint32_t)v, (old & ~7u) | ms);
    m1 = mw;
    l1_policy_update((uint32_t)v);
    // Cache::insertCacheLine counters (cache.cc:151-180), WRITE_THROUGH: no dirty evictions
    if (ev_line != GG_L1_INV_TAG) { c1[TR]++; c1[DR]++; c1[EV]++; }
    else c1[TR]++;
    c1[TW]++; c1[DW]++;
    way_out = v;
    if (ev_line != GG_L1_INV_TAG) {
      res |= GG_RES_L1_EVICT;
      // clear the L2 line's cached_loc (getCacheLineInfo + setCacheLineInfo)
      const uint32_t s = l2_set_of(ev_line);
      c2[TR]++;
      const int w = l2_find(s, l2_tag_of(ev_line));
      if (w < 0) { err |= GG_DERR_STATE; return; }
      const uint32_t b = l2_meta_byte(s, (uint32_t)w);
      if (!GG_M_LOC(b)) err |= GG_DERR_STATE;   // LOG_ASSERT_ERROR (l2_cache_cntlr.cc:152-157)
      l2_set_meta_byte(s, (uint32_t)w, b & ~4u);
      c2[TW]++;
    }
  }

  // Cache::updateMissCounters (cache.cc:321-360)
  __device__ static void miss_counters(uint32_t* c, bool wr, bool miss)
  {
    const uint32_t w = wr ? 1u : 0u, r = 1u - w, m = miss ? 1u : 0u;
    c[ACC]++; c[WACC] += w; c[RACC] += r;
    c[MISS] += m; c[WMISS] += m & w; c[RMISS] += m & r;
  }

  // L1CacheCntlr::processMemOpFromCore, private mode.  Returns GG_RES_* flags;
  // *ev = byte address of the L2 victim (or ~0).
  __device__ uint32_t access(uint64_t line, bool wr, uint64_t* ev_line)
  {
    uint32_t res = 0;
    *ev_line = ~0ull;
    // access_num == 1: operationPermissibleinL1Cache (l1:207-243)
    c1[TR]++;
    int w1 = l1_find(line);
    const uint32_t s1 = (w1 >= 0) ? GG_M_STATE(meta_byte(&m1, (uint32_t)w1)) : GG_MS_I;
    const bool hit1 = wr ? (s1 == GG_MS_M) : (s1 != GG_MS_I);
    miss_counters(c1, wr, !hit1);
    if (hit1) {
      l1_policy_update((uint32_t)w1);          // accessCache -> accessCacheLine
      c1[DW] += wr ? 1u : 0u; c1[DR] += wr ? 0u : 1u;
      if (wr) l2_access(line, true);           // write-through (L2CacheCntlr::writeCacheLine)
      return res;
    }
    l1_invalidate(line);                       // l1:135-137

    // L2CacheCntlr::processShmemRequestFromL1Cache (l2:180-224)
    const uint32_t s = l2_set_of(line), tag2 = l2_tag_of(line);
    uint32_t tags[A2];
#pragma unroll
    for (int w = 0; w < A2; ++w) tags[w] = st.tag(s, w);
    uint64_t mw[MW];
#pragma unroll
    for (int k = 0; k < MW; ++k) mw[k] = st.meta(s, k);
    int w2 = -1;
#pragma unroll
    for (int w = 0; w < A2; ++w) if (tags[w] == tag2) w2 = w;
    c2[TR]++;
    const uint32_t b2 = (w2 >= 0) ? meta_byte_t<MW>(mw, (uint32_t)w2) : 0u;
    const uint32_t s2st = GG_M_STATE(b2);
    const bool hit2 = wr ? (s2st == GG_MS_M) : (s2st != GG_MS_I);
    miss_counters(c2, wr, !hit2);

    if (hit2) {
      res |= GG_RES_L2_HIT;
      if (pol2 == GG_POLICY_LRU) lru_update<MW>(mw, (uint32_t)w2);   // readCacheLine
      c2[DR]++;
#pragma unroll
      for (int k = 0; k < MW; ++k) st.set_meta(s, k, mw[k]);
      int v1;
      insert_in_l1(line, s2st, res, v1);
      // setCachedLoc / setForcedCachedLoc(L1_DCACHE) + setCacheLineInfo
      l2_set_meta_byte(s, (uint32_t)w2, l2_meta_byte(s, (uint32_t)w2) | 4u);
      c2[TW]++;
      l1_policy_update((uint32_t)v1);          // accessCache (l1:145-159)
      c1[DW] += wr ? 1u : 0u; c1[DR] += wr ? 0u : 1u;
      if (wr) l2_access(line, true);
      return res;
    }

    // L2 miss -> directory (handleMsgFromL1Cache, l2:226-258)
    res |= GG_RES_DIRECTORY;
    uint32_t ns;
    uint32_t inv = 0;
#pragma unroll
    for (int w = 0; w < A2; ++w) inv |= (tags[w] == GG_L2_INV_TAG ? 1u : 0u) << w;
    if (wr) {                                  // processExReqFromL1Cache (l2:260-282)
      c2[TR]++;
      if (s2st == GG_MS_S) {
        // PrL2CacheLineInfo::invalidate + setCacheLineInfo: tag ~0, state I, loc I; age kept
#pragma unroll
        for (int w = 0; w < A2; ++w) if (w == w2) tags[w] = GG_L2_INV_TAG;
        st.set_tag(s, (uint32_t)w2, GG_L2_INV_TAG);
        meta_set_byte_t<MW>(mw, (uint32_t)w2, b2 & ~7u);
        inv |= 1u << w2;
        c2[TW]++;
        res |= GG_RES_UPGRADE;
      } else if (s2st != GG_MS_I) err |= GG_DERR_STATE;
      ns = GG_MS_M;
    } else {
      ns = GG_MS_S;
    }
    // insertCacheLineInHierarchy (l2:167-178) -> L2CacheCntlr::insertCacheLine (l2:74-116)
    int v2;
    if (pol2 == GG_POLICY_LRU) v2 = lru_victim<A2, MW>(inv, mw);
    else { v2 = (int)st.rr(s); st.set_rr(s, v2 == 0 ? (A2 - 1) : (v2 - 1)); }
    if (v2 < 0) { err |= GG_DERR_STATE; v2 = 0; }
    uint32_t vt = 0;
#pragma unroll
    for (int w = 0; w < A2; ++w) if (w == v2) vt = tags[w];
    const uint32_t vb = meta_byte_t<MW>(mw, (uint32_t)v2);
    if (vt != GG_L2_INV_TAG) {
      const uint64_t e = l2_line_of(s, vt);
      *ev_line = e;
      c2[TR]++; c2[DR]++; c2[EV]++;
      res |= GG_RES_L2_EVICT;
      if (GG_M_STATE(vb) == GG_MS_M) { c2[DEV]++; res |= GG_RES_L2_EVICT_DIRTY; }   // FLUSH_REP
      else if (GG_M_STATE(vb) != GG_MS_S) err |= GG_DERR_STATE;                       // INV_REP
      if (GG_M_LOC(vb)) {                      // invalidateCacheLineInL1 (l2:124-131)
        if (l1_invalidate(e)) res |= GG_RES_L2_EVICT_INV_L1;
      }
    } else {
      c2[TR]++;
    }
    c2[TW]++; c2[DW]++;
    st.set_tag(s, (uint32_t)v2, tag2);
    meta_set_byte_t<MW>(mw, (uint32_t)v2, (vb & ~7u) | ns | 4u);   // state, cached_loc = L1-D
    if (pol2 == GG_POLICY_LRU) lru_update<MW>(mw, (uint32_t)v2);
#pragma unroll
    for (int k = 0; k < MW; ++k) st.set_meta(s, k, mw[k]);
    int v1;
    insert_in_l1(line, ns, res, v1);           // insertCacheLineInL1
    // access_num == 2: the retry hits (no miss counters)
    c1[TR]++;
    l1_policy_update((uint32_t)v1);
    c1[DW] += wr ? 1u : 0u; c1[DR] += wr ? 0u : 1u;
    if (wr) l2_access(line, true);
    return res;
  }
};

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
__global__ void k_state_reset(gg_cache_state cs, gg_geom g)
{
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= g.units) return;
  uint64_t m1 = 0;
  for (uint32_t w = 0; w < 8; ++w)
    m1 |= (uint64_t)(w < g.a1 ? GG_M_MAKE(GG_MS_I, 0, w) : 0xF8u) << (8 * w);
  for (uint32_t w = 0; w < g.a1; ++w) cs.l1_tag[(uint64_t)w * g.units + u] = GG_L1_INV_TAG;
  cs.l1_meta[u] = m1;
  cs.l1_rr[u] = (uint8_t)(g.a1 - 1);       // round_robin_replacement_policy.cc:4-9
  for (uint32_t s = 0; s < g.s2; ++s) {
    for (uint32_t w = 0; w < g.a2; ++w) cs.l2_tag[(uint64_t)(s * g.a2 + w) * g.units + u] = GG_L2_INV_TAG;
    for (uint32_t k = 0; k < g.mw; ++k) {
      uint64_t m = 0;
      for (uint32_t b = 0; b < 8; ++b) {
        const uint32_t w = k * 8 + b;
        m |= (uint64_t)(w < g.a2 ? GG_M_MAKE(GG_MS_I, 0, w) : 0xF8u) << (8 * b);  // ages = way index
      }
      cs.l2_meta[(uint64_t)(s * g.mw + k) * g.units + u] = m;
    }
    cs.l2_rr[(uint64_t)s * g.units + u] = (uint8_t)(g.a2 - 1);
  }
}

// Pass 1 of the stable (tile, L1-D set) partition: per-chunk set histogram.
__global__ __launch_bounds__(256) void k_shard_hist(const uint64_t* __restrict__ addr,
    const uint32_t* __restrict__ chunk_tile, const uint64_t* __restrict__ chunk_start,
    const uint32_t* __restrict__ chunk_len, uint32_t* __restrict__ cnt, gg_geom g, uint32_t* err)
{
  __shared__ uint32_t h[1024];
  const uint32_t c = blockIdx.x;
  for (uint32_t s = threadIdx.x; s < g.u1; s += blockDim.x) h[s] = 0;
  __syncthreads();
  const uint64_t start = chunk_start[c];
  const uint32_t len = chunk_len[c];
  uint32_t bad = 0;
  for (uint32_t i = threadIdx.x; i < len; i += blockDim.x) {
    const uint64_t a = addr[start + i];
    bad |= (a >= g.addr_limit) ? 1u : 0u;
    atomicAdd(&h[(a >> g.log_line) & (g.u1 - 1)], 1u);
  }
  if (bad) atomicOr(err, GG_DERR_RANGE);
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < g.u1; s += blockDim.x) cnt[(uint64_t)c * g.u1 + s] = h[s];
}

// Pass 2: per tile, exclusive scan over its chunks per set (in place), unit
// lengths, and unit bases = tile offset + exclusive scan over sets.
__global__ void k_shard_scan(uint32_t* __restrict__ cnt, const uint32_t* __restrict__ tile_chunk0,
                             const uint64_t* __restrict__ tile_off, uint32_t* __restrict__ unit_len,
                             uint64_t* __restrict__ unit_base, gg_geom g)
{
  __shared__ uint64_t sc[1024];
  const uint32_t t = blockIdx.x, s = threadIdx.x;
  uint64_t acc = 0;
  if (s < g.u1) {
    for (uint32_t c = tile_chunk0[t]; c < tile_chunk0[t + 1]; ++c) {
      uint32_t* p = &cnt[(uint64_t)c * g.u1 + s];
      const uint32_t v = *p;
      *p = (uint32_t)acc;
      acc += v;
    }
    unit_len[(uint64_t)t * g.u1 + s] = (uint32_t)acc;
  }
  sc[s] = (s < g.u1) ? acc : 0;
  __syncthreads();
  for (uint32_t o = 1; o < blockDim.x; o <<= 1) {
    const uint64_t v = (s >= o) ? sc[s - o] : 0;
    __syncthreads();
    sc[s] += v;
    __syncthreads();
  }
  if (s < g.u1) unit_base[(uint64_t)t * g.u1 + s] = tile_off[t] + sc[s] - acc;
}

// Pass 3: one wave per chunk, 64 records per step in program order; lanes
// with the same set are matched with log2(u1) ballots so the rank of each
// record inside its unit is stable (program order is kept per unit).
__global__ __launch_bounds__(64) void k_shard_scatter(const uint64_t* __restrict__ addr,
    const uint32_t* __restrict__ meta, const uint32_t* __restrict__ chunk_tile,
    const uint64_t* __restrict__ chunk_start, const uint32_t* __restrict__ chunk_len,
    const uint32_t* __restrict__ cnt, const uint64_t* __restrict__ unit_base,
    const uint64_t* __restrict__ tile_off, uint64_t* __restrict__ sh_key,
    uint32_t* __restrict__ sh_idx, gg_geom g)
{
  __shared__ uint64_t base[1024];
  const uint32_t c = blockIdx.x, lane = threadIdx.x;
  const uint32_t t = chunk_tile[c];
  for (uint32_t s = lane; s < g.u1; s += GG_WAVE)
    base[s] = unit_base[(uint64_t)t * g.u1 + s] + cnt[(uint64_t)c * g.u1 + s];
  __syncthreads();
  const uint64_t start = chunk_start[c];
  const uint32_t len = chunk_len[c];
  const uint32_t rel0 = (uint32_t)(start - tile_off[t]);
  const uint64_t lt_mask = (1ull << lane) - 1;
  const uint64_t line_mask = ~((1ull << g.log_line) - 1);
  for (uint32_t i0 = 0; i0 < len; i0 += GG_WAVE) {
    const uint32_t i = i0 + lane;
    const bool valid = i < len;
    const uint64_t a = valid ? addr[start + i] : 0;
    const uint32_t m = valid ? meta[start + i] : 0;
    const uint32_t s = (uint32_t)(a >> g.log_line) & (g.u1 - 1);
    uint64_t peers = __ballot(valid);
    for (uint32_t b = 0; b < g.log_u1; ++b) {
      const bool bit = (s >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const uint32_t rank = __popcll(peers & lt_mask);
    const uint64_t b0 = valid ? base[s] : 0;
    __builtin_amdgcn_wave_barrier();
    if (valid && rank == 0) base[s] = b0 + __popcll(peers);
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      const uint64_t pos = b0 + rank;
      sh_key[pos] = (a & line_mask) | (m & GG_META_WRITE);
      sh_idx[pos] = rel0 + i;
    }
  }
}

// Replay: one lane per unit, 64 units per workgroup (one wave).
template <int A1, int A2>
__global__ __launch_bounds__(64) void k_cache_replay(gg_cache_state cs, gg_geom g,
    const uint64_t* __restrict__ sh_key, const uint32_t* __restrict__ sh_idx,
    const uint32_t* __restrict__ unit_len, const uint64_t* __restrict__ unit_base,
    const uint64_t* __restrict__ tile_off, uint32_t* __restrict__ result,
    uint64_t* __restrict__ evicted, uint32_t* err)
{
  constexpr int MW = (A2 + 7) / 8;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x;
  const uint64_t u = (uint64_t)blockIdx.x * GG_WAVE + lane;
  const bool active = u < g.units;
  const uint64_t uu = active ? u : 0;
  const uint32_t S2 = g.s2;

  Unit<A1, A2, L2Lds<A2>> U;
  U.st.T = reinterpret_cast<uint32_t*>(smem);
  U.st.M = reinterpret_cast<uint64_t*>(smem + (size_t)S2 * A2 * GG_WAVE * 4);
  U.st.R = reinterpret_cast<uint8_t*>(smem + (size_t)S2 * A2 * GG_WAVE * 4 + (size_t)S2 * GG_WAVE * MW * 8);
  U.st.lane = lane;
  U.l1set = (uint32_t)(uu & (g.u1 - 1));
  U.log_u1 = g.log_u1; U.s2 = S2; U.log_l2 = g.log_l2; U.pol1 = g.pol1; U.pol2 = g.pol2;
  U.err = 0;
#pragma unroll
  for (int k = 0; k < NC; ++k) { U.c1[k] = 0; U.c2[k] = 0; }

  // load state (coalesced: [field][unit])
#pragma unroll
  for (int w = 0; w < A1; ++w) U.t1[w] = cs.l1_tag[(uint64_t)w * g.units + uu];
  U.m1 = cs.l1_meta[uu];
  U.rr1 = cs.l1_rr[uu];
  for (uint32_t s = 0; s < S2; ++s) {
#pragma unroll
    for (int w = 0; w < A2; ++w) U.st.set_tag(s, w, cs.l2_tag[(uint64_t)(s * A2 + w) * g.units + uu]);
#pragma unroll
    for (int k = 0; k < MW; ++k) U.st.set_meta(s, k, cs.l2_meta[(uint64_t)(s * MW + k) * g.units + uu]);
    if (g.pol2 != GG_POLICY_LRU) U.st.set_rr(s, cs.l2_rr[(uint64_t)s * g.units + uu]);
  }

  const uint32_t len = active ? unit_len[uu] : 0;
  const uint64_t base = active ? unit_base[uu] : 0;
  const uint32_t tile = (uint32_t)(uu >> g.log_u1);
  const uint64_t rbase = tile_off[tile];
  uint32_t maxlen = len;
  for (int o = 32; o > 0; o >>= 1) maxlen = max(maxlen, (uint32_t)__shfl_xor((int)maxlen, o));

  uint64_t key = (len > 0) ? sh_key[base] : 0;
  uint32_t idx = (len > 0) ? sh_idx[base] : 0;
  for (uint32_t j = 0; j < maxlen; ++j) {
    const bool live = j < len;
    const bool more = j + 1 < len;
    const uint64_t nkey = more ? sh_key[base + j + 1] : 0;
    const uint32_t nidx = more ? sh_idx[base + j + 1] : 0;
    if (live) {
      uint64_t ev;
      const uint32_t r = U.access(key >> g.log_line, (key & 1u) != 0, &ev);
      if (result) result[rbase + idx] = r;
      if (evicted) evicted[rbase + idx] = (ev == ~0ull) ? ~0ull : (ev << g.log_line);
    }
    key = nkey; idx = nidx;
  }

  // store state back
  if (active) {
#pragma unroll
    for (int w = 0; w < A1; ++w) cs.l1_tag[(uint64_t)w * g.units + u] = U.t1[w];
    cs.l1_meta[u] = U.m1;
    cs.l1_rr[u] = (uint8_t)U.rr1;
    for (uint32_t s = 0; s < S2; ++s) {
#pragma unroll
      for (int w = 0; w < A2; ++w) cs.l2_tag[(uint64_t)(s * A2 + w) * g.units + u] = U.st.tag(s, w);
#pragma unroll
      for (int k = 0; k < MW; ++k) cs.l2_meta[(uint64_t)(s * MW + k) * g.units + u] = U.st.meta(s, k);
      if (g.pol2 != GG_POLICY_LRU) cs.l2_rr[(uint64_t)s * g.units + u] = (uint8_t)U.st.rr(s);
    }
  }
  if (U.err) atomicOr(err, U.err);

  // counters: all 64 lanes of the wave belong to one tile when u1 % 64 == 0
  uint64_t* ctr = cs.counters + (uint64_t)tile * 2 * NC;
  if ((g.u1 & (GG_WAVE - 1)) == 0) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      uint32_t a = U.c1[k], b = U.c2[k];
      for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o); b += __shfl_xor(b, o); }
      if (lane == 0) { if (a) atomicAdd((unsigned long long*)&ctr[k], a); if (b) atomicAdd((unsigned long long*)&ctr[NC + k], b); }
    }
  } else if (active) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      if (U.c1[k]) atomicAdd((unsigned long long*)&ctr[k], U.c1[k]);
      if (U.c2[k]) atomicAdd((unsigned long long*)&ctr[NC + k], U.c2[k]);
    }
  }
}

// ---------------------------------------------------------------------------
// Quartet (Cache::{get,set}CacheLineInfo, accessCacheLine, insertCacheLine)
// on one tile's HBM-resident state.  Single thread; slow path.
// ---------------------------------------------------------------------------
struct QuartetIO {
  int op, level;
  uint32_t tile;
  uint64_t addr;
  gg_line_info in, out;
  int eviction;
  uint64_t ev_addr;
  int status;
};

template <int A1, int A2>
__global__ void k_quartet(gg_cache_state cs, gg_geom g, QuartetIO* io)
{
  constexpr int MW = (A2 + 7) / 8;
  QuartetIO q = *io;
  const uint64_t line = q.addr >> g.log_line;
  const uint64_t u = (uint64_t)q.tile * g.u1 + (line & (g.u1 - 1));
  uint64_t* ctr = cs.counters + ((uint64_t)q.tile * 2 + (q.level == GG_L1D ? 0 : 1)) * NC;
  q.status = GG_OK;
  auto cstate_to_ms = [](uint32_t c, int* ok) -> uint32_t {
    if (c == GG_CSTATE_INVALID) return GG_MS_I;
    if (c == GG_CSTATE_SHARED) return GG_MS_S;
    if (c == GG_CSTATE_MODIFIED) return GG_MS_M;
    *ok = 0; return 0;
  };
  int ok = 1;
  if (q.level == GG_L1D) {
    uint64_t t1[A1];
    for (int w = 0; w < A1; ++w) t1[w] = cs.l1_tag[(uint64_t)w * g.units + u];
    uint64_t m1 = cs.l1_meta[u];
    int wf = -1;
    for (int w = A1 - 1; w >= 0; --w) if (t1[w] == line) { wf = w; break; }
    if (q.op == 0) {                                  // getCacheLineInfo
      if (wf >= 0) { q.out.tag = line; q.out.cstate = ms_to_cstate(GG_M_STATE(meta_byte(&m1, wf))); q.out.cached_loc = 0; }
      atomicAdd((unsigned long long*)&ctr[TR], 1ull);
    } else if (q.op == 1) {                           // setCacheLineInfo
      if (wf < 0) q.status = GG_ERR_STATE;
      else if (q.in.tag != ~0ull && q.in.tag != line) q.status = GG_ERR_UNSUPPORTED;
      else {
        uint32_t ms = cstate_to_ms(q.in.cstate, &ok);
        if (!ok) q.status = GG_ERR_UNSUPPORTED;
        else {
          cs.l1_tag[(uint64_t)wf * g.units + u] = q.in.tag;
          meta_set_byte(&m1, wf, (meta_byte(&m1, wf) & ~7u) | ms);
          cs.l1_meta[u] = m1;
          atomicAdd((unsigned long long*)&ctr[TW], 1ull);
        }
      }
    } else if (q.op == 2 || q.op == 3) {              // accessCacheLine
      if (wf < 0) q.status = GG_ERR_STATE;
      else {
        if (g.pol1 == GG_POLICY_LRU) lru_update<1>(&m1, wf);
        cs.l1_meta[u] = m1;
        atomicAdd((unsigned long long*)&ctr[q.op == 3 ? DW : DR], 1ull);
      }
    } else {                                          // insertCacheLine
      uint32_t ms = cstate_to_ms(q.in.cstate, &ok);
      if (!ok || q.in.tag != line) q.status = GG_ERR_UNSUPPORTED;
      else {
        int v;
        if (g.pol1 == GG_POLICY_LRU) {
          uint32_t inv = 0;
          for (int w = 0; w < A1; ++w) inv |= (t1[w] == GG_L1_INV_TAG ? 1u : 0u) << w;
          v = lru_victim<A1, 1>(inv, &m1);
        } else {
          uint32_t r = cs.l1_rr[u]; v = (int)r; cs.l1_rr[u] = (uint8_t)(r == 0 ? A1 - 1 : r - 1);
        }
        if (v < 0) q.status = GG_ERR_STATE;
        else {
          q.eviction = t1[v] != GG_L1_INV_TAG;
          if (q.eviction) { q.out.tag = t1[v]; q.out.cstate = ms_to_cstate(GG_M_STATE(meta_byte(&m1, v))); q.out.cached_loc = 0; }
          q.ev_addr = q.out.tag << g.log_line;
          cs.l1_tag[(uint64_t)v * g.units + u] = line;
          meta_set_byte(&m1, v, (meta_byte(&m1, v) & ~7u) | ms);
          if (g.pol1 == GG_POLICY_LRU) lru_update<1>(&m1, v);
          cs.l1_meta[u] = m1;
          if (q.eviction) { ctr[TR]++; ctr[DR]++; ctr[EV]++; } else ctr[TR]++;
          ctr[TW]++; ctr[DW]++;
        }
      }
    }
  } else {
    L2Hbm<A2> st{cs, g.units, u};
    const uint32_t s = (uint32_t)(line >> g.log_u1) & (g.s2 - 1);
    const uint32_t tag2 = (uint32_t)(line >> g.log_l2);
    const uint32_t l1set = (uint32_t)(line & (g.u1 - 1));
    int wf = -1;
    for (int w = A2 - 1; w >= 0; --w) if (st.tag(s, w) == tag2) { wf = w; break; }
    uint64_t mw[MW];
    for (int k = 0; k < MW; ++k) mw[k] = st.meta(s, k);
    if (q.op == 0) {
      if (wf >= 0) {
        const uint32_t b = meta_byte_t<MW>(mw, wf);
        q.out.tag = line; q.out.cstate = ms_to_cstate(GG_M_STATE(b)); q.out.cached_loc = GG_M_LOC(b) ? GG_LOC_L1D : GG_LOC_INVALID;
      }
      ctr[TR]++;
    } else if (q.op == 1) {
      if (wf < 0) q.status = GG_ERR_STATE;
      else if (q.in.tag != ~0ull && q.in.tag != line) q.status = GG_ERR_UNSUPPORTED;
      else {
        uint32_t ms = cstate_to_ms(q.in.cstate, &ok);
        if (!ok || (q.in.cached_loc != GG_LOC_INVALID && q.in.cached_loc != GG_LOC_L1D)) q.status = GG_ERR_UNSUPPORTED;
        else {
          st.set_tag(s, wf, q.in.tag == ~0ull ? GG_L2_INV_TAG : tag2);
          meta_set_byte_t<MW>(mw, wf, (meta_byte_t<MW>(mw, wf) & ~7u) | ms | (q.in.cached_loc == GG_LOC_L1D ? 4u : 0u));
          for (int k = 0; k < MW; ++k) st.set_meta(s, k, mw[k]);
          ctr[TW]++;
        }
      }
    } else if (q.op == 2 || q.op == 3) {
      if (wf < 0) q.status = GG_ERR_STATE;
      else {
        if (g.pol2 == GG_POLICY_LRU) lru_update<MW>(mw, wf);
        for (int k = 0; k < MW; ++k) st.set_meta(s, k, mw[k]);
        ctr[q.op == 3 ? DW : DR]++;
      }
    } else {
      uint32_t ms = cstate_to_ms(q.in.cstate, &ok);
      if (!ok || q.in.tag != line || (q.in.cached_loc != GG_LOC_INVALID && q.in.cached_loc != GG_LOC_L1D))
        q.status = GG_ERR_UNSUPPORTED;
      else {
        int v;
        if (g.pol2 == GG_POLICY_LRU) {
          uint32_t inv = 0;
          for (int w = 0; w < A2; ++w) inv |= (st.tag(s, w) == GG_L2_INV_TAG ? 1u : 0u) << w;
          v = lru_victim<A2, MW>(inv, mw);
        } else {
          uint32_t r = st.rr(s); v = (int)r; st.set_rr(s, r == 0 ? A2 - 1 : r - 1);
        }
        if (v < 0) q.status = GG_ERR_STATE;
        else {
          const uint32_t vt = st.tag(s, v);
          const uint32_t vb = meta_byte_t<MW>(mw, v);
          q.eviction = vt != GG_L2_INV_TAG;
          if (q.eviction) {
            q.out.tag = ((uint64_t)vt << g.log_l2) | ((uint64_t)s << g.log_u1) | l1set;
            q.out.cstate = ms_to_cstate(GG_M_STATE(vb));
            q.out.cached_loc = GG_M_LOC(vb) ? GG_LOC_L1D : GG_LOC_INVALID;
          }
          q.ev_addr = q.out.tag << g.log_line;
          st.set_tag(s, v, tag2);
          meta_set_byte_t<MW>(mw, v, (vb & ~7u) | ms | (q.in.cached_loc == GG_LOC_L1D ? 4u : 0u));
          if (g.pol2 == GG_POLICY_LRU) lru_update<MW>(mw, v);
          for (int k = 0; k < MW; ++k) st.set_meta(s, k, mw[k]);
          if (q.eviction) { ctr[TR]++; ctr[DR]++; ctr[EV]++; if (GG_M_STATE(vb) == GG_MS_M) ctr[DEV]++; }
          else ctr[TR]++;
          ctr[TW]++; ctr[DW]++;
        }
      }
    }
  }
  *io = q;
}

// ---------------------------------------------------------------------------
// dispatch over the instantiated geometries
// ---------------------------------------------------------------------------
typedef void (*replay_fn)(gg_cache_state, gg_geom, const uint64_t*, const uint32_t*, const uint32_t*,
                          const uint64_t*, const uint64_t*, uint32_t*, uint64_t*, uint32_t*);
typedef void (*quartet_fn)(gg_cache_state, gg_geom, QuartetIO*);

struct Kern { int a1, a2; replay_fn replay; quartet_fn quartet; };

#define GG_KERN(A1, A2) { A1, A2, k_cache_replay<A1, A2>, k_quartet<A1, A2> }
const Kern kKernels[] = {
  GG_KERN(4, 8), GG_KERN(4, 16), GG_KERN(4, 4),
  GG_KERN(2, 4), GG_KERN(2, 8), GG_KERN(2, 16),
  GG_KERN(8, 8), GG_KERN(8, 16), GG_KERN(8, 4),
  GG_KERN(1, 8), GG_KERN(4, 2), GG_KERN(4, 32),
};

const Kern* find_kernel(uint32_t a1, uint32_t a2)
{
  for (const Kern& k : kKernels) if ((uint32_t)k.a1 == a1 && (uint32_t)k.a2 == a2) return &k;
  return nullptr;
}

size_t replay_lds_bytes(const gg_geom& g)
{
  return (size_t)g.s2 * g.a2 * GG_WAVE * 4 + (size_t)g.s2 * GG_WAVE * g.mw * 8 +
         (g.pol2 == GG_POLICY_LRU ? 0 : (size_t)g.s2 * GG_WAVE);
}

template <class T>
gg_status grow(T** p, uint64_t* cap, uint64_t need)
{
  if (need <= *cap && *p) return GG_OK;
  if (*p) { hipFree(*p); *p = nullptr; }
  uint64_t n = std::max<uint64_t>(need, 1) + need / 8;
  GG_HIP(hipMalloc((void**)p, n * sizeof(T)));
  *cap = n;
  return GG_OK;
}

}  // namespace

gg_status gg_cache_state_alloc(gg_ctx* ctx)
{
  gg_geom& g = ctx->g;
  gg_cache_state& cs = ctx->cs;
  if (!find_kernel(g.a1, g.a2))
    return gg_fail(GG_ERR_UNSUPPORTED, "no replay kernel instantiated for L1-D assoc %u / L2 assoc %u", g.a1, g.a2);
  if (replay_lds_bytes(g) > 64 * 1024)
    return gg_fail(GG_ERR_UNSUPPORTED, "L2 lines per L1-D set (%u) too large for the LDS-resident replay", g.s2 * g.a2);
  GG_HIP(hipMalloc((void**)&cs.l1_tag, sizeof(uint64_t) * g.a1 * g.units));
  GG_HIP(hipMalloc((void**)&cs.l1_meta, sizeof(uint64_t) * g.units));
  GG_HIP(hipMalloc((void**)&cs.l1_rr, g.units));
  GG_HIP(hipMalloc((void**)&cs.l2_tag, sizeof(uint32_t) * g.s2 * g.a2 * g.units));
  GG_HIP(hipMalloc((void**)&cs.l2_meta, sizeof(uint64_t) * g.s2 * g.mw * g.units));
  GG_HIP(hipMalloc((void**)&cs.l2_rr, (size_t)g.s2 * g.units));
  GG_HIP(hipMalloc((void**)&cs.counters, sizeof(uint64_t) * g.tiles * 2 * GG_NUM_CACHE_COUNTERS));
  GG_HIP(hipMalloc((void**)&ctx->unit_len, sizeof(uint32_t) * g.units));
  GG_HIP(hipMalloc((void**)&ctx->unit_base, sizeof(uint64_t) * g.units));
  GG_HIP(hipMalloc((void**)&ctx->tile_off_dev, sizeof(uint64_t) * (g.tiles + 1)));
  return GG_OK;
}

void gg_cache_state_free(gg_ctx* ctx)
{
  gg_cache_state& cs = ctx->cs;
  void* ps[] = {cs.l1_tag, cs.l1_meta, cs.l1_rr, cs.l2_tag, cs.l2_meta, cs.l2_rr, cs.counters,
                ctx->sh_key, ctx->sh_idx, ctx->chunk_cnt, ctx->chunk_tile, ctx->chunk_start,
                ctx->chunk_len, ctx->unit_len, ctx->unit_base, ctx->tile_off_dev};
  for (void* p : ps) if (p) hipFree(p);
}

gg_status gg_cache_state_reset(gg_ctx* ctx, hipStream_t s)
{
  const gg_geom& g = ctx->g;
  const uint32_t blocks = (uint32_t)((g.units + 255) / 256);
  hipLaunchKernelGGL(k_state_reset, dim3(blocks), dim3(256), 0, s, ctx->cs, g);
  GG_HIP(hipGetLastError());
  GG_HIP(hipMemsetAsync(ctx->cs.counters, 0, sizeof(uint64_t) * g.tiles * 2 * GG_NUM_CACHE_COUNTERS, s));
  return GG_OK;
}

gg_status gg_cache_run_batch(gg_ctx* ctx, const gg_trace* tr, uint32_t* result, uint64_t* evicted, hipStream_t s)
{
  const gg_geom& g = ctx->g;
  if (!tr || !tr->tile_offsets) return gg_fail(GG_ERR_INVALID, "trace / tile_offsets is NULL");
  if (tr->tile_offsets[0] != 0 || tr->tile_offsets[g.tiles] != tr->num_records)
    return gg_fail(GG_ERR_INVALID, "tile_offsets must run from 0 to num_records");
  if (tr->num_records && (!tr->addr_dev || !tr->meta_dev)) return gg_fail(GG_ERR_INVALID, "addr/meta device pointers are NULL");
  // chunk table (host) — chunks never straddle tiles
  ctx->h_chunk_tile.clear(); ctx->h_chunk_start.clear(); ctx->h_chunk_len.clear();
  std::vector<uint32_t> tile_chunk0(g.tiles + 1);
  for (uint32_t t = 0; t < g.tiles; ++t) {
    const uint64_t b = tr->tile_offsets[t], e = tr->tile_offsets[t + 1];
    if (e < b) return gg_fail(GG_ERR_INVALID, "tile_offsets not monotonic at tile %u", t);
    if (e - b >= (1ull << 32)) return gg_fail(GG_ERR_RANGE, "tile %u has >= 2^32 records in one batch", t);
    tile_chunk0[t] = (uint32_t)ctx->h_chunk_tile.size();
    for (uint64_t c = b; c < e; c += kChunk) {
      ctx->h_chunk_tile.push_back(t);
      ctx->h_chunk_start.push_back(c);
      ctx->h_chunk_len.push_back((uint32_t)std::min<uint64_t>(kChunk, e - c));
    }
  }
  tile_chunk0[g.tiles] = (uint32_t)ctx->h_chunk_tile.size();
  const uint64_t nchunks = ctx->h_chunk_tile.size();
  const uint64_t n = tr->num_records;
  if (nchunks + 2 * (g.tiles + 1) > ctx->chunk_cap || !ctx->chunk_tile) {
    uint64_t cap = (nchunks + 2 * (g.tiles + 1)) * 2 + 64;
    if (ctx->chunk_cnt) { hipFree(ctx->chunk_cnt); hipFree(ctx->chunk_tile); hipFree(ctx->chunk_start); hipFree(ctx->chunk_len); }
    GG_HIP(hipMalloc((void**)&ctx->chunk_cnt, sizeof(uint32_t) * cap * g.u1));
    GG_HIP(hipMalloc((void**)&ctx->chunk_tile, sizeof(uint32_t) * cap));
    GG_HIP(hipMalloc((void**)&ctx->chunk_start, sizeof(uint64_t) * cap));
    GG_HIP(hipMalloc((void**)&ctx->chunk_len, sizeof(uint32_t) * cap));
    ctx->chunk_cap = cap;
  }
  uint64_t cap_key = ctx->sh_cap, cap_idx = ctx->sh_cap;
  if (gg_status st = grow(&ctx->sh_key, &cap_key, n)) return st;
  if (gg_status st = grow(&ctx->sh_idx, &cap_idx, n)) return st;
  ctx->sh_cap = std::min(cap_key, cap_idx);

  // upload tables (chunk_tile doubles as storage for tile_chunk0 after the chunk entries)
  GG_HIP(hipMemcpyAsync(ctx->chunk_tile, ctx->h_chunk_tile.data(), sizeof(uint32_t) * nchunks, hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(ctx->chunk_tile + nchunks, tile_chunk0.data(), sizeof(uint32_t) * (g.tiles + 1), hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(ctx->chunk_start, ctx->h_chunk_start.data(), sizeof(uint64_t) * nchunks, hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(ctx->chunk_len, ctx->h_chunk_len.data(), sizeof(uint32_t) * nchunks, hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(ctx->tile_off_dev, tr->tile_offsets, sizeof(uint64_t) * (g.tiles + 1), hipMemcpyHostToDevice, s));

  if (nchunks) {
    gg_timer_begin(ctx, "cache_shard", s);
    hipLaunchKernelGGL(k_shard_hist, dim3((uint32_t)nchunks), dim3(256), 0, s, tr->addr_dev, ctx->chunk_tile,
                       ctx->chunk_start, ctx->chunk_len, ctx->chunk_cnt, g, ctx->err_dev);
    GG_HIP(hipGetLastError());
  }
  uint32_t scan_threads = 64;
  while (scan_threads < g.u1) scan_threads <<= 1;
  hipLaunchKernelGGL(k_shard_scan, dim3(g.tiles), dim3(scan_threads), 0, s, ctx->chunk_cnt,
                     ctx->chunk_tile + nchunks, ctx->tile_off_dev, ctx->unit_len, ctx->unit_base, g);
  GG_HIP(hipGetLastError());
  if (nchunks) {
    hipLaunchKernelGGL(k_shard_scatter, dim3((uint32_t)nchunks), dim3(64), 0, s, tr->addr_dev, tr->meta_dev,
                       ctx->chunk_tile, ctx->chunk_start, ctx->chunk_len, ctx->chunk_cnt, ctx->unit_base,
                       ctx->tile_off_dev, ctx->sh_key, ctx->sh_idx, g);
    GG_HIP(hipGetLastError());
    gg_timer_end(ctx, "cache_shard", s);
  }
  const Kern* k = find_kernel(g.a1, g.a2);
  const uint32_t groups = (uint32_t)((g.units + GG_WAVE - 1) / GG_WAVE);
  gg_timer_begin(ctx, "cache_replay", s);
  hipLaunchKernelGGL(k->replay, dim3(groups), dim3(GG_WAVE), replay_lds_bytes(g), s, ctx->cs, g,
                     (const uint64_t*)ctx->sh_key, (const uint32_t*)ctx->sh_idx, (const uint32_t*)ctx->unit_len,
                     (const uint64_t*)ctx->unit_base, (const uint64_t*)ctx->tile_off_dev, result, evicted, ctx->err_dev);
  GG_HIP(hipGetLastError());
  gg_timer_end(ctx, "cache_replay", s);
  return GG_OK;
}

gg_status gg_cache_quartet(gg_ctx* ctx, int op, uint32_t tile, int level, uint64_t addr,
                           const gg_line_info* in, gg_line_info* out, int* eviction, uint64_t* ev_addr)
{
  const gg_geom& g = ctx->g;
  if (tile >= g.tiles || (level != GG_L1D && level != GG_L2)) return gg_fail(GG_ERR_INVALID, "bad tile/level");
  if (addr >= g.addr_limit) return gg_fail(GG_ERR_RANGE, "address beyond the encodable range");
  QuartetIO q{};
  q.op = op; q.level = level; q.tile = tile; q.addr = addr;
  if (in) q.in = *in;
  if (out) q.out = *out; else { q.out.tag = ~0ull; q.out.cstate = 0; q.out.cached_loc = 0; }
  QuartetIO* d = nullptr;
  GG_HIP(hipMalloc((void**)&d, sizeof(QuartetIO)));
  hipStream_t s = ctx->last_stream;
  GG_HIP(hipMemcpyAsync(d, &q, sizeof(q), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(find_kernel(g.a1, g.a2)->quartet, dim3(1), dim3(1), 0, s, ctx->cs, g, d);
  GG_HIP(hipGetLastError());
  GG_HIP(hipMemcpyAsync(&q, d, sizeof(q), hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  hipFree(d);
  if (out) *out = q.out;
  if (eviction) *eviction = q.eviction;
  if (ev_addr) *ev_addr = q.ev_addr;
  if (q.status != GG_OK) return gg_fail(q.status, "Cache quartet op %d rejected (tile %u, level %d, addr %#llx)",
                                        op, tile, level, (unsigned long long)addr);
  return GG_OK;
}
