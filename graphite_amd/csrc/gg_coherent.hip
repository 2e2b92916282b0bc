// gg_coherent.hip — the coherent ("Mode C") path on MI355X (gfx950):
// pr_l1_pr_l2_dram_directory_msi with the DRAM directory, DRAM controller,
// ShmemPerfModel clock, memory network and lax-barrier quanta, in the
// canonical step schedule of DESIGN.md §Mode C.
//
// Reference (nmtrmail/Graphite, common/tile/memory_subsystem/):
//   pr_l1_pr_l2_dram_directory_msi/l1_cache_cntlr.cc:89-305   L1 state machine
//   pr_l1_pr_l2_dram_directory_msi/l2_cache_cntlr.cc:74-527   L2 state machine
//   pr_l1_pr_l2_dram_directory_msi/dram_directory_cntlr.cc:43-550  MSI directory
//   cache/directory_cache.cc:102-348                          DirectoryCache
//   directory_schemes/directory_entry_full_map.cc:18-86       full-map sharers
//   dram_cntlr.cc:37-74, performance_models/dram_perf_model.cc:75-116  DRAM
//   performance_models/shmem_perf_model.cc:16-45              per-tile clock
//   network: gg_dev.h route_closed_form (emesh_hop_counter / magic)
//
// Layout: one lane = one tile (the tile's controllers are sequential by
// construction: a per-tile lock in the reference, memory_manager.cc:78-120).
// Every tile owns its state in HBM, indexed by local tile (tile - first owned):
// L1-D / L2 sets (u64 line tags + one meta byte per way: state, cached_loc,
// LRU age), the directory slice (16-byte entries + full-map sharer words), the
// replaced-entry pool, the per-address request FIFO and the DRAM history tree.
// A step is two launches: k_c_tiles (lane per tile: inbox, then trace) and
// k_c_route (thread per message: network latency, delivery into per-tile
// linked lists of the next step or into the quantum-boundary buffer).  Steps
// are launched in batches; a step that sends nothing sets `quiet`, and the
// launches after it return at once, so one host sync per batch suffices.
#include "gg_dev.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdlib>

namespace {
using namespace gg;

enum { M_EX_REQ = GG_MSG_EX_REQ, M_SH_REQ = GG_MSG_SH_REQ, M_INV_REQ = GG_MSG_INV_REQ,
       M_FLUSH_REQ = GG_MSG_FLUSH_REQ, M_WB_REQ = GG_MSG_WB_REQ, M_EX_REP = GG_MSG_EX_REP,
       M_SH_REP = GG_MSG_SH_REP, M_INV_REP = GG_MSG_INV_REP, M_FLUSH_REP = GG_MSG_FLUSH_REP,
       M_WB_REP = GG_MSG_WB_REP, M_NULLIFY_REQ = GG_MSG_NULLIFY_REQ };
enum { DS_UNCACHED = 0, DS_SHARED = 1, DS_MODIFIED = 2 };
enum { ST_I = 0, ST_S = 1, ST_M = 2 };           // meta byte bits 0-1
#define INV_ADDR (~0ull)
#define NO_ENT (-0x7fffffff)

__device__ __forceinline__ bool to_directory(uint32_t t)
{
  return t == M_EX_REQ || t == M_SH_REQ || t == M_INV_REP || t == M_FLUSH_REP || t == M_WB_REP;
}
__device__ __forceinline__ bool has_data(uint32_t t)
{
  return t == M_EX_REP || t == M_SH_REP || t == M_FLUSH_REP || t == M_WB_REP;
}

struct DEnt { uint64_t addr; int32_t owner; uint16_t dstate; uint16_t nsh; };   // 16 B
struct CReq { uint64_t addr, time; uint32_t type, requester; };                 // 24 B

struct CP {
  uint32_t T, K, tb, lt;                 // tiles, shards, first owned tile, owned tiles
  uint32_t s1, a1, s2, a2, log_line, pol1, pol2;
  uint32_t E, dassoc, log_dsets, log_slices, W, R, QC, IC;
  uint32_t bits_req, bits_data, max_list, analytical, dram_qm;
  uint32_t dram_qtype, dram_qaux;          // dram/queue_model/type (GG_QM_*) and its hq_aux parameter
  uint64_t lat_l1d, lat_l1t, lat_l2d, lat_l2t, lat_dir, gap_ps, dram_proc, dram_cost;
  uint64_t msg_cap;
  uint32_t tiles_per_block;              // 64: a lane per tile; 1: a wave per tile (lane 0)
  uint32_t stage_rq;                     // wave per tile: directory request FIFO staged in LDS per step
  NocParams np;
};

struct CS {
  uint64_t* l1_tag; uint8_t* l1_meta; uint8_t* l1_rr;
  uint64_t* l2_tag; uint8_t* l2_meta; uint8_t* l2_rr;
  uint64_t* cc;                          // [lt][2][12]
  uint64_t* st;                          // [lt][GG_NUM_TILE_STATS]
  uint64_t *rec, *rec_end, *clk, *pend_start, *out_addr, *out_time;
  uint32_t *blocked, *seq;
  DEnt* dir; uint64_t* dsh;              // [lt][E], [lt][E][W]
  DEnt* rep; uint64_t* rsh; uint32_t* nrep;   // [lt][R], [lt][R][W]
  CReq* rq; uint32_t* nrq;               // [lt][QC]
  HQueue* dq; HNode* dnd; int16_t* dfl;  // DRAM queue per tile
  const uint64_t* addr; const uint32_t* meta; uint64_t* out;
  gg_cmsg* buf0; gg_cmsg* buf1; uint32_t* cnt;   // cnt[2]
  int32_t* head0; int32_t* head1;                // [lt]
  gg_cmsg* bnd; uint32_t* bnd_cnt;
  uint32_t* scratch;                     // [lt][IC]
  uint32_t* quiet; uint64_t* ri;
  // hop-by-hop: the step's messages as packet arrays (gg_noc_hbh)
  uint32_t *pk_src, *pk_dst, *pk_len; uint64_t *pk_t0, *pk_khi, *pk_klo;
  uint64_t* ctr;                         // NoC counters [T][GG_NUM_NET_COUNTERS]
  uint32_t* err;
  // GG_COH_PROFILE=1 (diagnostics): shader-clock cycles per step phase
  unsigned long long* prof;              // [0..3] phase sums over tiles and steps, [8 + step] max tile total
  uint32_t prof_steps;
};

__device__ __forceinline__ gg_cmsg* bufp(const CS& S, int p) { return p ? S.buf1 : S.buf0; }
__device__ __forceinline__ int32_t* headp(const CS& S, int p) { return p ? S.head1 : S.head0; }

// ---------------------------------------------------------------------------
// one private cache (Cache + CacheSet + replacement policy, cache.cc / cache_set.cc)
// ---------------------------------------------------------------------------
#define CMAXW 16   // ways held in registers at once (larger associativities take the serial path)
struct Cache {
  uint64_t* tag; uint8_t* meta; uint8_t* rr; uint64_t* cg;
  uint32_t sets, ways, log_line, pol, wb;
  uint32_t c[GG_NUM_CACHE_COUNTERS];   // this step's counter increments (registers), flushed to cg

  __device__ __forceinline__ uint32_t set_of(uint64_t a) const { return (uint32_t)((a >> log_line) & (sets - 1)); }   // cache_hash_fn.h:17
  __device__ __forceinline__ uint64_t tag_of(uint64_t a) const { return a >> log_line; }                             // cache.cc:495
  // the set's tags and meta bytes, every way's load in flight at once
  __device__ __forceinline__ void load_set(uint32_t s, uint64_t (&tv)[CMAXW], uint8_t (&mv)[CMAXW]) const
  {
    const uint64_t* p = tag + (size_t)s * ways;
    const uint8_t* m = meta + (size_t)s * ways;
#pragma unroll
    for (int w = 0; w < CMAXW; ++w) { tv[w] = INV_ADDR; mv[w] = 0; if (w < (int)ways) { tv[w] = p[w]; mv[w] = m[w]; } }
  }
  // CacheSet::find (cache_set.cc:57-70); tags are unique, so any match is the match
  __device__ __forceinline__ int find(uint32_t s, uint64_t t, uint8_t& mb) const
  {
    if (ways <= CMAXW) {
      uint64_t tv[CMAXW]; uint8_t mv[CMAXW];
      load_set(s, tv, mv);
      int f = -1; mb = 0;
#pragma unroll
      for (int w = 0; w < CMAXW; ++w) if (w < (int)ways && tv[w] == t) { f = w; mb = mv[w]; }
      return f;
    }
    for (int w = (int)ways - 1; w >= 0; --w)
      if (tag[(size_t)s * ways + w] == t) { mb = meta[(size_t)s * ways + w]; return w; }
    return -1;
  }
  __device__ __forceinline__ void touch(uint32_t s, uint32_t w)                                                        // lru:40-50
  {
    if (pol != GG_POLICY_LRU) return;
    uint8_t* m = meta + (size_t)s * ways;
    if (ways <= CMAXW) {
      uint8_t v[CMAXW];
#pragma unroll
      for (int i = 0; i < CMAXW; ++i) { v[i] = 0; if (i < (int)ways) v[i] = m[i]; }
      uint32_t acc = 0;
#pragma unroll
      for (int i = 0; i < CMAXW; ++i) if (i == (int)w) acc = v[i] >> 3;
#pragma unroll
      for (int i = 0; i < CMAXW; ++i) {
        if (i >= (int)ways) continue;
        const uint32_t a = v[i] >> 3;
        const uint8_t nv = (i == (int)w) ? (uint8_t)(v[i] & 7u) : (a < acc ? (uint8_t)((v[i] & 7u) | ((a + 1) << 3)) : v[i]);
        if (nv != v[i]) m[i] = nv;
      }
      return;
    }
    const uint32_t acc = m[w] >> 3;
    for (uint32_t i = 0; i < ways; ++i) { uint32_t a = m[i] >> 3; if (a < acc) m[i] = (uint8_t)((m[i] & 7u) | ((a + 1) << 3)); }
    m[w] = (uint8_t)(m[w] & 7u);
  }
  // getReplacementWay: LRU (lru:23-38) = first invalid way, else the (last) way of age assoc-1;
  // round robin (rr:13-22).  Returns the way and its current tag / meta byte.
  __device__ __forceinline__ int victim(uint32_t s, uint64_t& vt, uint8_t& vm)
  {
    if (pol == GG_POLICY_LRU) {
      if (ways <= CMAXW) {
        uint64_t tv[CMAXW]; uint8_t mv[CMAXW];
        load_set(s, tv, mv);
        int inv = -1, way = -1;
#pragma unroll
        for (int i = CMAXW - 1; i >= 0; --i) if (i < (int)ways && tv[i] == INV_ADDR) inv = i;
#pragma unroll
        for (int i = 0; i < CMAXW; ++i) if (i < (int)ways && tv[i] != INV_ADDR && (uint32_t)(mv[i] >> 3) == ways - 1) way = i;
        const int r = inv >= 0 ? inv : way;
        vt = INV_ADDR; vm = 0;
#pragma unroll
        for (int i = 0; i < CMAXW; ++i) if (i == r) { vt = tv[i]; vm = mv[i]; }
        return r;
      }
      const uint8_t* m = meta + (size_t)s * ways;
      int way = -1;
      for (uint32_t i = 0; i < ways; ++i) {
        if (tag[(size_t)s * ways + i] == INV_ADDR) { vt = INV_ADDR; vm = m[i]; return (int)i; }
        else if ((uint32_t)(m[i] >> 3) == ways - 1) way = (int)i;
      }
      if (way >= 0) { vt = tag[(size_t)s * ways + way]; vm = m[way]; }
      return way;
    }
    const uint32_t cur = rr[s];
    rr[s] = (uint8_t)(cur == 0 ? ways - 1 : cur - 1);
    vt = tag[(size_t)s * ways + cur]; vm = meta[(size_t)s * ways + cur];
    return (int)cur;
  }
  __device__ __forceinline__ void miss_counters(bool wr, bool miss)                                                   // cache.cc:321-360
  {
    c[GG_CC_ACCESSES]++;
    if (wr) c[GG_CC_WRITE_ACCESSES]++; else c[GG_CC_READ_ACCESSES]++;
    if (miss) { c[GG_CC_MISSES]++; if (wr) c[GG_CC_WRITE_MISSES]++; else c[GG_CC_READ_MISSES]++; }
  }
  // getCacheLineInfo (cache.cc:187-215): state / loc of the line, I / 0 when absent
  __device__ __forceinline__ void get(uint64_t a, uint32_t& st, uint32_t& loc)
  {
    uint8_t m;
    const int w = find(set_of(a), tag_of(a), m);
    c[GG_CC_TAG_READS]++;
    if (w >= 0) { st = m & 3u; loc = (m >> 2) & 1u; }
    else { st = ST_I; loc = 0; }
  }
  // setCacheLineInfo (cache.cc:218-241): st == I writes the invalid tag (CacheLineInfo::invalidate)
  __device__ __forceinline__ bool set(uint64_t a, uint32_t st, uint32_t loc)
  {
    const uint32_t s = set_of(a);
    uint8_t m;
    const int w = find(s, tag_of(a), m);
    if (w < 0) return false;
    meta[(size_t)s * ways + w] = (uint8_t)((m & 0xF8u) | st | (loc << 2));
    if (st == ST_I) tag[(size_t)s * ways + w] = INV_ADDR;
    c[GG_CC_TAG_WRITES]++;
    return true;
  }
  // accessCacheLine (cache.cc:84-112)
  __device__ __forceinline__ bool access(uint64_t a, bool store)
  {
    const uint32_t s = set_of(a);
    uint8_t m;
    const int w = find(s, tag_of(a), m);
    if (w < 0) return false;
    touch(s, (uint32_t)w);
    if (store) c[GG_CC_DATA_WRITES]++; else c[GG_CC_DATA_READS]++;
    return true;
  }
  // insertCacheLine (cache.cc:114-184); returns false on a policy error
  __device__ __forceinline__ bool insert(uint64_t a, uint32_t st, uint32_t loc, bool& ev, uint64_t& ev_addr, uint32_t& ev_st,
                         uint32_t& ev_loc)
  {
    const uint32_t s = set_of(a);
    uint64_t vt; uint8_t vm;
    const int w = victim(s, vt, vm);
    if (w < 0 || (uint32_t)w >= ways) return false;
    const size_t i = (size_t)s * ways + w;
    ev = vt != INV_ADDR;
    if (ev) { ev_addr = vt << log_line; ev_st = vm & 3u; ev_loc = (vm >> 2) & 1u; }
    tag[i] = tag_of(a);
    meta[i] = (uint8_t)((vm & 0xF8u) | st | (loc << 2));
    touch(s, (uint32_t)w);
    c[GG_CC_TAG_READS]++;
    if (ev) {
      c[GG_CC_DATA_READS]++;
      c[GG_CC_EVICTIONS]++;
      if (wb && ev_st == ST_M) c[GG_CC_DIRTY_EVICTIONS]++;
    }
    c[GG_CC_TAG_WRITES]++; c[GG_CC_DATA_WRITES]++;
    return true;
  }
  // all loads in flight, then all stores (no load waits behind a store)
  __device__ __forceinline__ void flush()
  {
    uint64_t v[GG_NUM_CACHE_COUNTERS];
#pragma unroll
    for (int k = 0; k < GG_NUM_CACHE_COUNTERS; ++k) v[k] = cg[k];
#pragma unroll
    for (int k = 0; k < GG_NUM_CACHE_COUNTERS; ++k) cg[k] = v[k] + c[k];
  }
};

// work items of the directory controller's call chains (recursion in the
// reference, an explicit continuation stack here)
enum { W_NONE = 0, W_PROC, W_CONT, W_NEXT, W_NULLIFY };
struct Work { uint64_t addr; uint32_t kind, type, requester, cached; int32_t h; };
#define WSTACK 32

// ---------------------------------------------------------------------------
// one tile's controllers
// ---------------------------------------------------------------------------
struct Tile {
  const CP& P; const CS& S;
  uint32_t lt, tile; int po;
  Cache L1, L2;
  uint64_t* stg;
  uint64_t st[GG_NUM_TILE_STATS];       // this step's statistics increments (registers)
  // the tile's scalars, in registers for the step (written back by flush)
  uint64_t rec, rec_end, clk, pend_start, out_addr, out_time;
  uint32_t blocked, seq, nrep, nrq;
  // the tile's DRAM queue (history tree) and directory request FIFO: global
  // memory, or the step's LDS copies
  HQueue* dq; HNode* dnd; int16_t* dfl;
  CReq* rqp;

  __device__ __forceinline__ Tile(const CP& p, const CS& s, uint32_t l, int out_parity) : P(p), S(s), lt(l), tile(p.tb + l), po(out_parity)
  {
    L1 = Cache{S.l1_tag + (size_t)lt * P.s1 * P.a1, S.l1_meta + (size_t)lt * P.s1 * P.a1, S.l1_rr + (size_t)lt * P.s1,
               S.cc + (size_t)lt * 2 * GG_NUM_CACHE_COUNTERS, P.s1, P.a1, P.log_line, P.pol1, 0, {}};
    L2 = Cache{S.l2_tag + (size_t)lt * P.s2 * P.a2, S.l2_meta + (size_t)lt * P.s2 * P.a2, S.l2_rr + (size_t)lt * P.s2,
               S.cc + ((size_t)lt * 2 + 1) * GG_NUM_CACHE_COUNTERS, P.s2, P.a2, P.log_line, P.pol2, 1, {}};
    stg = S.st + (size_t)lt * GG_NUM_TILE_STATS;
#pragma unroll
    for (int k = 0; k < GG_NUM_TILE_STATS; ++k) st[k] = 0;
    rec = S.rec[lt]; rec_end = S.rec_end[lt]; clk = S.clk[lt]; pend_start = S.pend_start[lt];
    out_addr = S.out_addr[lt]; out_time = S.out_time[lt];
    blocked = S.blocked[lt]; seq = S.seq[lt]; nrep = S.nrep[lt]; nrq = S.nrq[lt];
    dq = S.dq + lt; dnd = S.dnd + (size_t)lt * P.max_list; dfl = S.dfl + (size_t)lt * P.max_list;
    rqp = S.rq + (size_t)lt * P.QC;
  }
  __device__ __forceinline__ void flush()
  {
    L1.flush(); L2.flush();
    uint64_t v[GG_NUM_TILE_STATS];
#pragma unroll
    for (int k = 0; k < GG_NUM_TILE_STATS; ++k) v[k] = stg[k];
#pragma unroll
    for (int k = 0; k < GG_NUM_TILE_STATS; ++k) stg[k] = (k == GG_CT_CLOCK_PS) ? clk : v[k] + st[k];
    S.rec[lt] = rec; S.clk[lt] = clk; S.pend_start[lt] = pend_start;
    S.out_addr[lt] = out_addr; S.out_time[lt] = out_time;
    S.blocked[lt] = blocked; S.seq[lt] = seq; S.nrep[lt] = nrep; S.nrq[lt] = nrq;
  }
  __device__ __forceinline__ void fail(uint32_t e = GG_DERR_STATE) const { atomicOr(S.err, e); }

  // MemoryManager::sendMsg (…msi/memory_manager.cc:306-332)
  __device__ __forceinline__ void send(uint32_t dst, uint32_t type, uint32_t requester, uint64_t addr, uint64_t t)
  {
    const uint64_t p0 = S.prof ? __builtin_amdgcn_s_memtime() : 0;
    send_(dst, type, requester, addr, t);
    if (S.prof) atomicAdd(&S.prof[11], (unsigned long long)(__builtin_amdgcn_s_memtime() - p0));
  }
  __device__ __forceinline__ void send_(uint32_t dst, uint32_t type, uint32_t requester, uint64_t addr, uint64_t t)
  {
    const uint32_t i = atomicAdd(&S.cnt[po], 1u);
    if (i >= P.msg_cap) { fail(GG_DERR_CAP); return; }
    gg_cmsg m;
    m.addr = addr; m.send_ps = t; m.arrival_ps = t; m.src = tile; m.dst = dst; m.requester = requester;
    m.seq = seq++; m.type = type; m.link = 0xFFFFFFFFu;
    bufp(S, po)[i] = m;
    st[GG_CT_MSGS_SENT]++;
#pragma unroll
    for (int k = 0; k < 11; ++k) if (type == (uint32_t)k + 1) st[GG_CT_SENT_BY_TYPE + k]++;
  }
  __device__ __forceinline__ uint32_t home(uint64_t a) const { return (uint32_t)((a >> 6) % P.T); }   // address_home_lookup.cc:19-26

  // ---- directory (DirectoryCache + DirectoryEntryFullMap) ------------------
  __device__ __forceinline__ DEnt* ent(int32_t h) const
  {
    return h >= 0 ? S.dir + (size_t)lt * P.E + h : S.rep + (size_t)lt * P.R + (-h - 1);
  }
  __device__ __forceinline__ uint64_t* shw(int32_t h) const
  {
    return h >= 0 ? S.dsh + ((size_t)lt * P.E + h) * P.W : S.rsh + ((size_t)lt * P.R + (-h - 1)) * P.W;
  }
  __device__ __forceinline__ bool has(int32_t h, uint32_t s) const { return (shw(h)[s >> 6] >> (s & 63)) & 1ull; }
  __device__ __forceinline__ void add_sharer(int32_t h, uint32_t s)                 // addSharer (full_map.cc:27-33)
  {
    if (has(h, s)) fail();
    shw(h)[s >> 6] |= 1ull << (s & 63); ent(h)->nsh++;
  }
  __device__ __forceinline__ void remove_sharer(int32_t h, uint32_t s)              // removeSharer (:35-41)
  {
    if (!has(h, s)) { fail(); return; }
    shw(h)[s >> 6] &= ~(1ull << (s & 63)); ent(h)->nsh--;
  }
  __device__ __forceinline__ void set_owner(int32_t h, int32_t o)                   // DirectoryEntry::setOwner
  {
    if (o >= 0 && !has(h, (uint32_t)o)) fail();
    ent(h)->owner = o;
  }
  __device__ __forceinline__ uint32_t dset(uint64_t a) const                        // computeSetIndex (directory_cache.cc:332-348)
  {
    uint64_t s = 0;
    const uint64_t mask = (1ull << P.log_dsets) - 1;
    for (uint32_t i = P.log_line + P.log_slices; i + P.log_dsets <= 64; i += P.log_dsets) s ^= (a >> i) & mask;
    return (uint32_t)s;
  }
  // getDirectoryEntry (directory_cache.cc:102-145)
  __device__ __forceinline__ int32_t dget(uint64_t a, uint64_t& t)
  {
    const uint64_t p0 = S.prof ? __builtin_amdgcn_s_memtime() : 0;
    const int32_t r = dget_(a, t);
    if (S.prof) atomicAdd(&S.prof[9], (unsigned long long)(__builtin_amdgcn_s_memtime() - p0));
    return r;
  }
  __device__ __forceinline__ int32_t dget_(uint64_t a, uint64_t& t)
  {
    t += P.lat_dir;
    st[GG_CT_DIR_ACCESSES]++;
    const uint32_t base = dset(a) * P.dassoc;
    DEnt* d = S.dir + (size_t)lt * P.E;
    if (P.dassoc <= 16) {                           // every way's address in flight at once
      uint64_t v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) { v[i] = 0; if (i < (int)P.dassoc) v[i] = d[base + i].addr; }
      int hit = -1, fr = -1;
#pragma unroll
      for (int i = 15; i >= 0; --i) if (i < (int)P.dassoc) { if (v[i] == a) hit = i; if (v[i] == INV_ADDR) fr = i; }
      if (hit >= 0) return (int32_t)(base + hit);
      if (fr >= 0) { d[base + fr].addr = a; return (int32_t)(base + fr); }
    } else {
      for (uint32_t i = 0; i < P.dassoc; ++i) if (d[base + i].addr == a) return (int32_t)(base + i);
      for (uint32_t i = 0; i < P.dassoc; ++i) if (d[base + i].addr == INV_ADDR) { d[base + i].addr = a; return (int32_t)(base + i); }
    }
    const uint32_t nr = nrep;
    for (uint32_t r = 0; r < nr; ++r) if (ent(-(int32_t)r - 1)->addr == a) return -(int32_t)r - 1;
    return NO_ENT;
  }
  // replaceDirectoryEntry (directory_cache.cc:163-213): the slot gets a fresh
  // entry, the old one moves to the replaced list
  __device__ __forceinline__ int32_t dreplace(uint64_t replaced, uint64_t a, uint64_t& t)
  {
    const uint32_t base = dset(replaced) * P.dassoc;
    DEnt* d = S.dir + (size_t)lt * P.E;
    int32_t slot = -1;
    for (uint32_t i = 0; i < P.dassoc; ++i) if (d[base + i].addr == replaced) { slot = (int32_t)(base + i); break; }
    if (slot < 0) { fail(); return NO_ENT; }
    const uint32_t r = nrep;
    if (r >= P.R) { fail(GG_DERR_CAP); return NO_ENT; }
    nrep = r + 1;
    *ent(-(int32_t)r - 1) = d[slot];
    uint64_t* so = shw(slot); uint64_t* sr = shw(-(int32_t)r - 1);
    for (uint32_t w = 0; w < P.W; ++w) { sr[w] = so[w]; so[w] = 0; }
    d[slot] = DEnt{a, -1, DS_UNCACHED, 0};
    t += P.lat_dir;
    st[GG_CT_DIR_ACCESSES]++;
    st[GG_CT_DIR_EVICTIONS]++;
    if (ent(-(int32_t)r - 1)->dstate != DS_UNCACHED) st[GG_CT_DIR_BACK_INVALIDATIONS]++;
    return slot;
  }
  // invalidateDirectoryEntry (directory_cache.cc:215-231): erase from the replaced list
  __device__ __forceinline__ void dinvalidate(uint64_t a)
  {
    const uint32_t nr = nrep;
    for (uint32_t r = 0; r < nr; ++r) {
      if (ent(-(int32_t)r - 1)->addr != a) continue;
      for (uint32_t k = r; k + 1 < nr; ++k) {
        *ent(-(int32_t)k - 1) = *ent(-(int32_t)k - 2);
        uint64_t* dst = shw(-(int32_t)k - 1); const uint64_t* src = shw(-(int32_t)k - 2);
        for (uint32_t w = 0; w < P.W; ++w) dst[w] = src[w];
      }
      nrep = nr - 1;
      return;
    }
    fail();
  }

  // ---- per-address request FIFO (HashMapList<IntPtr, ShmemReq*>) -----------
  __device__ __forceinline__ CReq* q() const { return rqp; }
  __device__ __forceinline__ uint32_t qcount(uint64_t a) const
  {
    const uint32_t n = nrq; uint32_t c = 0;
    for (uint32_t i = 0; i < n; ++i) c += (q()[i].addr == a);
    return c;
  }
  __device__ __forceinline__ int32_t qfront(uint64_t a) const
  {
    const uint32_t n = nrq;
    for (uint32_t i = 0; i < n; ++i) if (q()[i].addr == a) return (int32_t)i;
    return -1;
  }
  __device__ __forceinline__ void qpush(uint64_t a, uint64_t t, uint32_t type, uint32_t req)
  {
    const uint32_t n = nrq;
    if (n >= P.QC) { fail(GG_DERR_CAP); return; }
    q()[n] = CReq{a, t, type, req};
    nrq = n + 1;
  }
  __device__ __forceinline__ void qpop(uint64_t a)
  {
    const uint32_t n = nrq;
    for (uint32_t i = 0; i < n; ++i) {
      if (q()[i].addr != a) continue;
      for (uint32_t k = i; k + 1 < n; ++k) q()[k] = q()[k + 1];
      nrq = n - 1;
      return;
    }
  }
  __device__ __forceinline__ static void front_time(CReq& r, uint64_t& t)   // ShmemReq::updateTime + updateCurrTime
  {
    if (r.time < t) r.time = t;
    if (t < r.time) t = r.time;
  }

  // ---- DramCntlr / DramPerfModel --------------------------------------------
  __device__ __forceinline__ uint64_t dram_ps(uint64_t t)
  {
    const uint64_t p0 = S.prof ? __builtin_amdgcn_s_memtime() : 0;
    const uint64_t r = dram_ps_(t);
    if (S.prof) atomicAdd(&S.prof[10], (unsigned long long)(__builtin_amdgcn_s_memtime() - p0));
    return r;
  }
  __device__ __forceinline__ uint64_t dram_ps_(uint64_t t)
  {
    const uint64_t pkt_ns = (uint64_t)ceil(t / 1000.0);
    uint64_t qd = 0;
    if (P.dram_qm) {
      HTree tr{dq, dnd, dfl, P.dram_proc, P.analytical != 0};
      qd = tr.delay(pkt_ns, P.dram_proc, S.err);
      st[GG_CT_DRAM_QUEUE_REQUESTS]++;
    }
    const uint64_t lat = qd + P.dram_proc + P.dram_cost;
    st[GG_CT_DRAM_ACCESSES]++;
    st[GG_CT_DRAM_LATENCY_NS] += lat;
    st[GG_CT_DRAM_QUEUE_DELAY_NS] += qd;
    return lat_to_ps(lat, 1.0);
  }

  // ---- DramDirectoryCntlr: the call chains as a work loop -------------------
  __device__ __forceinline__ void directory_run(Work w, uint64_t& t)
  {
    Work stack[WSTACK];
    int sp = 0;
    for (;;) {
      switch (w.kind) {
      case W_PROC: {                     // processEx/ShReqFromL2Cache (:238-380): entry lookup
        int32_t h = dget(w.addr, t);
        if (h == NO_ENT) {               // processDirectoryEntryAllocationReq (:126-170)
          const uint64_t msg_time = t;
          if (dget(w.addr, t) != NO_ENT) fail();   // the assert in getReplacementCandidates (directory_cache.cc:161)
          const uint32_t base = dset(w.addr) * P.dassoc;
          const DEnt* d = S.dir + (size_t)lt * P.E;
          int32_t cand = -1;
          for (uint32_t i = 0; i < P.dassoc; ++i) {
            const DEnt& it = d[base + i];
            if ((cand < 0 || d[cand].nsh > it.nsh) && qcount(it.addr) == 0) cand = (int32_t)(base + i);
          }
          if (cand < 0) { fail(); return; }
          const uint64_t replaced = d[cand].addr;
          h = dreplace(replaced, w.addr, t);
          if (h == NO_ENT) return;
          qpush(replaced, msg_time, M_NULLIFY_REQ, w.requester);
          if (qcount(replaced) != 1) fail();
          if (sp >= WSTACK) { fail(GG_DERR_CAP); return; }
          Work c = w; c.kind = W_CONT; c.h = h;
          stack[sp++] = c;
          w = Work{replaced, W_NULLIFY, 0, w.requester, 0, 0};
          continue;
        }
        w.kind = W_CONT; w.h = h;
        continue;
      }
      case W_CONT: {                     // the directory-state switch
        DEnt* e = ent(w.h);
        if (w.type == M_EX_REQ) {
          if (e->dstate == DS_MODIFIED) {
            if (w.cached) fail();
            send((uint32_t)e->owner, M_FLUSH_REQ, w.requester, w.addr, t);
            w.kind = W_NONE;
          } else if (e->dstate == DS_SHARED) {
            if (w.cached) fail();
            const uint64_t* sh = shw(w.h);
            for (uint32_t k = 0; k < P.W; ++k) {                     // getSharersList: ascending
              uint64_t bits = sh[k];
              while (bits) {
                const uint32_t b = __builtin_ctzll(bits); bits &= bits - 1;
                send(k * 64 + b, M_INV_REQ, w.requester, w.addr, t);
              }
            }
            w.kind = W_NONE;
          } else {
            add_sharer(w.h, w.requester);
            set_owner(w.h, (int32_t)w.requester);
            ent(w.h)->dstate = DS_MODIFIED;
            if (!w.cached) t += dram_ps(t);                         // retrieveDataAndSendToL2Cache (:382-408)
            send(w.requester, M_EX_REP, w.requester, w.addr, t);
            w.kind = W_NEXT;
          }
        } else {
          if (e->dstate == DS_MODIFIED) {
            if (w.cached) fail();
            send((uint32_t)e->owner, M_WB_REQ, w.requester, w.addr, t);
            w.kind = W_NONE;
          } else {
            add_sharer(w.h, w.requester);
            ent(w.h)->dstate = DS_SHARED;
            if (!w.cached) t += dram_ps(t);
            send(w.requester, M_SH_REP, w.requester, w.addr, t);
            w.kind = W_NEXT;
          }
        }
        continue;
      }
      case W_NEXT: {                     // processNextReqFromL2Cache (:98-124)
        if (qcount(w.addr) < 1) { fail(); return; }
        qpop(w.addr);
        const int32_t f = qfront(w.addr);
        if (f < 0) { w.kind = W_NONE; continue; }
        CReq& r = q()[f];
        front_time(r, t);
        if (r.type != M_EX_REQ && r.type != M_SH_REQ) { fail(); return; }
        w = Work{w.addr, W_PROC, r.type, r.requester, 0, 0};
        continue;
      }
      case W_NULLIFY: {                  // processNullifyReq (:172-236)
        const int32_t h = dget(w.addr, t);
        if (h == NO_ENT) { fail(); return; }
        DEnt* e = ent(h);
        if (e->dstate == DS_MODIFIED) {
          send((uint32_t)e->owner, M_FLUSH_REQ, w.requester, w.addr, t);
          w.kind = W_NONE;
        } else if (e->dstate == DS_SHARED) {
          const uint64_t* sh = shw(h);
          for (uint32_t k = 0; k < P.W; ++k) {
            uint64_t bits = sh[k];
            while (bits) {
              const uint32_t b = __builtin_ctzll(bits); bits &= bits - 1;
              send(k * 64 + b, M_INV_REQ, w.requester, w.addr, t);
            }
          }
          w.kind = W_NONE;
        } else {
          dinvalidate(w.addr);
          w.kind = W_NEXT;
        }
        continue;
      }
      default:
        if (sp == 0) return;
        w = stack[--sp];
        continue;
      }
    }
  }

  // handleMsgFromL2Cache (:43-96) + processInv/Flush/WbRepFromL2Cache (:410-543); every
  // path ends in at most one directory call chain (one call site keeps the lane's
  // state in registers)
  __device__ __forceinline__ void directory_msg(const gg_cmsg& m)
  {
    uint64_t t = m.arrival_ps;           // __handleMsgFromNetwork: setCurrTime(packet.time)
    const uint64_t a = m.addr;
    Work w{a, W_NONE, 0, 0, 0, 0};
    if (m.type == M_EX_REQ || m.type == M_SH_REQ) {
      qpush(a, t, m.type, m.requester);
      if (qcount(a) == 1) w = Work{a, W_PROC, m.type, m.requester, 0, 0};
    } else {
      const int32_t h = dget(a, t);
      if (h == NO_ENT) { fail(); return; }
      DEnt* e = ent(h);
      const uint32_t ds = e->dstate;
      if (m.type == M_INV_REP) {
        if (ds != DS_SHARED) { fail(); return; }
        remove_sharer(h, m.src);
        const bool unc = e->nsh == 0;
        if (unc) e->dstate = DS_UNCACHED;
        const int32_t f = qfront(a);
        if (f >= 0) {
          CReq& r = q()[f];
          front_time(r, t);
          if (r.type == M_EX_REQ) { if (unc) w = Work{a, W_PROC, M_EX_REQ, r.requester, 0, 0}; }
          else if (r.type == M_SH_REQ) w = Work{a, W_PROC, M_SH_REQ, r.requester, 0, 0};
          else { if (unc) w = Work{a, W_NULLIFY, 0, r.requester, 0, 0}; }
        }
      } else if (m.type == M_FLUSH_REP) {
        if (ds != DS_MODIFIED) { fail(); return; }
        remove_sharer(h, m.src);
        set_owner(h, -1);
        e->dstate = DS_UNCACHED;
        const int32_t f = qfront(a);
        if (f < 0) { (void)dram_ps(t); return; }                    // putDataToDram: queue model, no latency
        CReq& r = q()[f];
        front_time(r, t);
        if (r.type == M_EX_REQ) w = Work{a, W_PROC, M_EX_REQ, r.requester, 1, 0};
        else if (r.type == M_SH_REQ) { (void)dram_ps(t); w = Work{a, W_PROC, M_SH_REQ, r.requester, 1, 0}; }
        else { (void)dram_ps(t); w = Work{a, W_NULLIFY, 0, r.requester, 0, 0}; }
      } else if (m.type == M_WB_REP) {
        if (ds != DS_MODIFIED || !has(h, m.src)) { fail(); return; }
        set_owner(h, -1);
        e->dstate = DS_SHARED;
        const int32_t f = qfront(a);
        if (f < 0) { fail(); return; }
        CReq& r = q()[f];
        front_time(r, t);
        (void)dram_ps(t);
        if (r.type != M_SH_REQ) { fail(); return; }
        w = Work{a, W_PROC, M_SH_REQ, r.requester, 1, 0};
      } else {
        fail();
        return;
      }
    }
    if (w.kind != W_NONE) directory_run(w, t);
  }

  // ---- L1 / L2 controllers ---------------------------------------------------
  __device__ __forceinline__ void l1_invalidate(uint64_t a)                          // l1_cache_cntlr.cc:293-305
  {
    uint32_t s, l;
    L1.get(a, s, l);
    if (s != ST_I && !L1.set(a, ST_I, 0)) fail();
  }
  __device__ __forceinline__ void l1_access(uint64_t a, bool wr)                    // l1:182-205 (+ write-through, l2:66-70)
  {
    if (!L1.access(a, wr)) fail();
    if (wr && !L2.access(a, true)) fail();
  }
  __device__ __forceinline__ void insert_in_l1(uint64_t a, uint32_t cs)             // l2_cache_cntlr.cc:133-165
  {
    bool ev; uint64_t ea = 0; uint32_t es = 0, el = 0;
    if (!L1.insert(a, cs, 0, ev, ea, es, el)) { fail(); return; }
    if (ev) {
      uint32_t s2, l2;
      L2.get(ea, s2, l2);
      if (l2 != 1) { fail(); return; }                               // cached_loc must be L1-D
      if (!L2.set(ea, s2, 0)) fail();                                // clearCachedLoc
    }
  }
  __device__ __forceinline__ void l2_insert(uint64_t a, uint32_t cs, uint64_t t)    // l2_cache_cntlr.cc:74-116
  {
    bool ev; uint64_t ea = 0; uint32_t es = 0, el = 0;
    if (!L2.insert(a, cs, 1, ev, ea, es, el)) { fail(); return; }
    if (ev) {
      if (el) l1_invalidate(ea);
      if (es == ST_M) send(home(ea), M_FLUSH_REP, tile, ea, t);
      else if (es == ST_S) send(home(ea), M_INV_REP, tile, ea, t);
      else fail();
    }
  }
  __device__ __forceinline__ void finish(uint64_t start, uint64_t end, uint32_t level)
  {
    const uint64_t r = rec;
    const uint64_t lat = end - start;
    if (S.out) S.out[r] = (lat << 2) | level;
    st[GG_CT_ACCESSES]++;
    st[GG_CT_LATENCY_PS] += lat;
    if (level == GG_LVL_L1) st[GG_CT_L1_HITS]++; else if (level == GG_LVL_L2) st[GG_CT_L2_HITS]++; else st[GG_CT_L2_MISSES]++;
    clk = end;
    rec = r + 1;
  }
  // Core::initiateMemoryAccess -> L1CacheCntlr::processMemOpFromCore, first attempt (l1:89-180)
  __device__ __forceinline__ void app_access(uint64_t a, bool wr, uint64_t s)
  {
    uint64_t t = s;
    uint32_t cs, loc;
    L1.get(a, cs, loc);
    const bool hit = wr ? cs == ST_M : cs != ST_I;
    L1.miss_counters(wr, !hit);
    if (hit) { t += P.lat_l1d; l1_access(a, wr); finish(s, t, GG_LVL_L1); return; }
    t += P.lat_l1t;
    l1_invalidate(a);
    uint32_t c2, l2;                                                 // processShmemRequestFromL1Cache (l2:180-224)
    L2.get(a, c2, l2);
    const bool hit2 = wr ? c2 == ST_M : c2 != ST_I;
    L2.miss_counters(wr, !hit2);
    if (hit2) {
      if (!L2.access(a, false)) fail();
      insert_in_l1(a, c2);
      if (!L2.set(a, c2, 1)) fail();                                 // set(Forced)CachedLoc(L1-D)
      t += P.lat_l2d; t += P.lat_l1d;
      l1_access(a, wr);
      finish(s, t, GG_LVL_L2);
      return;
    }
    t += P.lat_l2t;
    if (out_addr != INV_ADDR) fail();                          // handleMsgFromL1Cache (l2:226-258)
    out_addr = a; out_time = t;
    const uint32_t h = home(a);
    if (wr) {                                                        // processExReqFromL1Cache (l2:260-282)
      uint32_t x, xl;
      L2.get(a, x, xl);
      if (x == ST_S) { if (!L2.set(a, ST_I, 0)) fail(); send(h, M_INV_REP, tile, a, t); }
      else if (x != ST_I) fail();
      send(h, M_EX_REQ, tile, a, t);
    } else {
      send(h, M_SH_REQ, tile, a, t);
    }
    blocked = 1;
    pend_start = s;
  }
  // L2CacheCntlr::handleMsgFromDramDirectory (l2:294-502) + the core's second attempt
  __device__ __forceinline__ void l2_msg(const gg_cmsg& m)
  {
    uint64_t t = m.arrival_ps;
    const uint64_t a = m.addr;
    if (m.type == M_EX_REP || m.type == M_SH_REP) {
      const uint32_t cs = m.type == M_EX_REP ? ST_M : ST_S;
      if (!blocked || out_addr != a) { fail(); return; }
      l2_insert(a, cs, t);
      insert_in_l1(a, cs);
      if (out_time > t) fail();
      t += P.lat_l2d;
      out_addr = INV_ADDR;
      const bool wr = (S.meta[rec] & GG_META_WRITE) != 0;     // access_num == 2 (l1:106-126)
      uint32_t c1, l1;
      L1.get(a, c1, l1);
      const bool hit = wr ? c1 == ST_M : c1 != ST_I;
      if (!hit) { fail(); return; }
      t += P.lat_l1d;
      l1_access(a, wr);
      blocked = 0;
      finish(pend_start, t, GG_LVL_DIR);
      return;
    }
    uint32_t c2, loc;
    L2.get(a, c2, loc);
    if (c2 == ST_I) { t += P.lat_l2t; return; }                      // line already gone: tags only, no reply
    if (m.type == M_INV_REQ) {                                       // l2:369-410
      if (c2 != ST_S) { fail(); return; }
      t += P.lat_l2t;
      if (loc) { t += P.lat_l1t; l1_invalidate(a); }
      if (!L2.set(a, ST_I, 0)) fail();
      send(m.src, M_INV_REP, m.requester, a, t);
    } else if (m.type == M_FLUSH_REQ) {                              // l2:412-455
      if (c2 != ST_M) { fail(); return; }
      t += P.lat_l2d;
      if (loc) { t += P.lat_l1t; l1_invalidate(a); }
      if (!L2.access(a, false)) fail();
      if (!L2.set(a, ST_I, 0)) fail();
      send(m.src, M_FLUSH_REP, m.requester, a, t);
    } else if (m.type == M_WB_REQ) {                                 // l2:457-502
      if (c2 != ST_M) { fail(); return; }
      t += P.lat_l2d;
      if (loc) {
        t += P.lat_l1t;
        uint32_t c1, l1;                                             // setCacheLineState (l1:278-291)
        L1.get(a, c1, l1);
        if (c1 == ST_I) fail();
        if (!L1.set(a, ST_S, 0)) fail();
      }
      if (!L2.access(a, false)) fail();
      if (!L2.set(a, ST_S, loc)) fail();
      send(m.src, M_WB_REP, m.requester, a, t);
    } else {
      fail();
    }
  }
};

__device__ __forceinline__ bool chan_lt(const gg_cmsg& a, const gg_cmsg& b)
{
  return a.src < b.src || (a.src == b.src && a.seq < b.seq);
}

// A step, lane per owned tile: the inbox (per-channel FIFO, channels merged by
// (arrival, sender)), then the trace up to the barrier or the next miss.
// One tile per wave (a one-lane workgroup): the tiles' controller paths diverge
// completely, so packing 64 tiles into one wave would serialize the union of
// their paths; one wave per tile costs issue slots the chip has to spare.
// The DRAM history tree of a wave-per-tile step lives in LDS for the step: the
// wave copies it in (HQueue + max_list nodes + free list, 16 B per lane per
// load) before lane 0 runs the tile, and back after.  Its AVL operations are
// chains of dependent node accesses, each an HBM/MALL round trip otherwise.
constexpr uint32_t kTreeLds = 128;           // largest max_list_size staged (carbon_sim.cfg: 100)
struct TreeLds {
  HQueue q;
  HNode nd[kTreeLds];
  int16_t fl[kTreeLds];
};

__device__ __forceinline__ void copy_words(uint32_t* dst, const uint32_t* src, uint32_t words, uint32_t lane)
{
  for (uint32_t i = lane; i < words; i += GG_WAVE) dst[i] = src[i];
}
// bytes (multiple of 4) between 16-B aligned buffers where possible
__device__ __forceinline__ void copy_bytes(void* dst, const void* src, uint32_t bytes, uint32_t lane)
{
  if ((((uintptr_t)dst | (uintptr_t)src | bytes) & 15) == 0) {
    uint4* d = (uint4*)dst; const uint4* q = (const uint4*)src;
    for (uint32_t i = lane; i < bytes / 16; i += GG_WAVE) d[i] = q[i];
  } else {
    copy_words((uint32_t*)dst, (const uint32_t*)src, bytes / 4, lane);
  }
}

struct StepLds { TreeLds* tree; CReq* rq; uint32_t* nrq_out; };

__device__ __forceinline__ void c_tile_step(const CP& P, const CS& S, int p, uint64_t barrier, uint32_t lt, const StepLds* sl);

__global__ void __launch_bounds__(64) k_c_tiles(CP P, CS S, int p, uint64_t barrier)
{
  if (*(volatile uint32_t*)S.quiet) return;
  if (P.tiles_per_block != 1) {
    const uint32_t lt = blockIdx.x * blockDim.x + threadIdx.x;
    if (lt == 0) S.ri[GG_RI_STEPS]++;
    if (lt < P.lt) c_tile_step(P, S, p, barrier, lt, nullptr);
    return;
  }
  const uint32_t lt = blockIdx.x, lane = threadIdx.x;
  if (lt == 0 && lane == 0) S.ri[GG_RI_STEPS]++;
  __shared__ TreeLds tl;
  extern __shared__ __attribute__((aligned(16))) uint8_t csm[];
  StepLds sl{};
  const bool tree = P.dram_qm && P.max_list <= kTreeLds && (P.max_list % 2) == 0;
  const uint32_t qw = sizeof(HQueue) / 4, nw = P.max_list * sizeof(HNode) / 4, fw = (P.max_list + 1) / 2;
  sl.tree = tree ? &tl : nullptr;
  if (tree) {
    copy_words((uint32_t*)&tl.q, (const uint32_t*)(S.dq + lt), qw, lane);
    copy_words((uint32_t*)tl.nd, (const uint32_t*)(S.dnd + (size_t)lt * P.max_list), nw, lane);
    copy_words((uint32_t*)tl.fl, (const uint32_t*)(S.dfl + (size_t)lt * P.max_list), fw, lane);
  }
  // the directory request FIFO (HashMapList of dram_directory_cntlr.h:46): its
  // scans are loops of dependent loads; staged when QC entries fit
  __shared__ uint32_t nrq_out;
  CReq* grq = S.rq + (size_t)lt * P.QC;
  if (P.stage_rq) {
    sl.rq = (CReq*)csm;
    sl.nrq_out = &nrq_out;
    copy_words((uint32_t*)sl.rq, (const uint32_t*)grq, S.nrq[lt] * (sizeof(CReq) / 4), lane);
  }
  __syncthreads();
  if (lane == 0) c_tile_step(P, S, p, barrier, lt, &sl);
  __syncthreads();
  if (P.stage_rq) copy_words((uint32_t*)grq, (const uint32_t*)sl.rq, nrq_out * (sizeof(CReq) / 4), lane);
  if (tree) {
    copy_words((uint32_t*)(S.dq + lt), (const uint32_t*)&tl.q, qw, lane);
    copy_words((uint32_t*)(S.dnd + (size_t)lt * P.max_list), (const uint32_t*)tl.nd, nw, lane);
    copy_words((uint32_t*)(S.dfl + (size_t)lt * P.max_list), (const uint32_t*)tl.fl, fw, lane);
  }
}

__device__ __forceinline__ void c_tile_step(const CP& P, const CS& S, int p, uint64_t barrier, uint32_t lt, const StepLds* sl)
{
  const uint64_t c0 = S.prof ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t r0 = S.prof ? __builtin_amdgcn_s_memrealtime() : 0;
  Tile T(P, S, lt, 1 - p);
  if (sl && sl->tree) { T.dq = &sl->tree->q; T.dnd = sl->tree->nd; T.dfl = sl->tree->fl; }
  if (sl && sl->rq) T.rqp = sl->rq;
  // 1. gather the inbox list
  int32_t* head = headp(S, p);
  const gg_cmsg* in = bufp(S, p);
  uint32_t* idx = S.scratch + (size_t)lt * P.IC;
  uint32_t n = 0;
  for (int32_t i = head[lt]; i >= 0; i = (int32_t)in[i].link) {
    if (n >= P.IC) { T.fail(GG_DERR_CAP); return; }
    idx[n++] = (uint32_t)i;
  }
  head[lt] = -1;
  // insertion sort by (sender, sequence)
  for (uint32_t i = 1; i < n; ++i) {
    const uint32_t v = idx[i];
    const gg_cmsg& mv = in[v];
    uint32_t j = i;
    while (j > 0 && chan_lt(mv, in[idx[j - 1]])) { idx[j] = idx[j - 1]; --j; }
    idx[j] = v;
  }
  const uint64_t c1 = S.prof ? __builtin_amdgcn_s_memtime() : 0;
  // merge the channels: repeatedly the channel head with the least (arrival, sender)
  for (uint32_t k = 0; k < n; ++k) {
    uint32_t best = ~0u, prev_src = ~0u;
    for (uint32_t i = 0; i < n; ++i) {
      if (idx[i] == ~0u) continue;
      const gg_cmsg& m = in[idx[i]];
      if (m.src == prev_src) continue;               // not the head of its channel
      prev_src = m.src;
      if (best == ~0u) { best = i; continue; }
      const gg_cmsg& b = in[idx[best]];
      if (m.arrival_ps < b.arrival_ps || (m.arrival_ps == b.arrival_ps && m.src < b.src)) best = i;
    }
    const gg_cmsg m = in[idx[best]];
    idx[best] = ~0u;
    T.st[GG_CT_MSGS_RECEIVED]++;
    const uint64_t h0 = S.prof ? __builtin_amdgcn_s_memtime() : 0;
    if (to_directory(m.type)) T.directory_msg(m); else T.l2_msg(m);
    if (S.prof) atomicAdd(&S.prof[to_directory(m.type) ? 5 : 6], (unsigned long long)(__builtin_amdgcn_s_memtime() - h0));
  }
  const uint64_t c2 = S.prof ? __builtin_amdgcn_s_memtime() : 0;
  // 2. the trace
  const uint64_t line_mask = ~((1ull << P.log_line) - 1);
  while (!T.blocked) {
    const uint64_t r = T.rec;
    if (r >= T.rec_end) break;
    const uint32_t meta = S.meta[r];
    const uint64_t s = T.clk + (uint64_t)((meta & 0x7FFFFFFFu) >> 1) * P.gap_ps;
    if (s >= barrier) break;
    T.app_access(S.addr[r] & line_mask, (meta & GG_META_WRITE) != 0, s);
  }
  const uint64_t c3 = S.prof ? __builtin_amdgcn_s_memtime() : 0;
  T.flush();
  if (sl && sl->nrq_out) *sl->nrq_out = T.nrq;
  if (S.prof) {
    const uint64_t c4 = __builtin_amdgcn_s_memtime();
    atomicAdd(&S.prof[0], (unsigned long long)(c1 - c0));     // tile load + inbox gather + sort
    atomicAdd(&S.prof[1], (unsigned long long)(c2 - c1));     // message handlers
    atomicAdd(&S.prof[2], (unsigned long long)(c3 - c2));     // trace
    atomicAdd(&S.prof[3], (unsigned long long)(c4 - c3));     // flush
    atomicAdd(&S.prof[4], (unsigned long long)n);
    atomicAdd(&S.prof[7], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - r0));   // 100 MHz ticks
    const uint32_t st = (uint32_t)S.ri[GG_RI_STEPS];
    if (st < S.prof_steps) atomicMax(&S.prof[16 + st], (unsigned long long)(c4 - c0));
  }
}

// A step's messages: network latency (closed form, or the arrival the
// hop-by-hop pipeline computed), then delivery (same shard: the next step's
// inbox list; otherwise the quantum-boundary buffer).
__global__ void k_c_route(CP P, CS S, int p, const uint64_t* hbh_arrival)
{
  if (*(volatile uint32_t*)S.quiet) return;
  const int po = 1 - p;
  const uint32_t n = min(S.cnt[po], (uint32_t)P.msg_cap);
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid == 0) {
    if (n == 0) *S.quiet = 1;
    S.cnt[p] = 0;                                  // the outbox of the next step
  }
  gg_cmsg* B = bufp(S, po);
  int32_t* head = headp(S, po);
  for (uint32_t i = gid; i < n; i += gridDim.x * blockDim.x) {
    gg_cmsg m = B[i];
    if (hbh_arrival) {
      m.arrival_ps = hbh_arrival[i];
    } else {
      uint64_t zl;
      m.arrival_ps = route_closed_form(P.np, m.src, m.dst, has_data(m.type) ? P.bits_data : P.bits_req,
                                       m.send_ps, zl, S.ctr);
    }
    atomicAdd((unsigned long long*)&S.ri[m.src == m.dst ? GG_RI_SELF_MSGS : GG_RI_NET_MSGS], 1ull);
    const uint32_t ss = (uint32_t)(((uint64_t)m.src * P.K) / P.T), ds = (uint32_t)(((uint64_t)m.dst * P.K) / P.T);
    if (ss == ds) {
      m.link = (uint32_t)atomicExch(&head[m.dst - P.tb], (int32_t)i);
      B[i] = m;
    } else {
      const uint32_t j = atomicAdd(S.bnd_cnt, 1u);
      if (j >= P.msg_cap) { atomicOr(S.err, GG_DERR_CAP); continue; }
      S.bnd[j] = m;
      atomicAdd((unsigned long long*)&S.ri[GG_RI_BOUNDARY_MSGS], 1ull);
    }
  }
}

// hop-by-hop: the step's messages as packets, keyed (send time, sender, sequence)
// — the order the oracle routes a step's batch in (oracle/gg_coherent.inc c_route_step)
__global__ void k_c_packets(CP P, CS S, int p)
{
  if (*(volatile uint32_t*)S.quiet) return;
  const int po = 1 - p;
  const uint32_t n = min(S.cnt[po], (uint32_t)P.msg_cap);
  const gg_cmsg* B = bufp(S, po);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const gg_cmsg m = B[i];
    S.pk_src[i] = m.src; S.pk_dst[i] = m.dst;
    S.pk_len[i] = has_data(m.type) ? P.bits_data : P.bits_req;
    S.pk_t0[i] = m.send_ps; S.pk_khi[i] = m.send_ps; S.pk_klo[i] = ((uint64_t)m.src << 32) | m.seq;
  }
}

// Deliver imported (boundary) messages into the inbox of the quantum's first step.
__global__ void k_c_import(CP P, CS S, const gg_cmsg* in, uint32_t n)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  gg_cmsg m = in[i];
  if (m.dst < P.tb || m.dst >= P.tb + P.lt) { atomicOr(S.err, GG_DERR_STATE); return; }
  m.link = (uint32_t)atomicExch(&S.head0[m.dst - P.tb], (int32_t)i);
  S.buf0[i] = m;
}

// Status after a quantum: active / blocked tiles, least next-access start.
__global__ void k_c_status(CP P, CS S, uint64_t* out /* [active, blocked, min_next] */)
{
  const uint32_t lt = blockIdx.x * blockDim.x + threadIdx.x;
  if (lt >= P.lt) return;
  const uint64_t r = S.rec[lt];
  if (r >= S.rec_end[lt]) return;
  atomicAdd((unsigned long long*)&out[0], 1ull);
  if (S.blocked[lt]) { atomicAdd((unsigned long long*)&out[1], 1ull); return; }
  const uint64_t s = S.clk[lt] + (uint64_t)((S.meta[r] & 0x7FFFFFFFu) >> 1) * P.gap_ps;
  atomicMin((unsigned long long*)&out[2], (unsigned long long)s);
}

__global__ void k_c_reset(CP P, CS S, const uint64_t* offs)
{
  const uint32_t lt = blockIdx.x * blockDim.x + threadIdx.x;
  if (lt >= P.lt) return;
  for (uint32_t i = 0; i < P.s1 * P.a1; ++i) { S.l1_tag[(size_t)lt * P.s1 * P.a1 + i] = INV_ADDR;
                                               S.l1_meta[(size_t)lt * P.s1 * P.a1 + i] = (uint8_t)((i % P.a1) << 3); }
  for (uint32_t i = 0; i < P.s1; ++i) S.l1_rr[(size_t)lt * P.s1 + i] = (uint8_t)(P.a1 - 1);
  for (uint32_t i = 0; i < P.s2 * P.a2; ++i) { S.l2_tag[(size_t)lt * P.s2 * P.a2 + i] = INV_ADDR;
                                               S.l2_meta[(size_t)lt * P.s2 * P.a2 + i] = (uint8_t)((i % P.a2) << 3); }
  for (uint32_t i = 0; i < P.s2; ++i) S.l2_rr[(size_t)lt * P.s2 + i] = (uint8_t)(P.a2 - 1);
  for (uint32_t i = 0; i < 2 * GG_NUM_CACHE_COUNTERS; ++i) S.cc[(size_t)lt * 2 * GG_NUM_CACHE_COUNTERS + i] = 0;
  for (uint32_t i = 0; i < GG_NUM_TILE_STATS; ++i) S.st[(size_t)lt * GG_NUM_TILE_STATS + i] = 0;
  for (uint32_t i = 0; i < P.E; ++i) S.dir[(size_t)lt * P.E + i] = DEnt{INV_ADDR, -1, DS_UNCACHED, 0};
  for (uint64_t i = 0; i < (uint64_t)P.E * P.W; ++i) S.dsh[(size_t)lt * P.E * P.W + i] = 0;
  S.nrep[lt] = 0; S.nrq[lt] = 0;
  const uint32_t tile = P.tb + lt;
  S.rec[lt] = offs[tile]; S.rec_end[lt] = offs[tile + 1];
  S.clk[lt] = 0; S.pend_start[lt] = 0; S.out_addr[lt] = INV_ADDR; S.out_time[lt] = 0;
  S.blocked[lt] = 0; S.seq[lt] = 0;
  S.head0[lt] = -1; S.head1[lt] = -1;
  if (P.dram_qm)                                     // QueueModel::create(dram/queue_model/type, min_processing_time)
    hq_init(S.dq + lt, S.dnd + (size_t)lt * P.max_list, S.dfl + (size_t)lt * P.max_list, P.max_list, P.dram_qtype,
            P.dram_qaux);
}

__global__ void k_c_final_stats(CP P, CS S)
{
  const uint32_t lt = blockIdx.x * blockDim.x + threadIdx.x;
  if (lt >= P.lt || !P.dram_qm) return;
  S.st[(size_t)lt * GG_NUM_TILE_STATS + GG_CT_DRAM_QUEUE_ANALYTICAL] = S.dq[lt].analytical;
  S.st[(size_t)lt * GG_NUM_TILE_STATS + GG_CT_DRAM_QUEUE_UTILIZED_NS] = S.dq[lt].util;
  S.st[(size_t)lt * GG_NUM_TILE_STATS + GG_CT_DRAM_QUEUE_LAST_NS] = S.dq[lt].last_req;
}

// export: group the boundary messages by destination shard
__global__ void k_c_export_count(CP P, const gg_cmsg* b, uint32_t n, uint32_t* counts)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd(&counts[((uint64_t)b[i].dst * P.K) / P.T], 1u);
}
__global__ void k_c_export_scatter(CP P, const gg_cmsg* b, uint32_t n, const uint32_t* base, uint32_t* cursor,
                                   gg_cmsg* out)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = (uint32_t)(((uint64_t)b[i].dst * P.K) / P.T);
  out[base[k] + atomicAdd(&cursor[k], 1u)] = b[i];
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct gg_coh_state {
  CP P{};
  CS S{};
  std::vector<void*> allocs;
  uint64_t* status_dev = nullptr;
  uint32_t* ecount_dev = nullptr;    // export counts + cursors
  uint64_t* offs_dev = nullptr;
  uint64_t n_records = 0;
  bool begun = false;
};

static int ilog2(uint64_t v) { int p = -1; while (v) { v >>= 1; ++p; } return p; }
static int clog2(uint64_t v) { int p = ilog2(v); return ((1ull << p) == v) ? p : p + 1; }
static uint64_t lat_ps_host(uint64_t cycles, double f) { return (uint64_t)ceil(((double)1000 * cycles) / f); }

template <class T> static gg_status dalloc(gg_coh_state* C, T** p, uint64_t n)
{
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (n ? n : 1));
  if (e != hipSuccess) return gg_hip_check(e, "hipMalloc(coherent state)");
  C->allocs.push_back((void*)*p);
  return GG_OK;
}

void gg_coh_free(gg_ctx* ctx)
{
  gg_coh_state* C = ctx->coh;
  if (!C) return;
  for (void* p : C->allocs) hipFree(p);
  delete C;
  ctx->coh = nullptr;
}

static gg_status coh_alloc(gg_ctx* ctx)
{
  if (ctx->coh) return GG_OK;
  const gg_config& c = ctx->cfg;
  gg_coh_state* C = new gg_coh_state();
  ctx->coh = C;
  CP& P = C->P;
  P.T = c.num_tiles;
  P.K = c.num_shards ? c.num_shards : 1;
  const uint32_t k0 = c.shard_begin, k1 = c.shard_end ? c.shard_end : P.K;
  if (k0 >= k1 || k1 > P.K || P.K > P.T) return gg_fail(GG_ERR_INVALID, "bad shard range [%u, %u) of %u", k0, k1, P.K);
  // tiles of shard k: { t : t*K/T == k } = [ceil(k*T/K), ceil((k+1)*T/K))
  P.tb = (uint32_t)(((uint64_t)k0 * P.T + P.K - 1) / P.K);
  const uint32_t te = (uint32_t)(((uint64_t)k1 * P.T + P.K - 1) / P.K);
  P.lt = te - P.tb;
  if (c.net_model == GG_NET_EMESH_HOP_BY_HOP && P.K > 1)
    return gg_fail(GG_ERR_UNSUPPORTED, "coherent mode: emesh_hop_by_hop with more than one logical shard "
                   "(router queues split by shard) is not built yet");
  if (c.l1d_assoc > 31 || c.l2_assoc > 31) return gg_fail(GG_ERR_UNSUPPORTED, "coherent mode: associativity above 31");
  P.log_line = (uint32_t)ilog2(c.line_size);
  P.s1 = c.l1d_size_kb * 1024u / (c.l1d_assoc * c.line_size); P.a1 = c.l1d_assoc; P.pol1 = c.l1d_policy;
  P.s2 = c.l2_size_kb * 1024u / (c.l2_assoc * c.line_size); P.a2 = c.l2_assoc; P.pol2 = c.l2_policy;
  const double f = c.frequency_ghz;
  P.lat_l1d = lat_ps_host(c.l1d_data_cycles, f); P.lat_l1t = lat_ps_host(c.l1d_tags_cycles, f);
  P.lat_l2d = lat_ps_host(c.l2_data_cycles, f); P.lat_l2t = lat_ps_host(c.l2_tags_cycles, f);
  P.gap_ps = lat_ps_host(1, f);
  // DirectoryCache sizing and access time (directory_cache.cc:46-90, 243-322)
  P.dassoc = c.dir_assoc;
  const uint32_t slices = P.T;
  uint32_t entries;
  if (c.dir_total_entries == 0) {
    uint32_t sets = (uint32_t)ceil(2.0 * c.l2_size_kb * 1024 * P.T / (64.0 * c.dir_assoc * slices));
    sets = 1u << clog2(sets);
    entries = sets * c.dir_assoc;
  } else entries = c.dir_total_entries;
  P.E = entries;
  const uint32_t dsets = entries / c.dir_assoc;
  if (dsets == 0 || (dsets & (dsets - 1))) return gg_fail(GG_ERR_UNSUPPORTED, "directory sets must be a power of two");
  P.log_dsets = (uint32_t)ilog2(dsets);
  P.log_slices = (uint32_t)clog2(slices);
  const uint64_t dir_size = (uint64_t)entries * (uint64_t)ceil(1.0 * P.T / 8);
  uint64_t cyc = c.dir_access_cycles;
  if (cyc == 0) {
    const uint32_t kb = (uint32_t)ceil(1.0 * dir_size / 1024);
    cyc = kb <= 16 ? 1 : kb <= 32 ? 2 : kb <= 64 ? 4 : kb <= 128 ? 6 : kb <= 256 ? 8 :
          kb <= 512 ? 10 : kb <= 1024 ? 13 : kb <= 2048 ? 16 : 20;
  }
  P.lat_dir = lat_ps_host(cyc, f);
  P.W = (P.T + 63) / 64;
  P.R = 64;
  P.QC = P.T + P.R + 8;
  P.IC = 2 * P.T + 256;
  const uint32_t idb = P.T > 1 ? (uint32_t)clog2(P.T) : 0;
  P.bits_req = 2 * idb + 4 + 48;
  P.bits_data = P.bits_req + 8 * c.line_size;
  P.dram_qm = c.dram_queue_model_enabled;
  P.dram_qtype = c.dram_queue_model_type;
  P.dram_qaux = hq_aux(c.dram_queue_model_type, c.basic_moving_avg, c.history_list_no_interleaving);
  if (P.dram_qm)
    if (gg_status e = gg_check_queue_model(P.dram_qtype, P.dram_qaux, c.max_list_size ? c.max_list_size : 100)) return e;
  P.max_list = c.max_list_size ? c.max_list_size : 100;
  P.analytical = c.analytical_enabled;
  P.dram_proc = (uint64_t)((float)c.line_size / c.dram_bandwidth) + 1;
  P.dram_cost = (uint64_t)(float)c.dram_latency_ns;
  P.msg_cap = (uint64_t)64 * P.T + 65536;
  // a wave per tile (default; GG_COH_TILES_PER_BLOCK=64 packs a lane per tile, for A/B runs)
  { const char* e = getenv("GG_COH_TILES_PER_BLOCK"); P.tiles_per_block = (e && atoi(e) == 64) ? 64 : 1; }
  {
    const uint64_t rq = (uint64_t)P.QC * sizeof(CReq);
    const char* r = getenv("GG_COH_STAGE_RQ");
    P.stage_rq = (P.tiles_per_block == 1 && rq <= 48 * 1024 && !(r && atoi(r) == 0)) ? 1 : 0;
  }
  if (getenv("GG_COH_PROFILE") && atoi(getenv("GG_COH_PROFILE"))) {
    C->S.prof_steps = 1u << 16;
    if (gg_status st = dalloc(C, &C->S.prof, 16 + C->S.prof_steps)) return st;
    GG_HIP(hipMemset(C->S.prof, 0, sizeof(unsigned long long) * (16 + C->S.prof_steps)));
  }
  P.np = gg_noc_params(ctx);
  const uint64_t L = P.lt;
  CS& S = C->S;
  gg_status st = GG_OK;
#define A(ptr, n) if (st == GG_OK) st = dalloc(C, &S.ptr, (n))
  A(l1_tag, L * P.s1 * P.a1); A(l1_meta, L * P.s1 * P.a1); A(l1_rr, L * P.s1);
  A(l2_tag, L * P.s2 * P.a2); A(l2_meta, L * P.s2 * P.a2); A(l2_rr, L * P.s2);
  A(cc, L * 2 * GG_NUM_CACHE_COUNTERS); A(st, L * GG_NUM_TILE_STATS);
  A(rec, L); A(rec_end, L); A(clk, L); A(pend_start, L); A(out_addr, L); A(out_time, L);
  A(blocked, L); A(seq, L);
  A(dir, L * P.E); A(dsh, L * P.E * P.W);
  A(rep, L * P.R); A(rsh, L * P.R * P.W); A(nrep, L);
  A(rq, L * P.QC); A(nrq, L);
  A(dq, L); A(dnd, L * P.max_list); A(dfl, L * P.max_list);
  A(buf0, P.msg_cap); A(buf1, P.msg_cap); A(cnt, 2);
  A(head0, L); A(head1, L);
  A(bnd, P.msg_cap); A(bnd_cnt, 1);
  A(scratch, L * P.IC);
  A(quiet, 1); A(ri, GG_NUM_RUN_INFO);
  const uint64_t pk = (c.net_model == GG_NET_EMESH_HOP_BY_HOP) ? P.msg_cap : 1;
  A(pk_src, pk); A(pk_dst, pk); A(pk_len, pk); A(pk_t0, pk); A(pk_khi, pk); A(pk_klo, pk);
#undef A
  if (st == GG_OK) st = dalloc(C, &C->status_dev, 4);
  if (st == GG_OK) st = dalloc(C, &C->ecount_dev, 2 * (uint64_t)P.K + 2);
  if (st == GG_OK) st = dalloc(C, &C->offs_dev, (uint64_t)P.T + 1);
  S.ctr = gg_noc_ctr(ctx);
  S.err = ctx->err_dev;
  return st;
}

static gg_status coh_check(gg_ctx* ctx)
{
  uint32_t e = 0;
  GG_HIP(hipMemcpy(&e, ctx->err_dev, sizeof(e), hipMemcpyDeviceToHost));
  if (e & GG_DERR_CAP) return gg_fail(GG_ERR_UNSUPPORTED, "coherent mode: a device capacity (messages / inbox / "
                                      "request queue / replaced entries / call chain) was exceeded");
  if (e & GG_DERR_STATE) return gg_fail(GG_ERR_STATE, "coherent mode: a state the reference would reject "
                                        "(LOG_ASSERT_ERROR / assert)");
  return GG_OK;
}

gg_status gg_coherent_begin(gg_ctx* ctx, const gg_trace* tr, uint64_t* access_out_dev, void* stream)
{
  if (!ctx || !tr || !tr->tile_offsets) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  ctx->last_stream = s;
  if (gg_status st = coh_alloc(ctx)) return st;
  gg_coh_state* C = ctx->coh;
  const CP& P = C->P;
  if (tr->tile_offsets[P.T] != tr->num_records) return gg_fail(GG_ERR_INVALID, "tile_offsets[num_tiles] != num_records");
  for (uint32_t t = 0; t < P.T; ++t)
    if (tr->tile_offsets[t] > tr->tile_offsets[t + 1]) return gg_fail(GG_ERR_INVALID, "tile_offsets not monotone");
  if (tr->num_records && (!tr->addr_dev || !tr->meta_dev)) return gg_fail(GG_ERR_INVALID, "NULL trace pointers");
  C->S.addr = tr->addr_dev; C->S.meta = tr->meta_dev; C->S.out = access_out_dev;
  C->n_records = tr->num_records;
  GG_HIP(hipMemcpyAsync(C->offs_dev, tr->tile_offsets, sizeof(uint64_t) * (P.T + 1), hipMemcpyHostToDevice, s));
  if (gg_status st = gg_noc_reset(ctx, s)) return st;
  GG_HIP(hipMemsetAsync(ctx->err_dev, 0, sizeof(uint32_t), s));
  GG_HIP(hipMemsetAsync(C->S.ri, 0, sizeof(uint64_t) * GG_NUM_RUN_INFO, s));
  GG_HIP(hipMemsetAsync(C->S.cnt, 0, sizeof(uint32_t) * 2, s));
  GG_HIP(hipMemsetAsync(C->S.bnd_cnt, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_c_reset, dim3((P.lt + 63) / 64), dim3(64), 0, s, P, C->S, (const uint64_t*)C->offs_dev);
  GG_HIP(hipGetLastError());
  GG_HIP(hipStreamSynchronize(s));
  C->begun = true;
  return coh_check(ctx);
}

gg_status gg_coherent_quantum(gg_ctx* ctx, uint64_t q, gg_coherent_status* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  gg_coh_state* C = ctx->coh;
  if (!C || !C->begun) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  const CP& P = C->P;
  const uint64_t quantum_ps = (uint64_t)ctx->cfg.quantum_ns * 1000ull;
  const uint64_t barrier = (q + 1) * quantum_ps;
  GG_HIP(hipMemsetAsync(C->S.quiet, 0, sizeof(uint32_t), s));
  const uint32_t tb = (P.lt + 63) / 64;
  const uint32_t rb = (uint32_t)std::min<uint64_t>((P.msg_cap + 255) / 256, 1024);
  const uint32_t dyn_lds = P.stage_rq ? P.QC * (uint32_t)sizeof(CReq) : 0u;
  if (dyn_lds)
    GG_HIP(hipFuncSetAttribute((const void*)k_c_tiles, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(dyn_lds + sizeof(TreeLds) + 16)));
  uint64_t steps = 0;
  uint32_t batch = 8;
  for (;;) {
    for (uint32_t k = 0; k < batch; ++k) {
      const int p = (int)((steps + k) & 1);
      if (P.tiles_per_block == 1)
        hipLaunchKernelGGL(k_c_tiles, dim3(P.lt), dim3(64), dyn_lds, s, P, C->S, p, barrier);
      else
        hipLaunchKernelGGL(k_c_tiles, dim3(tb), dim3(64), 0, s, P, C->S, p, barrier);
      if (ctx->cfg.net_model == GG_NET_EMESH_HOP_BY_HOP) {
        hipLaunchKernelGGL(k_c_packets, dim3(rb), dim3(256), 0, s, P, C->S, p);
        if (gg_status e = gg_noc_hbh(ctx, C->S.pk_src, C->S.pk_dst, C->S.pk_len, C->S.pk_t0, C->S.pk_khi,
                                     C->S.pk_klo, P.msg_cap, C->S.cnt + (1 - p), s))
          return e;
        hipLaunchKernelGGL(k_c_route, dim3(rb), dim3(256), 0, s, P, C->S, p, gg_noc_packet_times(ctx));
      } else {
        hipLaunchKernelGGL(k_c_route, dim3(rb), dim3(256), 0, s, P, C->S, p, (const uint64_t*)nullptr);
      }
    }
    GG_HIP(hipGetLastError());
    steps += batch;
    uint32_t quiet = 0, err = 0;
    GG_HIP(hipMemcpyAsync(&quiet, C->S.quiet, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GG_HIP(hipMemcpyAsync(&err, ctx->err_dev, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    if (err) return coh_check(ctx);
    if (quiet) break;
    if (batch < 64) batch *= 2;
  }
  uint64_t init[4] = {0, 0, ~0ull, 0};
  GG_HIP(hipMemcpyAsync(C->status_dev, init, sizeof(init), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_c_status, dim3(tb), dim3(64), 0, s, P, C->S, C->status_dev);
  GG_HIP(hipGetLastError());
  uint64_t res[4];
  uint32_t nb = 0;
  uint64_t ri[GG_NUM_RUN_INFO];
  GG_HIP(hipMemcpyAsync(res, C->status_dev, sizeof(res), hipMemcpyDeviceToHost, s));
  GG_HIP(hipMemcpyAsync(&nb, C->S.bnd_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  GG_HIP(hipMemcpyAsync(ri, C->S.ri, sizeof(ri), hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  ri[GG_RI_QUANTA]++;
  ri[GG_RI_FINAL_QUANTUM] = q;
  GG_HIP(hipMemcpyAsync(C->S.ri, ri, sizeof(ri), hipMemcpyHostToDevice, s));
  out->steps = 0;
  out->boundary_msgs = nb;
  out->min_next_ps = res[2];
  out->active_tiles = (uint32_t)res[0];
  out->blocked_tiles = (uint32_t)res[1];
  return coh_check(ctx);
}

gg_status gg_coherent_export(gg_ctx* ctx, gg_cmsg* out_dev, uint64_t cap, uint64_t* per_shard_counts)
{
  if (!ctx || !per_shard_counts) return gg_fail(GG_ERR_INVALID, "NULL argument");
  gg_coh_state* C = ctx->coh;
  if (!C || !C->begun) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  const CP& P = C->P;
  uint32_t nb = 0;
  GG_HIP(hipMemcpy(&nb, C->S.bnd_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (nb > cap) return gg_fail(GG_ERR_RANGE, "export buffer holds %llu messages, %u waiting",
                               (unsigned long long)cap, nb);
  if (nb && !out_dev) return gg_fail(GG_ERR_INVALID, "NULL export buffer");
  std::vector<uint32_t> counts(P.K, 0), base(P.K, 0);
  if (nb) {
    GG_HIP(hipMemsetAsync(C->ecount_dev, 0, sizeof(uint32_t) * 2 * P.K, s));
    hipLaunchKernelGGL(k_c_export_count, dim3((nb + 255) / 256), dim3(256), 0, s, P, C->S.bnd, nb, C->ecount_dev);
    GG_HIP(hipMemcpyAsync(counts.data(), C->ecount_dev, sizeof(uint32_t) * P.K, hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    uint32_t a = 0;
    for (uint32_t k = 0; k < P.K; ++k) { base[k] = a; a += counts[k]; }
    GG_HIP(hipMemcpyAsync(C->ecount_dev, base.data(), sizeof(uint32_t) * P.K, hipMemcpyHostToDevice, s));
    GG_HIP(hipMemsetAsync(C->ecount_dev + P.K, 0, sizeof(uint32_t) * P.K, s));
    hipLaunchKernelGGL(k_c_export_scatter, dim3((nb + 255) / 256), dim3(256), 0, s, P, C->S.bnd, nb,
                       C->ecount_dev, C->ecount_dev + P.K, out_dev);
    GG_HIP(hipGetLastError());
  }
  GG_HIP(hipMemsetAsync(C->S.bnd_cnt, 0, sizeof(uint32_t), s));
  GG_HIP(hipStreamSynchronize(s));
  for (uint32_t k = 0; k < P.K; ++k) per_shard_counts[k] = counts[k];
  return GG_OK;
}

gg_status gg_coherent_import(gg_ctx* ctx, const gg_cmsg* in_dev, uint64_t n)
{
  if (!ctx) return gg_fail(GG_ERR_INVALID, "NULL argument");
  gg_coh_state* C = ctx->coh;
  if (!C || !C->begun) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  if (n == 0) return GG_OK;
  if (!in_dev) return gg_fail(GG_ERR_INVALID, "NULL import buffer");
  if (n > C->P.msg_cap) return gg_fail(GG_ERR_UNSUPPORTED, "import of %llu messages beyond the step buffer",
                                       (unsigned long long)n);
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  // the quantum's first step reads buffer 0; its outbox (buffer 1) starts empty
  GG_HIP(hipMemsetAsync(C->S.cnt + 1, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_c_import, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, C->P, C->S, in_dev, (uint32_t)n);
  GG_HIP(hipGetLastError());
  GG_HIP(hipStreamSynchronize(s));
  return coh_check(ctx);
}

gg_status gg_coherent_run(gg_ctx* ctx, const gg_trace* tr, uint64_t* access_out_dev, void* stream)
{
  if (!ctx) return gg_fail(GG_ERR_INVALID, "NULL argument");
  const gg_config& c = ctx->cfg;
  const uint32_t K = c.num_shards ? c.num_shards : 1;
  if (c.shard_begin != 0 || (c.shard_end != 0 && c.shard_end != K))
    return gg_fail(GG_ERR_INVALID, "gg_coherent_run needs a context that owns every shard");
  if (gg_status st = gg_coherent_begin(ctx, tr, access_out_dev, stream)) return st;
  gg_coh_state* C = ctx->coh;
  hipStream_t s = ctx->last_stream;
  const uint64_t quantum_ps = (uint64_t)c.quantum_ns * 1000ull;
  gg_timer_begin(ctx, "coherent_run", s);
  uint64_t q = 0;
  for (;;) {
    gg_coherent_status st;
    if (gg_status e = gg_coherent_quantum(ctx, q, &st)) return e;
    const uint64_t nb = st.boundary_msgs;
    if (nb) {                                          // the boundary: held messages -> next inboxes
      GG_HIP(hipMemcpyAsync(C->S.buf1, C->S.bnd, sizeof(gg_cmsg) * nb, hipMemcpyDeviceToDevice, s));
      GG_HIP(hipMemsetAsync(C->S.bnd_cnt, 0, sizeof(uint32_t), s));
      if (gg_status e = gg_coherent_import(ctx, C->S.buf1, nb)) return e;
    }
    if (st.active_tiles == 0 && nb == 0) break;
    if (nb == 0 && st.blocked_tiles == 0) {
      const uint64_t nq = st.min_next_ps / quantum_ps;
      q = nq > q + 1 ? nq : q + 1;
    } else if (nb == 0) {
      return gg_fail(GG_ERR_STATE, "coherent run deadlocked: tiles blocked with no message in flight");
    } else {
      q = q + 1;
    }
  }
  gg_timer_end(ctx, "coherent_run", s);
  GG_HIP(hipStreamSynchronize(s));
  if (C->S.prof) {
    std::vector<unsigned long long> h(16 + C->S.prof_steps);
    GG_HIP(hipMemcpy(h.data(), C->S.prof, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    unsigned long long crit = 0, nst = 0;
    for (uint32_t i = 0; i < C->S.prof_steps; ++i) { crit += h[16 + i]; nst += h[16 + i] ? 1 : 0; }
    fprintf(stderr, "[gg_coh] tile-step cycles summed over tiles: gather+sort %llu handlers %llu (directory %llu, L2 %llu)"
            " trace %llu flush %llu | msgs %llu | critical path (max tile per step, %llu steps) %llu cycles"
            " | memtime/memrealtime %.1f MHz | dget %llu dram %llu send %llu\n",
            h[0], h[1], h[5], h[6], h[2], h[3], h[4], nst, crit,
            h[7] ? 100.0 * (double)(h[0] + h[1] + h[2] + h[3]) / (double)h[7] : 0.0, h[9], h[10], h[11]);
  }
  return coh_check(ctx);
}

gg_status gg_coherent_get_stats(gg_ctx* ctx, uint64_t* tile_stats, uint64_t* cache, uint64_t* run_info)
{
  if (!ctx) return gg_fail(GG_ERR_INVALID, "NULL argument");
  gg_coh_state* C = ctx->coh;
  if (!C) return gg_fail(GG_ERR_INVALID, "no coherent run on this context");
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  const CP& P = C->P;
  hipLaunchKernelGGL(k_c_final_stats, dim3((P.lt + 63) / 64), dim3(64), 0, s, P, C->S);
  GG_HIP(hipGetLastError());
  GG_HIP(hipStreamSynchronize(s));
  if (tile_stats) {
    std::memset(tile_stats, 0, sizeof(uint64_t) * P.T * GG_NUM_TILE_STATS);
    GG_HIP(hipMemcpy(tile_stats + (size_t)P.tb * GG_NUM_TILE_STATS, C->S.st,
                     sizeof(uint64_t) * P.lt * GG_NUM_TILE_STATS, hipMemcpyDeviceToHost));
  }
  if (cache) {
    std::memset(cache, 0, sizeof(uint64_t) * P.T * 2 * GG_NUM_CACHE_COUNTERS);
    GG_HIP(hipMemcpy(cache + (size_t)P.tb * 2 * GG_NUM_CACHE_COUNTERS, C->S.cc,
                     sizeof(uint64_t) * P.lt * 2 * GG_NUM_CACHE_COUNTERS, hipMemcpyDeviceToHost));
  }
  if (run_info) GG_HIP(hipMemcpy(run_info, C->S.ri, sizeof(uint64_t) * GG_NUM_RUN_INFO, hipMemcpyDeviceToHost));
  return coh_check(ctx);
}
