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
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <type_traits>

namespace {

constexpr uint32_t kChunk = 1024;        // records per shard chunk (one wave, staged in LDS)
constexpr uint32_t kPerLane = kChunk / 64;
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
    const uint32_t* __restrict__ meta, const uint32_t* __restrict__ chunk_tile, const uint64_t* __restrict__ chunk_start,
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
    bad |= meta[start + i] == GG_META_BARRIER ? 2u : 0u;              // coherent-mode records only
    atomicAdd(&h[(a >> g.log_line) & (g.u1 - 1)], 1u);
  }
  if (bad & 1u) atomicOr(err, GG_DERR_RANGE);
  if (bad & 2u) atomicOr(err, GG_DERR_BARRIER);
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < g.u1; s += blockDim.x) cnt[(uint64_t)c * g.u1 + s] = h[s];
}

// Pass 2: per tile, exclusive scan over its chunks per set (in place) and the
// unit lengths.
__global__ void k_shard_scan(uint32_t* __restrict__ cnt, const uint32_t* __restrict__ tile_chunk0,
                             uint32_t* __restrict__ unit_len, gg_geom g)
{
  const uint32_t t = blockIdx.x, s = threadIdx.x;
  if (s >= g.u1) return;
  uint64_t acc = 0;
  for (uint32_t c = tile_chunk0[t]; c < tile_chunk0[t + 1]; ++c) {
    uint32_t* p = &cnt[(uint64_t)c * g.u1 + s];
    const uint32_t v = *p;
    *p = (uint32_t)acc;
    acc += v;
  }
  unit_len[(uint64_t)t * g.u1 + s] = (uint32_t)acc;
}

// Pass 2b: unit-contiguous sharded layout.  Unit u's records are stored
// contiguously from unit_base[u], each unit padded to a multiple of 8 records
// so a lane streams its records in 64-byte blocks.  One block; writes the
// total slot count to *total.
__global__ __launch_bounds__(1024) void k_unit_scan(const uint32_t* __restrict__ unit_len, uint64_t units,
                                                    uint64_t* __restrict__ unit_base, uint64_t* __restrict__ total)
{
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (units + blockDim.x - 1) / blockDim.x;
  const uint64_t u0 = t * per, u1 = min(units, u0 + per);
  uint64_t sum = 0;
  for (uint64_t u = u0; u < u1; ++u) sum += (unit_len[u] + 7u) & ~7u;
  part[t] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < blockDim.x; o <<= 1) {
    const uint64_t v = (t >= o) ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t base = part[t] - sum;
  if (t == blockDim.x - 1) *total = part[t];
  for (uint64_t u = u0; u < u1; ++u) { unit_base[u] = base; base += (unit_len[u] + 7u) & ~7u; }
}

// Sharded record ("replay key"), built once by the scatter so the replay
// decodes nothing wider than 32 bits:
//   bits 63..32  L2 tag (line >> log2 L2 sets, < 2^32 by gg_geom::addr_limit)
//   bits 16..25  L1-D set (line mod u1; used by the scatter's write-out only)
//   bits  1..15  L2 set within the unit ((line >> log2 u1) mod S2)
//   bit   0      WRITE
__device__ __forceinline__ uint64_t replay_key(uint64_t a, uint32_t m, const gg_geom& g)
{
  const uint64_t line = a >> g.log_line;
  const uint32_t lo = (m & GG_META_WRITE) | (((uint32_t)(line >> g.log_u1) & (g.s2 - 1)) << 1) |
                      (((uint32_t)line & (g.u1 - 1)) << 16);
  return ((uint64_t)(uint32_t)(line >> g.log_l2) << 32) | lo;
}
__device__ __forceinline__ uint32_t key_l1set(uint64_t k, uint32_t smask) { return ((uint32_t)k >> 16) & smask; }

// Workgroup -> chunk map that gives each XCD a contiguous range of chunks.
// Workgroups are dealt round-robin to the 8 XCDs (blockIdx % 8); mapping
// XCD x to chunks [x*q + min(x,r), ...) keeps adjacent chunks of a tile on the
// same XCD, so the partial cache lines at the ends of their per-set runs
// merge in that XCD's L2 instead of being written back half-filled.
__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t n)
{
  const uint32_t q = n / GG_NUM_XCD, r = n % GG_NUM_XCD, x = b % GG_NUM_XCD, k = b / GG_NUM_XCD;
  return x * q + min(x, r) + k;
}

// Pass 3: one wave per chunk of kChunk records.  The chunk's keys are held in
// VGPRs, counted per L1-D set with LDS atomics, ranked in program order (lanes
// with the same set matched by log2(u1) ballots, so each unit keeps program
// order), staged in LDS sorted by set, then written out per set as contiguous
// runs (consecutive lanes -> consecutive addresses).  Each record's slot goes
// to rec_slot[] in program order (coalesced), for k_unshard.
//
// Persistent: workgroup b walks chunks b, b+G, b+2G, ... (G = gridDim.x, a
// multiple of 8, so every chunk of a workgroup lies in its XCD's range), and
// the next chunk's addr/meta loads are in flight while the current chunk is
// ranked and written.  The workgroup is one wave, so LDS hand-offs between
// phases need only a wave barrier (LDS instructions of a wave execute in order).
template <int PER, bool PERSIST>    // PER = L1-D sets per lane: max(1, u1 / 64)
__global__ __launch_bounds__(64) void k_shard_scatter(const uint64_t* __restrict__ addr,
    const uint32_t* __restrict__ meta, const uint32_t* __restrict__ chunk_tile,
    const uint64_t* __restrict__ chunk_start, const uint32_t* __restrict__ chunk_len,
    const uint32_t* __restrict__ cnt, const uint64_t* __restrict__ unit_base,
    uint64_t* __restrict__ sh_key, uint32_t* __restrict__ rec_slot, gg_geom g, uint32_t nchunks)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t* skey = reinterpret_cast<uint64_t*>(smem);                      // [kChunk]
  uint64_t* dbase = skey + kChunk;                                         // [u1] dest - local offset
  uint32_t* lcnt = reinterpret_cast<uint32_t*>(dbase + g.u1);             // [u1] count, then running rank
  uint32_t* loff = lcnt + g.u1;                                            // [u1] exclusive prefix
  const uint32_t lane = threadIdx.x, G = gridDim.x;
  const uint32_t smask = g.u1 - 1;
  const uint64_t lt_mask = (1ull << lane) - 1;
  auto wave_sync = [] { __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); };

  uint32_t i = blockIdx.x;
  if (i >= nchunks) return;
  uint32_t c = xcd_chunk(i, nchunks);
  uint64_t pa[kPerLane];
  uint32_t pm[kPerLane];
  auto issue = [&](uint32_t cc) {
    const uint64_t st = chunk_start[cc];
    const uint32_t ln = chunk_len[cc];
#pragma unroll
    for (uint32_t k = 0; k < kPerLane; ++k) {
      const uint32_t j = k * GG_WAVE + lane;
      pa[k] = (j < ln) ? addr[st + j] : 0;
      pm[k] = (j < ln) ? meta[st + j] : 0;
    }
  };
  issue(c);
  for (;;) {
    const uint32_t t = chunk_tile[c];
    const uint64_t start = chunk_start[c];
    const uint32_t len = chunk_len[c];
    // this chunk's per-set bases (issued before the next chunk's prefetch)
    uint64_t ub[PER];
    uint32_t cb[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t s = lane * PER + k;
      ub[k] = (s < g.u1) ? unit_base[(uint64_t)t * g.u1 + s] : 0;
      cb[k] = (s < g.u1) ? cnt[(uint64_t)c * g.u1 + s] : 0;
    }
    uint64_t key[kPerLane];
#pragma unroll
    for (uint32_t k = 0; k < kPerLane; ++k) key[k] = replay_key(pa[k], pm[k], g);
    const uint32_t inext = i + G;
    const bool more = PERSIST && inext < nchunks;
    const uint32_t cn = more ? xcd_chunk(inext, nchunks) : c;
    if (more) issue(cn);

    for (uint32_t s = lane; s < g.u1; s += GG_WAVE) lcnt[s] = 0;
    wave_sync();
#pragma unroll
    for (uint32_t k = 0; k < kPerLane; ++k)
      if (k * GG_WAVE + lane < len) atomicAdd(&lcnt[key_l1set(key[k], smask)], 1u);
    wave_sync();
    // exclusive prefix of the per-set counts (lane-blocked + wave scan)
    {
      uint32_t lc[PER];
      uint32_t sum = 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) { const uint32_t s = lane * PER + k; lc[k] = (s < g.u1) ? lcnt[s] : 0; sum += lc[k]; }
      uint32_t incl = sum;
      for (int o = 1; o < GG_WAVE; o <<= 1) { const uint32_t v = __shfl_up(incl, o); if ((int)lane >= o) incl += v; }
      uint32_t run = incl - sum;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const uint32_t s = lane * PER + k;
        if (s < g.u1) { loff[s] = run; dbase[s] = ub[k] + cb[k] - run; lcnt[s] = 0; }
        run += lc[k];
      }
    }
    wave_sync();
#pragma unroll
    for (uint32_t k = 0; k < kPerLane; ++k) {
      const uint32_t j = k * GG_WAVE + lane;
      const bool valid = j < len;
      const uint32_t s = key_l1set(key[k], smask);
      uint64_t peers = __ballot(valid);
      for (uint32_t b = 0; b < g.log_u1; ++b) {
        const bool bit = (s >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        peers &= bit ? bb : ~bb;
      }
      const uint32_t rank = __popcll(peers & lt_mask);
      const uint32_t r0 = valid ? lcnt[s] : 0;
      wave_sync();
      if (valid && rank == 0) lcnt[s] = r0 + (uint32_t)__popcll(peers);
      wave_sync();
      if (valid) {
        const uint32_t q = loff[s] + r0 + rank;
        skey[q] = key[k];
        rec_slot[start + j] = (uint32_t)(dbase[s] + q);
      }
    }
    wave_sync();
    for (uint32_t q = lane; q < len; q += GG_WAVE) {
      const uint64_t k = skey[q];
      sh_key[dbase[key_l1set(k, smask)] + q] = k;
    }
    wave_sync();
    if (!more) break;
    i = inext;
    c = cn;
  }
}

size_t scatter_lds_bytes(const gg_geom& g) { return (size_t)kChunk * 8 + (size_t)g.u1 * (8 + 4 + 4); }

// Pass 5: program-order results.  result[i] = sh_res[rec_slot[i]]: each lane
// takes 4 consecutive records (dwordx4 slot load and result store) and issues
// its 4 gathers together; 4 such groups per lane are in flight per iteration.
// The gathers of one workgroup fall in the per-set runs of a few chunks.
constexpr uint32_t kUnshardPer = 16;                   // records per lane per iteration
__global__ __launch_bounds__(256) void k_unshard(const uint32_t* __restrict__ rec_slot,
    const uint32_t* __restrict__ sh_res, const uint64_t* __restrict__ sh_ev, uint32_t* __restrict__ result,
    uint64_t* __restrict__ evicted, uint64_t n)
{
  constexpr uint32_t G = kUnshardPer / 4;
  const uint64_t per_block = 256ull * kUnshardPer;
  const uint64_t nb = (n + per_block - 1) / per_block;
  const bool vec = (((uintptr_t)result | (uintptr_t)evicted) & 15) == 0;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint64_t base = b * per_block;
    if (vec && base + per_block <= n) {
      uint4 sl[G];
#pragma unroll
      for (uint32_t k = 0; k < G; ++k)
        sl[k] = *reinterpret_cast<const uint4*>(rec_slot + base + (k * 256 + threadIdx.x) * 4);
      if (result) {
        uint4 r[G];
#pragma unroll
        for (uint32_t k = 0; k < G; ++k)
          r[k] = make_uint4(sh_res[sl[k].x], sh_res[sl[k].y], sh_res[sl[k].z], sh_res[sl[k].w]);
#pragma unroll
        for (uint32_t k = 0; k < G; ++k)
          *reinterpret_cast<uint4*>(result + base + (k * 256 + threadIdx.x) * 4) = r[k];
      }
      if (evicted) {
#pragma unroll
        for (uint32_t k = 0; k < G; ++k) {
          const uint64_t i = base + (k * 256 + threadIdx.x) * 4;
          const uint64_t e0 = sh_ev[sl[k].x], e1 = sh_ev[sl[k].y], e2 = sh_ev[sl[k].z], e3 = sh_ev[sl[k].w];
          reinterpret_cast<uint4*>(evicted + i)[0] = make_uint4((uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)e1, (uint32_t)(e1 >> 32));
          reinterpret_cast<uint4*>(evicted + i)[1] = make_uint4((uint32_t)e2, (uint32_t)(e2 >> 32), (uint32_t)e3, (uint32_t)(e3 >> 32));
        }
      }
    } else {
      for (uint64_t i = base + threadIdx.x; i < min(n, base + per_block); i += 256) {
        const uint32_t sl = rec_slot[i];
        if (result) result[i] = sh_res[sl];
        if (evicted) evicted[i] = sh_ev[sl];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Replay kernel.  One lane per unit (tile, L1-D set), 64 units per wave.
//
// Every access runs the same straight-line, select-based sequence (no
// divergent control flow): L1-D lookup in VGPRs, one LDS read of the accessed
// L2 set (tags [s][lane][A2] via ds_read_b128, meta [s][lane] via
// ds_read_b64), the hit / L2-hit / directory paths of
// L1CacheCntlr::processMemOpFromCore folded into predicated updates, one LDS
// write-back.  Two facts of the private path keep it to ONE L2 set per access:
//   * PrL2CacheLineInfo::_cached_loc == L1-D  <=>  the L1-D holds the line
//     (it is set on every L1-D insert, l2_cache_cntlr.cc:98/160-163, and
//     cleared on every L1-D eviction, :145-164; the only other L1-D
//     invalidation, l1_cache_cntlr.cc:137, precedes an upgrade that
//     invalidates the L2 line too).  So the L1-D eviction's
//     getCacheLineInfo/setCacheLineInfo pair on the victim's L2 set changes
//     only counters, and invalidateCacheLineInL1 fires exactly when the L1-D
//     holds the L2 victim.  The kernel checks the invariant on entry and
//     writes the cached_loc bits back on exit, so the persisted state is the
//     reference's.
//   * every counter of Cache::outputSummary is a linear function of 11
//     per-access indicator sums (see kCounterMap below).
// ---------------------------------------------------------------------------
enum { I_WR = 0, I_NH1, I_NH1W, I_M2, I_M2W, I_W1V, I_L1EV, I_L2EV, I_DIRTY, I_INVL1, I_UPG, NI };

template <int A1>
__device__ __forceinline__ int match_u64(const uint64_t (&t)[A1], uint64_t x)
{
  int w1 = -1;
#pragma unroll
  for (int w = 0; w < A1; ++w) w1 = (t[w] == x) ? w : w1;
  return w1;
}

template <int A2>
__device__ __forceinline__ int match_u32(const uint32_t (&t)[A2], uint32_t x)
{
  int w2 = -1;
#pragma unroll
  for (int w = 0; w < A2; ++w) w2 = (t[w] == x) ? w : w2;
  return w2;
}

template <int A>
__device__ __forceinline__ uint32_t inv_mask_u64(const uint64_t (&t)[A])
{
  uint32_t m = 0;
#pragma unroll
  for (int w = 0; w < A; ++w) m |= (t[w] == GG_L1_INV_TAG ? 1u : 0u) << w;
  return m;
}

template <int A>
__device__ __forceinline__ uint32_t inv_mask_u32(const uint32_t (&t)[A])
{
  uint32_t m = 0;
#pragma unroll
  for (int w = 0; w < A; ++w) m |= (t[w] == GG_L2_INV_TAG ? 1u : 0u) << w;
  return m;
}

// LRU update of way `way` applied only when `cond`
template <int MW>
__device__ __forceinline__ void lru_update_if(uint64_t* mw, uint32_t way, bool cond)
{
  uint64_t nw[MW];
#pragma unroll
  for (int k = 0; k < MW; ++k) nw[k] = mw[k];
  lru_update<MW>(nw, way);
#pragma unroll
  for (int k = 0; k < MW; ++k) mw[k] = cond ? nw[k] : mw[k];
}

// Cache::outputSummary counters of one unit from its indicator sums, reduced
// over the wave and added to the tile's counters.
__device__ void replay_counters(const gg_cache_state& cs, const gg_geom& g, const uint32_t (&cnt)[NI],
                                uint32_t len, uint32_t tile, uint32_t lane, bool active)
{
  const uint32_t n = len;
  const uint32_t nwr = cnt[I_WR], nh1 = cnt[I_NH1], nh1w = cnt[I_NH1W], m2 = cnt[I_M2], m2w = cnt[I_M2W];
  const uint32_t w1v = cnt[I_W1V], l1ev = cnt[I_L1EV], l2ev = cnt[I_L2EV], drt = cnt[I_DIRTY];
  const uint32_t invl1 = cnt[I_INVL1], upg = cnt[I_UPG], h2 = nh1 - m2;
  uint32_t c[2 * NC];
  // L1-D
  c[ACC] = n; c[WACC] = nwr; c[RACC] = n - nwr; c[MISS] = nh1; c[WMISS] = nh1w; c[RMISS] = nh1 - nh1w;
  c[EV] = l1ev; c[DEV] = 0;
  c[TR] = n + 2 * nh1 + m2 + invl1;           // probe, invalidate probe + insert, retry probe, L2-evict probe
  c[TW] = w1v + nh1 + invl1;                  // invalidate, insert, L2-evict invalidation
  c[DR] = (n - nwr) + l1ev;                   // load access, eviction
  c[DW] = nwr + nh1;                          // store access, insert
  // L2
  c[NC + ACC] = nh1; c[NC + WACC] = nh1w; c[NC + RACC] = nh1 - nh1w;
  c[NC + MISS] = m2; c[NC + WMISS] = m2w; c[NC + RMISS] = m2 - m2w;
  c[NC + EV] = l2ev; c[NC + DEV] = drt;
  c[NC + TR] = nh1 + m2w + m2 + l1ev;         // probe, EX_REQ probe, insert, L1-D-eviction probe
  c[NC + TW] = upg + m2 + l1ev + h2;          // upgrade, insert, cached_loc clear, cached_loc set
  c[NC + DR] = h2 + l2ev;                     // readCacheLine, eviction
  c[NC + DW] = nwr + m2;                      // write-through, insert
  uint64_t* ctr = cs.counters + (uint64_t)tile * 2 * NC;
  if ((g.u1 & (GG_WAVE - 1)) == 0) {
#pragma unroll
    for (int k = 0; k < 2 * NC; ++k) {
      uint32_t a = active ? c[k] : 0u;
      for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
      if (lane == 0 && a) atomicAdd((unsigned long long*)&ctr[k], (unsigned long long)a);
    }
  } else if (active) {
#pragma unroll
    for (int k = 0; k < 2 * NC; ++k)
      if (c[k]) atomicAdd((unsigned long long*)&ctr[k], (unsigned long long)c[k]);
  }
}

template <int A1, int A2, bool LRU1, bool LRU2>
__global__ __launch_bounds__(64) void k_cache_replay(gg_cache_state cs, gg_geom g,
    const uint64_t* __restrict__ sh_key, const uint32_t* __restrict__ unit_len,
    const uint64_t* __restrict__ unit_base, uint32_t* __restrict__ sh_res,
    uint64_t* __restrict__ sh_ev, uint32_t* err)
{
  constexpr int MW = (A2 + 7) / 8;
  constexpr int TQ = (A2 + 3) / 4;                 // uint4 quads of tags per set
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x;
  const uint64_t u = (uint64_t)blockIdx.x * GG_WAVE + lane;
  const bool active = u < g.units;
  const uint64_t uu = active ? u : 0;
  const uint32_t S2 = g.s2;
  const uint32_t l1set = (uint32_t)(uu & (g.u1 - 1));
  uint32_t errv = 0;

  // LDS carve: tags [s][lane][TQ*4] u32 | meta [s][lane][MW] u64 | rr [s][lane] u8
  uint32_t* T = reinterpret_cast<uint32_t*>(smem);
  uint64_t* Mv = reinterpret_cast<uint64_t*>(smem + (size_t)S2 * GG_WAVE * TQ * 16);
  uint8_t* R = reinterpret_cast<uint8_t*>(smem + (size_t)S2 * GG_WAVE * TQ * 16 + (size_t)S2 * GG_WAVE * MW * 8);
  auto tq = [&](uint32_t s, int q) -> uint4* { return reinterpret_cast<uint4*>(T) + ((size_t)s * GG_WAVE + lane) * TQ + q; };
  auto mp = [&](uint32_t s, int k) -> uint64_t* { return Mv + ((size_t)s * GG_WAVE + lane) * MW + k; };

  // ---- load state (coalesced [field][unit] -> LDS / VGPRs) ----
  uint64_t t1[A1];
#pragma unroll
  for (int w = 0; w < A1; ++w) t1[w] = cs.l1_tag[(uint64_t)w * g.units + uu];
  uint64_t m1 = cs.l1_meta[uu];
  uint32_t rr1 = cs.l1_rr[uu];
  uint32_t nloc = 0, nl1 = 0;
  for (uint32_t s = 0; s < S2; ++s) {
    uint32_t tg[TQ * 4];
#pragma unroll
    for (int w = 0; w < TQ * 4; ++w)
      tg[w] = (w < A2) ? cs.l2_tag[(uint64_t)(s * A2 + w) * g.units + uu] : GG_L2_INV_TAG;
#pragma unroll
    for (int q = 0; q < TQ; ++q) *tq(s, q) = make_uint4(tg[4 * q], tg[4 * q + 1], tg[4 * q + 2], tg[4 * q + 3]);
    uint64_t mw[MW];
#pragma unroll
    for (int k = 0; k < MW; ++k) mw[k] = cs.l2_meta[(uint64_t)(s * MW + k) * g.units + uu];
    // cached_loc invariant check: loc bit <=> the L1-D holds the line
#pragma unroll
    for (int w = 0; w < A2; ++w) {
      const uint64_t ln = ((uint64_t)tg[w] << g.log_l2) | ((uint64_t)s << g.log_u1) | l1set;
      const bool held = tg[w] != GG_L2_INV_TAG && match_u64<A1>(t1, ln) >= 0;
      const bool loc = GG_M_LOC(meta_byte_t<MW>(mw, w)) != 0;
      nloc += loc ? 1u : 0u;
      errv |= (loc != held) ? GG_DERR_STATE : 0u;
      meta_set_byte_t<MW>(mw, w, meta_byte_t<MW>(mw, w) & ~4u);   // loc is implicit during the replay
    }
#pragma unroll
    for (int k = 0; k < MW; ++k) *mp(s, k) = mw[k];
    if (!LRU2) R[s * GG_WAVE + lane] = cs.l2_rr[(uint64_t)s * g.units + uu];
  }
#pragma unroll
  for (int w = 0; w < A1; ++w) nl1 += (t1[w] != GG_L1_INV_TAG) ? 1u : 0u;
  if (active && nl1 != nloc) errv |= GG_DERR_STATE;                 // an L1-D line missing from L2

  const uint32_t len = active ? unit_len[uu] : 0;
  const uint64_t base = active ? unit_base[uu] : 0;
  const uint32_t tile = (uint32_t)(uu >> g.log_u1);
  uint32_t maxlen = len;
  for (int o = 32; o > 0; o >>= 1) maxlen = max(maxlen, (uint32_t)__shfl_xor((int)maxlen, o));

  uint32_t cnt[NI];
#pragma unroll
  for (int k = 0; k < NI; ++k) cnt[k] = 0;

  // prefetch ring of the lane's record stream (distance 4)
  constexpr int PD = 4;
  uint64_t kr[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d) kr[d] = (d < (int)len) ? sh_key[base + d] : 0;
  const uint64_t lmask = (g.s2 - 1);

  for (uint32_t j = 0; j < maxlen; ++j) {
    const bool live = j < len;
    const uint64_t key = kr[0];
#pragma unroll
    for (int d = 0; d < PD - 1; ++d) kr[d] = kr[d + 1];
    const bool more = j + PD < len;
    kr[PD - 1] = more ? sh_key[base + j + PD] : 0;
    if (!live) continue;

    const bool wr = (key & 1u) != 0;
    const uint32_t s = ((uint32_t)key >> 1) & (uint32_t)lmask;
    const uint32_t tag2 = (uint32_t)(key >> 32);
    const uint64_t line = ((uint64_t)tag2 << g.log_l2) | ((uint64_t)s << g.log_u1) | l1set;

    // -- L2 set s (one LDS round trip) --
    uint32_t tg[TQ * 4];
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const uint4 v = *tq(s, q);
      tg[4 * q] = v.x; tg[4 * q + 1] = v.y; tg[4 * q + 2] = v.z; tg[4 * q + 3] = v.w;
    }
    uint64_t mw[MW];
#pragma unroll
    for (int k = 0; k < MW; ++k) mw[k] = *mp(s, k);
    uint32_t rr2 = LRU2 ? 0u : R[s * GG_WAVE + lane];

    // -- operationPermissibleinL1Cache (l1:207-243) --
    const int w1 = match_u64<A1>(t1, line);
    const uint32_t s1 = (w1 >= 0) ? GG_M_STATE(meta_byte(&m1, (uint32_t)w1)) : GG_MS_I;
    const bool hit1 = wr ? (s1 == GG_MS_M) : (s1 != GG_MS_I);

    // -- processShmemRequestFromL1Cache (l2:180-224) --
    uint32_t tga[A2];
#pragma unroll
    for (int w = 0; w < A2; ++w) tga[w] = tg[w];
    const int w2 = match_u32<A2>(tga, tag2);
    const uint32_t b2 = (w2 >= 0) ? meta_byte_t<MW>(mw, (uint32_t)w2) : 0u;
    const uint32_t s2 = GG_M_STATE(b2);
    const bool hit2 = !hit1 && (wr ? (s2 == GG_MS_M) : (s2 != GG_MS_I));
    const bool miss2 = !hit1 && !hit2;
    const bool upg = miss2 && wr && (s2 == GG_MS_S);                 // processExReqFromL1Cache (l2:260-282)
    const bool w1v = !hit1 && (w1 >= 0);
    errv |= (hit1 && wr && w2 < 0) ? GG_DERR_STATE : 0u;             // write-through needs the L2 copy

    // L1CacheCntlr::invalidateCacheLine of the missing line (l1:135-137)
#pragma unroll
    for (int w = 0; w < A1; ++w) t1[w] = (w1v && w == w1) ? GG_L1_INV_TAG : t1[w];
    if (w1v) m1 &= ~(7ull << (8 * w1));
    // upgrade: PrL2CacheLineInfo::invalidate + setCacheLineInfo (tag, state, loc; age kept)
#pragma unroll
    for (int w = 0; w < A2; ++w) tga[w] = (upg && w == w2) ? GG_L2_INV_TAG : tga[w];
    if (upg) meta_set_byte_t<MW>(mw, (uint32_t)w2, b2 & ~7u);

    // -- L2CacheCntlr::insertCacheLine (l2:74-116): victim, eviction, install --
    int v2;
    if (LRU2) v2 = lru_victim<A2, MW>(inv_mask_u32<A2>(tga), mw);
    else v2 = (int)rr2;
    errv |= (miss2 && v2 < 0) ? GG_DERR_STATE : 0u;
    v2 = v2 < 0 ? 0 : v2;
    uint32_t vt = GG_L2_INV_TAG;
#pragma unroll
    for (int w = 0; w < A2; ++w) vt = (w == v2) ? tga[w] : vt;
    const uint32_t vb = meta_byte_t<MW>(mw, (uint32_t)v2);
    const bool l2ev = miss2 && vt != GG_L2_INV_TAG;
    const bool dirty = l2ev && GG_M_STATE(vb) == GG_MS_M;            // FLUSH_REP (else INV_REP)
    errv |= (l2ev && GG_M_STATE(vb) == GG_MS_I) ? GG_DERR_STATE : 0u;
    const uint64_t e2 = ((uint64_t)vt << g.log_l2) | ((uint64_t)s << g.log_u1) | l1set;
    // invalidateCacheLineInL1: fires iff the L1-D holds the victim (cached_loc invariant)
    const int we = match_u64<A1>(t1, e2);
    const bool invl1 = l2ev && we >= 0;
#pragma unroll
    for (int w = 0; w < A1; ++w) t1[w] = (invl1 && w == we) ? GG_L1_INV_TAG : t1[w];
    if (invl1) m1 &= ~(7ull << (8 * we));
    const uint32_t ns = wr ? GG_MS_M : GG_MS_S;                      // EX_REP / SH_REP
#pragma unroll
    for (int w = 0; w < A2; ++w) tga[w] = (miss2 && w == v2) ? tag2 : tga[w];
    if (miss2) meta_set_byte_t<MW>(mw, (uint32_t)v2, (vb & ~7u) | ns);
    if (!LRU2 && miss2) rr2 = (rr2 == 0) ? (A2 - 1) : (rr2 - 1);
    // L2 replacement update: readCacheLine (hit2), install (miss2), write-through (hit1 && wr)
    if (LRU2) lru_update_if<MW>(mw, (uint32_t)(miss2 ? v2 : (w2 < 0 ? 0 : w2)), (!hit1 || wr) && (miss2 || w2 >= 0));

    // -- insertCacheLineInL1 (l2:133-165): victim after both invalidations --
    int v1;
    if (LRU1) v1 = lru_victim<A1, 1>(inv_mask_u64<A1>(t1), &m1);
    else v1 = (int)rr1;
    errv |= (!hit1 && v1 < 0) ? GG_DERR_STATE : 0u;
    v1 = v1 < 0 ? 0 : v1;
    uint64_t et = GG_L1_INV_TAG;
#pragma unroll
    for (int w = 0; w < A1; ++w) et = (w == v1) ? t1[w] : et;
    const bool l1ev = !hit1 && et != GG_L1_INV_TAG;
    const uint32_t ins = hit2 ? s2 : ns;
#pragma unroll
    for (int w = 0; w < A1; ++w) t1[w] = (!hit1 && w == v1) ? line : t1[w];
    if (!hit1) meta_set_byte(&m1, (uint32_t)v1, (meta_byte(&m1, (uint32_t)v1) & ~7u) | ins);
    if (!LRU1 && !hit1) rr1 = (rr1 == 0) ? (A1 - 1) : (rr1 - 1);
    // L1-D replacement update: accessCache on the hit way or the inserted way
    if (LRU1) lru_update<1>(&m1, (uint32_t)(hit1 ? w1 : v1));

    // -- write the L2 set back --
#pragma unroll
    for (int w = A2; w < TQ * 4; ++w) tg[w] = GG_L2_INV_TAG;
#pragma unroll
    for (int w = 0; w < A2; ++w) tg[w] = tga[w];
#pragma unroll
    for (int q = 0; q < TQ; ++q) *tq(s, q) = make_uint4(tg[4 * q], tg[4 * q + 1], tg[4 * q + 2], tg[4 * q + 3]);
#pragma unroll
    for (int k = 0; k < MW; ++k) *mp(s, k) = mw[k];
    if (!LRU2 && miss2) R[s * GG_WAVE + lane] = (uint8_t)rr2;

    // -- indicator sums and outputs --
    cnt[I_WR] += wr; cnt[I_NH1] += !hit1; cnt[I_NH1W] += (!hit1 && wr); cnt[I_M2] += miss2;
    cnt[I_M2W] += (miss2 && wr); cnt[I_W1V] += w1v; cnt[I_L1EV] += l1ev; cnt[I_L2EV] += l2ev;
    cnt[I_DIRTY] += dirty; cnt[I_INVL1] += invl1; cnt[I_UPG] += upg;
    const uint32_t res = (hit1 ? 0u : GG_RES_L1_MISS) | (miss2 ? GG_RES_L2_MISS : 0u) | (w1v ? GG_RES_L1_INVAL : 0u) |
                         (upg ? GG_RES_UPGRADE : 0u) | (l1ev ? GG_RES_L1_EVICT : 0u) |
                         (l2ev ? GG_RES_L2_EVICT : 0u) | (dirty ? GG_RES_L2_EVICT_DIRTY : 0u) |
                         (invl1 ? GG_RES_L2_EVICT_INV_L1 : 0u);
    if (sh_res) sh_res[base + j] = res;
    if (sh_ev) sh_ev[base + j] = l2ev ? (e2 << g.log_line) : ~0ull;
  }

  // ---- store state back, with cached_loc materialised from the L1-D ----
  if (active) {
#pragma unroll
    for (int w = 0; w < A1; ++w) cs.l1_tag[(uint64_t)w * g.units + u] = t1[w];
    cs.l1_meta[u] = m1;
    cs.l1_rr[u] = (uint8_t)rr1;
    for (uint32_t s = 0; s < S2; ++s) {
      uint32_t tg[TQ * 4];
#pragma unroll
      for (int q = 0; q < TQ; ++q) {
        const uint4 v = *tq(s, q);
        tg[4 * q] = v.x; tg[4 * q + 1] = v.y; tg[4 * q + 2] = v.z; tg[4 * q + 3] = v.w;
      }
      uint64_t mw[MW];
#pragma unroll
      for (int k = 0; k < MW; ++k) mw[k] = *mp(s, k);
#pragma unroll
      for (int w = 0; w < A2; ++w) {
        const uint64_t ln = ((uint64_t)tg[w] << g.log_l2) | ((uint64_t)s << g.log_u1) | l1set;
        const bool held = tg[w] != GG_L2_INV_TAG && match_u64<A1>(t1, ln) >= 0;
        meta_set_byte_t<MW>(mw, w, (meta_byte_t<MW>(mw, w) & ~4u) | (held ? 4u : 0u));
        cs.l2_tag[(uint64_t)(s * A2 + w) * g.units + u] = tg[w];
      }
#pragma unroll
      for (int k = 0; k < MW; ++k) cs.l2_meta[(uint64_t)(s * MW + k) * g.units + u] = mw[k];
      if (!LRU2) cs.l2_rr[(uint64_t)s * g.units + u] = R[s * GG_WAVE + lane];
    }
  }
  if (!active) errv = 0;
  if (errv) atomicOr(err, errv);

  replay_counters(cs, g, cnt, len, tile, lane, active);
}

// ---------------------------------------------------------------------------
// Lean replay for the reference geometries (L1-D assoc <= 4, L2 assoc <= 8).
// Same semantics as k_cache_replay; per-unit state re-packed for fewer
// instructions per access:
//   L1-D: no tags.  The private L1-D is inclusive in the L2 (every L1-D line
//         has its L2 copy, cached_loc invariant above), so an L1-D way is
//         named by the L2 slot of its line: pos1 = per-way byte s * A2 + way
//         (0xFF = invalid way).  "Does the L1-D hold the line" and "does the
//         L1-D hold the L2 victim" are one SWAR byte match each; tags are
//         rebuilt from the L2 at exit.  st1 = 2-bit states, a1 = 4-bit ages.
//   L2:   tags [s][lane][4*TQ] u32 in LDS (canonical: ~0 = invalid, updated by
//         predicated ds_write_b32), meta [s][lane] = {ages u32, states u16 | rr}.
//   Counters: the result word has one flag per 4-bit field, so the 8 result
//         words of a block are summed field-wise (3 add3) and folded into
//         byte-wide accumulators (flushed every 31 blocks) instead of 11
//         per-access counter increments.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t zero_nibbles(uint32_t x)
{
  return ~(((x & 0x77777777u) + 0x77777777u) | x | 0x77777777u) & 0x88888888u;
}
__device__ __forceinline__ uint32_t zero_bytes32(uint32_t x)
{
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu) & 0x80808080u;
}
// LRUReplacementPolicy::update on nibble-packed ages (ages < 8; unused = 0xF)
__device__ __forceinline__ uint32_t lru_nib(uint32_t ages, uint32_t way)
{
  const uint32_t sh = 4 * way;
  const uint32_t acc = (ages >> sh) & 0xFu;
  // acc in every nibble (v_perm byte broadcast instead of a 32-bit multiply)
  const uint32_t x = (ages | 0x88888888u) - __builtin_amdgcn_perm(0u, acc | (acc << 4), 0u);  // bit 3: age >= acc
  const uint32_t lt = ~x & 0x88888888u;
  return (ages + (lt >> 3)) & ~(0xFu << sh);
}
// getReplacementWay: first invalid way (2-bit state == 0) else the last way with age A-1
template <int A>
__device__ __forceinline__ int victim_nib(uint32_t states, uint32_t ages)
{
  constexpr uint32_t PAIRS = (A >= 16) ? 0x55555555u : ((1u << (2 * A)) - 1) & 0x55555555u;
  const uint32_t ip = ~(states | (states >> 1)) & PAIRS;
  const int fi = (int)(__builtin_ctz(ip | 0x80000000u) >> 1);
  const uint32_t zn = zero_nibbles(ages ^ ((uint32_t)(A - 1) * 0x11111111u));
  const int lw = zn ? (int)((31 - __builtin_clz(zn)) >> 2) : -1;
  return ip ? fi : lw;
}

// 16 nibble ages (16-way L2, ages 0..15 leave no spare bit per nibble): the
// same update with the even and the odd nibbles compared as bytes
__device__ __forceinline__ uint64_t lru_nib64(uint64_t ages, uint32_t way)
{
  constexpr uint64_t L = 0x0F0F0F0F0F0F0F0Full, G = 0x8080808080808080ull;
  const uint32_t sh = 4 * way;
  const uint64_t accb = ((ages >> sh) & 0xFull) * 0x0101010101010101ull;
  uint64_t e = ages & L, o = (ages >> 4) & L;
  e += (~((e | G) - accb) & G) >> 7;                 // +1 where age < the accessed way's age
  o += (~((o | G) - accb) & G) >> 7;
  return (e | (o << 4)) & ~(0xFull << sh);
}
__device__ __forceinline__ int victim_nib64(uint32_t states, uint64_t ages)
{
  const uint32_t ip = ~(states | (states >> 1)) & 0x55555555u;
  const int fi = (int)(__builtin_ctz(ip | 0x80000000u) >> 1);
  const uint64_t zn = (uint64_t)zero_nibbles(~(uint32_t)ages) | ((uint64_t)zero_nibbles(~(uint32_t)(ages >> 32)) << 32);
  const int lw = zn ? (int)((63 - __builtin_clzll(zn)) >> 2) : -1;
  return ip ? fi : lw;
}

template <int A1, int A2, bool LRU1, bool LRU2>
__global__ __launch_bounds__(64) void k_cache_replay_lean(gg_cache_state cs, gg_geom g,
    const uint64_t* __restrict__ sh_key, const uint32_t* __restrict__ unit_len,
    const uint64_t* __restrict__ unit_base, uint32_t* __restrict__ sh_res,
    uint64_t* __restrict__ sh_ev, uint32_t* err)
{
  static_assert(A1 <= 4 && A2 <= 8, "lean replay covers L1-D assoc <= 4, L2 assoc <= 8");
  constexpr int TQ = (A2 + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x;
  const uint64_t u = (uint64_t)blockIdx.x * GG_WAVE + lane;
  const bool active = u < g.units;
  const uint64_t uu = active ? u : 0;
  const uint32_t S2 = g.s2;
  const uint32_t l1set = (uint32_t)(uu & (g.u1 - 1));
  uint32_t errv = 0;

  uint32_t* T = reinterpret_cast<uint32_t*>(smem);                                   // [s][lane][4*TQ]
  uint2* Mt = reinterpret_cast<uint2*>(smem + (size_t)S2 * GG_WAVE * TQ * 16);        // [s][lane]
  auto tptr = [&](uint32_t s) -> uint32_t* { return T + ((size_t)s * GG_WAVE + lane) * (4 * TQ); };

  // ---- load + re-pack state ----
  uint32_t st1 = 0, a1 = 0xFFFFFFFFu, pos1 = 0xFFFFFFFFu;
  uint64_t t1[A1];
  {
    const uint64_t m1 = cs.l1_meta[uu];
#pragma unroll
    for (int w = 0; w < A1; ++w) {
      t1[w] = cs.l1_tag[(uint64_t)w * g.units + uu];
      const uint32_t b = (uint32_t)(m1 >> (8 * w)) & 0xFFu;
      const uint32_t st = (t1[w] == GG_L1_INV_TAG) ? 0u : GG_M_STATE(b);
      errv |= (t1[w] != GG_L1_INV_TAG && st == GG_MS_I) ? GG_DERR_STATE : 0u;   // valid tag, INVALID state
      st1 |= st << (2 * w);
      a1 = (a1 & ~(0xFu << (4 * w))) | ((GG_M_AGE(b) & 0xFu) << (4 * w));
    }
  }
  uint32_t rr1 = cs.l1_rr[uu];
  uint32_t nheld = 0;
  for (uint32_t s = 0; s < S2; ++s) {
    uint32_t tg[4 * TQ];
#pragma unroll
    for (int w = 0; w < 4 * TQ; ++w)
      tg[w] = (w < A2) ? cs.l2_tag[(uint64_t)(s * A2 + w) * g.units + uu] : GG_L2_INV_TAG;
    const uint64_t mw = cs.l2_meta[(uint64_t)s * g.units + uu];
    uint32_t ages = 0xFFFFFFFFu, st = 0;
#pragma unroll
    for (int w = 0; w < A2; ++w) {
      const uint32_t b = (uint32_t)(mw >> (8 * w)) & 0xFFu;
      const bool valid = tg[w] != GG_L2_INV_TAG;
      errv |= (valid != (GG_M_STATE(b) != GG_MS_I)) ? GG_DERR_STATE : 0u;
      st |= (valid ? GG_M_STATE(b) : 0u) << (2 * w);
      ages = (ages & ~(0xFu << (4 * w))) | ((GG_M_AGE(b) & 0xFu) << (4 * w));
      // cached_loc invariant + the L1-D way holding this line
      const uint64_t ln = ((uint64_t)tg[w] << g.log_l2) | ((uint64_t)s << g.log_u1) | l1set;
      int hw = -1;
#pragma unroll
      for (int k = 0; k < A1; ++k) hw = (valid && ((st1 >> (2 * k)) & 3u) && t1[k] == ln) ? k : hw;
      const bool loc = GG_M_LOC(b) != 0;
      nheld += (hw >= 0) ? 1u : 0u;
      errv |= (loc != (hw >= 0)) ? GG_DERR_STATE : 0u;
      if (hw >= 0) pos1 = (pos1 & ~(0xFFu << (8 * hw))) | ((s * A2 + w) << (8 * hw));
    }
    uint32_t* tp = tptr(s);
#pragma unroll
    for (int q = 0; q < TQ; ++q)
      *reinterpret_cast<uint4*>(tp + 4 * q) = make_uint4(tg[4 * q], tg[4 * q + 1], tg[4 * q + 2], tg[4 * q + 3]);
    const uint32_t rr = LRU2 ? 0u : cs.l2_rr[(uint64_t)s * g.units + uu];
    Mt[s * GG_WAVE + lane] = make_uint2(ages, st | (rr << 16));
  }
  {
    uint32_t nvalid = 0;
#pragma unroll
    for (int k = 0; k < A1; ++k) nvalid += ((st1 >> (2 * k)) & 3u) ? 1u : 0u;
    if (active && nvalid != nheld) errv |= GG_DERR_STATE;          // an L1-D line without its L2 copy
  }

  const uint32_t len = active ? unit_len[uu] : 0;
  const uint64_t base = active ? unit_base[uu] : 0;
  const uint32_t tile = (uint32_t)(uu >> g.log_u1);
  uint32_t maxlen = len;
  for (int o = 32; o > 0; o >>= 1) maxlen = max(maxlen, (uint32_t)__shfl_xor((int)maxlen, o));

  const uint32_t log_s2 = (uint32_t)__builtin_ctz(S2);
  const uint32_t log_line = g.log_line, log_u1 = g.log_u1, log_l2 = g.log_l2;

  // One access of this lane's unit (the body of processMemOpFromCore); returns
  // the result word, and the evicted L2 line address through *ev.
  auto step = [&](const uint32_t klo, const uint32_t tag2, uint64_t* ev) -> uint32_t {
    const uint32_t wr = klo & 1u;
    const uint32_t s = __builtin_amdgcn_ubfe(klo, 1, log_s2);
    uint32_t* tp = tptr(s);
    uint32_t tg[4 * TQ];
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const uint4 v = *reinterpret_cast<const uint4*>(tp + 4 * q);
      tg[4 * q] = v.x; tg[4 * q + 1] = v.y; tg[4 * q + 2] = v.z; tg[4 * q + 3] = v.w;
    }
    const uint2 mt = Mt[s * GG_WAVE + lane];
    uint32_t ages2 = mt.x, st2 = mt.y & 0xFFFFu, rr2 = (mt.y >> 16) & 0xFFu;

    // L2 lookup (processShmemRequestFromL1Cache): valid tags are unique in a
    // set and the invalid tag never matches, so at most one way hits
    uint32_t mm2 = 0;
#pragma unroll
    for (int w = 0; w < A2; ++w) mm2 |= (tg[w] == tag2) ? (1u << w) : 0u;
    const uint32_t w2 = (uint32_t)__builtin_ctz(mm2 | (1u << A2));     // A2 when absent
    const uint32_t s2 = (st2 >> (2 * w2)) & 3u;                        // 0 when absent
    // L1-D lookup (operationPermissibleinL1Cache): the L1-D holds the line
    // iff one of its ways names the line's L2 slot
    const uint32_t zb1 = mm2 ? zero_bytes32(pos1 ^ ((s * A2 + w2) * 0x01010101u)) : 0u;
    const uint32_t w1 = (uint32_t)__builtin_ctz(zb1 | 0x80000000u) >> 3;
    const uint32_t s1 = zb1 ? (st1 >> (2 * w1)) & 3u : 0u;
    const bool hit1 = s1 > wr;                                         // READ: readable, WRITE: writable
    const bool hit2n = s2 > wr;
    const bool hit2 = !hit1 && hit2n;
    const bool miss2 = !hit1 && !hit2n;
    const bool upg = miss2 && wr && s2 == GG_MS_S;
    const bool w1v = !hit1 && zb1 != 0;

    // invalidate the L1-D copy before going to L2 (l1:135-137)
    st1 = w1v ? (st1 & ~(3u << (2 * w1))) : st1;
    pos1 = w1v ? (pos1 | (0xFFu << (8 * w1))) : pos1;
    // upgrade: invalidate the SHARED L2 line (l2:260-282)
    if (upg) tp[w2] = GG_L2_INV_TAG;
    st2 = upg ? (st2 & ~(3u << (2 * w2))) : st2;
    // L2 victim / eviction (l2:74-116)
    int v2 = LRU2 ? victim_nib<A2>(st2, ages2) : (int)rr2;
    errv |= (miss2 && v2 < 0) ? GG_DERR_STATE : 0u;
    v2 &= 7;
    const uint32_t sv = (st2 >> (2 * v2)) & 3u;
    const bool l2ev = miss2 && sv != 0;
    const bool dirty = l2ev && sv == GG_MS_M;
    uint32_t vt = 0;
    if (sh_ev) {
#pragma unroll
      for (int w = 0; w < A2; ++w) vt = (w == v2) ? tg[w] : vt;
    }
    // invalidateCacheLineInL1: does the L1-D hold L2 slot (s, v2)?
    const uint32_t zb = zero_bytes32(pos1 ^ ((s * A2 + v2) * 0x01010101u));
    const bool invl1 = l2ev && zb != 0;
    const uint32_t we = (uint32_t)__builtin_ctz(zb | 0x80000000u) >> 3;
    st1 = invl1 ? (st1 & ~(3u << (2 * we))) : st1;
    pos1 = invl1 ? (pos1 | (0xFFu << (8 * we))) : pos1;
    // install (EX_REP -> MODIFIED, SH_REP -> SHARED)
    const uint32_t ns = 1u + wr;
    if (miss2) tp[v2] = tag2;
    st2 = miss2 ? ((st2 & ~(3u << (2 * v2))) | (ns << (2 * v2))) : st2;
    if (!LRU2 && miss2) rr2 = rr2 ? rr2 - 1 : (A2 - 1);
    // L2 LRU: readCacheLine (hit2) / insert (miss2) / write-through (hit1 && wr)
    if (LRU2) {
      const uint32_t x2 = miss2 ? (uint32_t)v2 : (w2 & 7u);
      const uint32_t nb = lru_nib(ages2, x2);
      ages2 = (!hit1 || wr) ? nb : ages2;
    }
    // L1-D insert (insertCacheLineInL1) after both invalidations
    int v1 = LRU1 ? victim_nib<A1>(st1, a1) : (int)rr1;
    errv |= (!hit1 && v1 < 0) ? GG_DERR_STATE : 0u;
    v1 &= 3;
    const bool l1ev = !hit1 && ((st1 >> (2 * v1)) & 3u) != 0;
    const uint32_t ins = hit2 ? s2 : ns;
    const uint32_t slot = s * A2 + (hit2 ? w2 : (uint32_t)v2);
    st1 = !hit1 ? ((st1 & ~(3u << (2 * v1))) | (ins << (2 * v1))) : st1;
    pos1 = !hit1 ? ((pos1 & ~(0xFFu << (8 * v1))) | (slot << (8 * v1))) : pos1;
    if (!LRU1 && !hit1) rr1 = rr1 ? rr1 - 1 : (A1 - 1);
    // L1-D LRU: accessCache on the hit way or the inserted way
    if (LRU1) a1 = lru_nib(a1, hit1 ? (w1 & 3u) : (uint32_t)v1);

    Mt[s * GG_WAVE + lane] = make_uint2(ages2, st2 | (rr2 << 16));
    if (sh_ev) {
      const uint64_t e2 = ((uint64_t)vt << log_l2) | ((uint64_t)s << log_u1) | l1set;
      *ev = l2ev ? (e2 << log_line) : ~0ull;
    }
    return (hit1 ? 0u : GG_RES_L1_MISS) | (miss2 ? GG_RES_L2_MISS : 0u) | (w1v ? GG_RES_L1_INVAL : 0u) |
           (l1ev ? GG_RES_L1_EVICT : 0u) | (l2ev ? GG_RES_L2_EVICT : 0u) | (dirty ? GG_RES_L2_EVICT_DIRTY : 0u) |
           (invl1 ? GG_RES_L2_EVICT_INV_L1 : 0u) | (upg ? GG_RES_UPGRADE : 0u);
  };

  // Counter fields, in result-word nibble order: 0 L1 miss, 1 L2 miss,
  // 2 L1 inval, 3 L1 evict, 4 L2 evict, 5 dirty, 6 inv-L1, 7 upgrade.
  uint32_t f8[8], fw[2], nwr = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) f8[k] = 0;
  fw[0] = fw[1] = 0;
  uint32_t acc_lo = 0, acc_hi = 0, acc_w = 0, nblk = 0;
  auto flush = [&]() {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f8[2 * k] += (acc_lo >> (8 * k)) & 0xFFu;
      f8[2 * k + 1] += (acc_hi >> (8 * k)) & 0xFFu;
    }
    fw[0] += acc_w & 0xFFFFu;
    fw[1] += acc_w >> 16;
    acc_lo = acc_hi = acc_w = 0;
    nblk = 0;
  };

  // The unit's records are contiguous from `base` (8-record aligned): stream
  // them in 8-record blocks (4 dwordx4 loads), next block in flight while the
  // current one is replayed from registers; the block's 8 results go out as
  // 2 dwordx4 stores to the same slots of sh_res (padding slots included).
  constexpr int KB = 8;
  const uint4* kp = reinterpret_cast<const uint4*>(sh_key + base);
  uint4* rp = reinterpret_cast<uint4*>(sh_res + base);
  uint4* ep = reinterpret_cast<uint4*>(sh_ev + base);
  uint4 kb[KB / 2];
  if (len > 0) {
#pragma unroll
    for (int q = 0; q < KB / 2; ++q) kb[q] = kp[q];
  }
  for (uint32_t j0 = 0; j0 < maxlen; j0 += KB) {
    uint4 nkb[KB / 2];
    const bool more = j0 + KB < len;
    if (more) {
#pragma unroll
      for (int q = 0; q < KB / 2; ++q) nkb[q] = kp[(j0 + KB) / 2 + q];
    }
    uint32_t rv[KB], wm[KB];
    uint64_t ev[KB];
#pragma unroll
    for (int d = 0; d < KB; ++d) {
      rv[d] = 0; wm[d] = 0; ev[d] = ~0ull;
      if (j0 + d < len) {
        const uint4 kv = kb[d / 2];
        const uint32_t klo = (d & 1) ? kv.z : kv.x, tag2 = (d & 1) ? kv.w : kv.y;
        rv[d] = step(klo, tag2, &ev[d]);
        wm[d] = klo & 1u;
      }
    }
    if (j0 < len) {
      if (sh_res) {
        rp[j0 / 4] = make_uint4(rv[0], rv[1], rv[2], rv[3]);
        rp[j0 / 4 + 1] = make_uint4(rv[4], rv[5], rv[6], rv[7]);
      }
      if (sh_ev) {
#pragma unroll
        for (int q = 0; q < KB / 2; ++q)
          ep[j0 / 2 + q] = make_uint4((uint32_t)ev[2 * q], (uint32_t)(ev[2 * q] >> 32),
                                      (uint32_t)ev[2 * q + 1], (uint32_t)(ev[2 * q + 1] >> 32));
      }
    }
    // field-wise sums of the block's result words (each field <= 8)
    const uint32_t sum = rv[0] + rv[1] + rv[2] + rv[3] + rv[4] + rv[5] + rv[6] + rv[7];
    uint32_t sw = 0, nw = 0;
#pragma unroll
    for (int d = 0; d < KB; ++d) { sw += rv[d] & (wm[d] * 0x11u); nw += wm[d]; }
    acc_lo += sum & 0x0F0F0F0Fu;
    acc_hi += (sum >> 4) & 0x0F0F0F0Fu;
    acc_w += (sw & 0xFu) | ((sw & 0xF0u) << 12);
    nwr += nw;
    if (++nblk == 31) flush();
    if (more) {
#pragma unroll
      for (int q = 0; q < KB / 2; ++q) kb[q] = nkb[q];
    }
  }
  flush();

  // ---- store state back in the HBM format (canonical tags, byte meta, cached_loc) ----
  if (active) {
    uint64_t m1 = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      if (w < A1) {
        const uint32_t st = (st1 >> (2 * w)) & 3u;
        uint64_t tag1 = GG_L1_INV_TAG;
        if (st) {                                     // rebuild the line from its L2 slot
          const uint32_t slot = (pos1 >> (8 * w)) & 0xFFu;
          const uint32_t ss = slot / A2, ww = slot % A2;
          tag1 = ((uint64_t)tptr(ss)[ww] << g.log_l2) | ((uint64_t)ss << g.log_u1) | l1set;
        }
        cs.l1_tag[(uint64_t)w * g.units + u] = tag1;
        m1 |= (uint64_t)GG_M_MAKE(st, 0, (a1 >> (4 * w)) & 0xFu) << (8 * w);
      } else {
        m1 |= 0xF8ull << (8 * w);
      }
    }
    cs.l1_meta[u] = m1;
    cs.l1_rr[u] = (uint8_t)rr1;
    for (uint32_t s = 0; s < S2; ++s) {
      const uint32_t* tp = tptr(s);
      const uint2 mt = Mt[s * GG_WAVE + lane];
      uint64_t mw = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        if (w < A2) {
          const uint32_t st = (mt.y >> (2 * w)) & 3u;
          // cached_loc: does an L1-D way name this slot?
          const uint32_t zb = zero_bytes32(pos1 ^ ((s * A2 + w) * 0x01010101u));
          mw |= (uint64_t)GG_M_MAKE(st, (zb != 0) ? 1u : 0u, (mt.x >> (4 * w)) & 0xFu) << (8 * w);
          cs.l2_tag[(uint64_t)(s * A2 + w) * g.units + u] = tp[w];
        } else {
          mw |= 0xF8ull << (8 * w);
        }
      }
      cs.l2_meta[(uint64_t)s * g.units + u] = mw;
      if (!LRU2) cs.l2_rr[(uint64_t)s * g.units + u] = (uint8_t)((mt.y >> 16) & 0xFFu);
    }
  }
  if (!active) errv = 0;
  if (errv) atomicOr(err, errv);
  uint32_t cnt[NI];
  cnt[I_WR] = nwr; cnt[I_NH1] = f8[0]; cnt[I_NH1W] = fw[0]; cnt[I_M2] = f8[1]; cnt[I_M2W] = fw[1];
  cnt[I_W1V] = f8[2]; cnt[I_L1EV] = f8[3]; cnt[I_L2EV] = f8[4]; cnt[I_DIRTY] = f8[5]; cnt[I_INVL1] = f8[6];
  cnt[I_UPG] = f8[7];
  replay_counters(cs, g, cnt, len, tile, lane, active);
}

// ---------------------------------------------------------------------------
// Streaming replay (the default batch path): ONE kernel, one workgroup per
// tile, reading the caller's program-order trace once and writing each
// result once (16 B of HBM per access: 8 addr + 4 meta in, 4 result out).
//
//   * NCW consumer waves = the tile's u1 units (lane = L1-D set), each
//     running the access step of k_cache_replay_lean on its unit.  The tile's
//     L2 sets stay in LDS for the whole batch ([s][q][u] uint4, 16-B lane
//     stride: conflict-free ds_read_b128), the L1-D set in VGPRs.
//   * one producer wave streams the tile's records (4 rounds of 64 coalesced
//     8-B + 4-B loads in flight while the previous 4 are distributed) and
//     appends each to its unit's LDS ring (kRing records per unit).  Records
//     of one round that name the same unit are ranked by lane (log2 u1
//     ballots), so every unit receives its records in program order — the
//     only order the reference's per-set state depends on.
//   * hand-off: the producer writes ring slots, waits for them
//     (lgkmcnt), then publishes the unit's tail; a consumer reads the tail
//     before the slot (volatile, so in issue order; one CU's LDS serves a
//     wave's instructions in order).  A consumer publishes its head after
//     each access; the producer waits for ring space on it.  Both waits are
//     bounded: consumers always drain a published record, and the producer
//     publishes at most kRing records of a unit per sub-round.
//   * ring entry: high word = the 32-bit L2 tag; low word = WRITE (bit 0),
//     L2 set within the unit (bits 1..log2 S2), the record's index within the
//     tile above that; the consumer stores its result word straight to
//     result[tile base + index] (scattered dword stores that fill whole lines
//     in L2 while the tile's window is in flight).
// ---------------------------------------------------------------------------
#ifndef GG_RING
#define GG_RING 32
#endif
#ifndef GG_PK
#define GG_PK 4
#endif
constexpr uint32_t kRing = GG_RING;
constexpr uint32_t kSpinLimit = 1u << 22;   // s_sleep(1) polls (~64 cycles each) before giving up
constexpr uint16_t kLgkm0 = 0xC07F;         // s_waitcnt lgkmcnt(0) (vmcnt/expcnt fields at their maxima)

size_t stream_lds_bytes(uint32_t u1, uint32_t s2, uint32_t a2)
{
  const size_t tq = (a2 + 3) / 4;
  return (size_t)s2 * u1 * (tq * 16 + (a2 > 8 ? 16 : 8)) + (size_t)kRing * u1 * 8 + (size_t)u1 * 12 + 16 + (size_t)u1 * 8 + (size_t)u1 * 4;
}

template <int A1, int A2, bool LRU1, bool LRU2, int NCW, bool EV>
__global__ __launch_bounds__((NCW + 1) * GG_WAVE) void k_cache_stream(gg_cache_state cs, gg_geom g,
    const uint64_t* __restrict__ addr, const uint32_t* __restrict__ meta, const uint64_t* __restrict__ tile_off,
    uint32_t* __restrict__ result, uint64_t* __restrict__ evicted, uint32_t* err, unsigned long long* dbg)
{
  static_assert(A1 <= 4 && (A2 <= 8 || A2 == 16), "streaming replay covers L1-D assoc <= 4, L2 assoc <= 8 or 16");
  constexpr uint32_t U1 = NCW * GG_WAVE;   // == g.u1 (host-checked)
  constexpr int TQ = (A2 + 3) / 4;
  constexpr int MW = (A2 + 7) / 8;         // HBM meta words per L2 set
  // per (L2 set, unit): LRU ages (nibble per way), 2-bit states, round-robin
  // way; 16 ways take 64-bit ages in a 16-B record
  constexpr bool W16 = A2 > 8;
  using AgT = typename std::conditional<W16, uint64_t, uint32_t>::type;
  using MtT = typename std::conditional<W16, uint4, uint2>::type;
  auto mt_pack = [](AgT ages, uint32_t st, uint32_t rr) -> MtT {
    if constexpr (W16) return make_uint4((uint32_t)ages, (uint32_t)((uint64_t)ages >> 32), st, rr);
    else return make_uint2((uint32_t)ages, st | (rr << 16));
  };
  auto mt_ages = [](const MtT& m) -> AgT {
    if constexpr (W16) return ((uint64_t)m.y << 32) | m.x; else return m.x;
  };
  auto mt_st = [](const MtT& m) -> uint32_t { if constexpr (W16) return m.z; else return m.y & 0xFFFFu; };
  auto mt_rr = [](const MtT& m) -> uint32_t { if constexpr (W16) return m.w & 0xFFu; else return (m.y >> 16) & 0xFFu; };
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t S2 = g.s2;
  uint4* T = reinterpret_cast<uint4*>(smem);                                            // [s][q][u]
  MtT* Mt = reinterpret_cast<MtT*>(smem + (size_t)S2 * U1 * TQ * 16);                    // [s][u]
  uint64_t* ring = reinterpret_cast<uint64_t*>(smem + (size_t)S2 * U1 * (TQ * 16 + sizeof(MtT)));  // [kRing][u]
  uint32_t* tailp = reinterpret_cast<uint32_t*>(ring + kRing * U1);                      // [u]
  uint32_t* headp = tailp + U1;                                                          // [u]
  uint32_t* resv = headp + U1;                                                           // [u] producer-private
  uint32_t* donep = resv + U1;
  uint64_t* pmask = reinterpret_cast<uint64_t*>(donep + 4);                              // [u] producer peer masks
  uint32_t* dummy = reinterpret_cast<uint32_t*>(pmask + U1);                             // [u] sink of masked-off writes
  // Cross-wave LDS words go through relaxed workgroup-scope atomics: they stay
  // ds_* instructions (a volatile generic pointer would become a flat access)
  // and keep their program order.
  auto ld32 = [](uint32_t* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto ld64 = [](uint64_t* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto st32 = [](uint32_t* q, uint32_t v) { __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto st64 = [](uint64_t* q, uint64_t v) { __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };

  const uint32_t tile = blockIdx.x;
  const uint64_t base = tile_off[tile];
  const uint32_t n = (uint32_t)(tile_off[tile + 1] - base);
  const uint32_t wave = threadIdx.x / GG_WAVE, lane = threadIdx.x % GG_WAVE;
  const uint32_t log_s2 = (uint32_t)__builtin_ctz(S2);
  const bool producer = wave == NCW;

  // ---- consumer: load + re-pack the unit's state (as k_cache_replay_lean) ----
  const uint32_t u = producer ? 0u : threadIdx.x;
  const uint64_t gu = (uint64_t)tile * U1 + u;
  const uint32_t l1set = u;
  uint32_t errv = 0;
  uint32_t st1 = 0, a1 = 0xFFFFFFFFu, pos1 = 0xFFFFFFFFu, rr1 = 0;
  auto tag_at = [&](uint32_t s, uint32_t w) -> uint32_t& {
    return reinterpret_cast<uint32_t*>(&T[((size_t)s * TQ + w / 4) * U1 + u])[w % 4];
  };
  if (!producer) {
    uint64_t t1[A1];
    const uint64_t m1 = cs.l1_meta[gu];
#pragma unroll
    for (int w = 0; w < A1; ++w) {
      t1[w] = cs.l1_tag[(uint64_t)w * g.units + gu];
      const uint32_t b = (uint32_t)(m1 >> (8 * w)) & 0xFFu;
      const uint32_t st = (t1[w] == GG_L1_INV_TAG) ? 0u : GG_M_STATE(b);
      errv |= (t1[w] != GG_L1_INV_TAG && st == GG_MS_I) ? GG_DERR_STATE : 0u;
      st1 |= st << (2 * w);
      a1 = (a1 & ~(0xFu << (4 * w))) | ((GG_M_AGE(b) & 0xFu) << (4 * w));
    }
    rr1 = cs.l1_rr[gu];
    uint32_t nheld = 0;
    for (uint32_t s = 0; s < S2; ++s) {
      uint32_t tg[4 * TQ];
#pragma unroll
      for (int w = 0; w < 4 * TQ; ++w)
        tg[w] = (w < A2) ? cs.l2_tag[(uint64_t)(s * A2 + w) * g.units + gu] : GG_L2_INV_TAG;
      uint64_t mwv[MW];
#pragma unroll
      for (int k = 0; k < MW; ++k) mwv[k] = cs.l2_meta[(uint64_t)(s * MW + k) * g.units + gu];
      AgT ages = ~(AgT)0;
      uint32_t st = 0;
#pragma unroll
      for (int w = 0; w < A2; ++w) {
        const uint32_t b = (uint32_t)(mwv[w / 8] >> (8 * (w % 8))) & 0xFFu;
        const bool valid = tg[w] != GG_L2_INV_TAG;
        errv |= (valid != (GG_M_STATE(b) != GG_MS_I)) ? GG_DERR_STATE : 0u;
        st |= (valid ? GG_M_STATE(b) : 0u) << (2 * w);
        ages = (ages & ~((AgT)0xF << (4 * w))) | ((AgT)(GG_M_AGE(b) & 0xFu) << (4 * w));
        const uint64_t ln = ((uint64_t)tg[w] << g.log_l2) | ((uint64_t)s << g.log_u1) | l1set;
        int hw = -1;
#pragma unroll
        for (int k = 0; k < A1; ++k) hw = (valid && ((st1 >> (2 * k)) & 3u) && t1[k] == ln) ? k : hw;
        nheld += (hw >= 0) ? 1u : 0u;
        errv |= ((GG_M_LOC(b) != 0) != (hw >= 0)) ? GG_DERR_STATE : 0u;
        if (hw >= 0) pos1 = (pos1 & ~(0xFFu << (8 * hw))) | ((s * A2 + w) << (8 * hw));
      }
#pragma unroll
      for (int q = 0; q < TQ; ++q)
        T[((size_t)s * TQ + q) * U1 + u] = make_uint4(tg[4 * q], tg[4 * q + 1], tg[4 * q + 2], tg[4 * q + 3]);
      const uint32_t rr = LRU2 ? 0u : cs.l2_rr[(uint64_t)s * g.units + gu];
      Mt[s * U1 + u] = mt_pack(ages, st, rr);
    }
    uint32_t nvalid = 0;
#pragma unroll
    for (int k = 0; k < A1; ++k) nvalid += ((st1 >> (2 * k)) & 3u) ? 1u : 0u;
    if (nvalid != nheld) errv |= GG_DERR_STATE;
  } else {
    for (uint32_t k = lane; k < U1; k += GG_WAVE) { tailp[k] = 0; headp[k] = 0; resv[k] = 0; }
    for (uint32_t k = lane; k < U1; k += GG_WAVE) pmask[k] = 0;
    if (lane == 0) *donep = 0;
  }
  __syncthreads();

  if (producer) {
    // ---------------- producer: program-order trace -> per-unit rings ----------------
    // Batches of K rounds x 64 records, the next two batches' loads in flight.
    // Per round, five LDS operations issued back to back (no waits between
    // rounds; one wave's LDS operations execute in order):
    //   ds_or   pmask[unit] |= lane bit      -> after the round: lanes of the unit
    //   ds_read pmask[unit]; ds_write pmask[unit] = 0
    //   ds_read resv[unit]                    -> ring position base of the round
    //   ds_add  resv[unit] += 1               -> += the round's count of the unit
    // position = base + lanes of the unit below this lane (program order).
    // Space and publication are checked per unit (lane l owns units l + 64 i).
#ifdef GG_PROD_PRIO
    __builtin_amdgcn_s_setprio(GG_PROD_PRIO);
#endif
    constexpr int K = GG_PK;
    const uint64_t* ap = addr + base;
    const uint32_t* mp = meta + base;
    const uint64_t lt_mask = (1ull << lane) - 1;
    // test knob (GG_STREAM_BAD_INDEX): the tile's first record is handed off
    // with an index past the tile's end, as a broken hand-off would; the
    // consumer must flag it (GG_DERR_CAP) and store nothing
    const uint32_t bad_idx = (dbg && dbg[6] == 1) ? n : 0u;
    uint64_t pa[K], na[K], qa[K];
    uint32_t pm[K], nm[K], qm[K];
    uint32_t bad = 0;
    bool hung = false;
    uint32_t d_batch = 0, d_slow = 0, d_spin = 0;
    // unconditional loads (index clamped to the tile's last record): no
    // branches around them, so the waits stay per-register
    auto load = [&](uint32_t c0, uint64_t (&a)[K], uint32_t (&m)[K]) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t j = min(c0 + k * GG_WAVE + lane, n - 1);
        a[k] = __builtin_nontemporal_load(ap + j);
        m[k] = __builtin_nontemporal_load(mp + j);
      }
    };
    auto batch = [&](const uint32_t c, const uint64_t (&pa)[K], const uint32_t (&pm)[K]) {
      uint64_t key[K], msk[K];
      uint32_t set[K], p[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t j = c + k * GG_WAVE + lane;
        const bool valid = j < n;
        bad |= (valid && pa[k] >= g.addr_limit) ? 1u : 0u;
        bad |= (valid && pm[k] == GG_META_BARRIER) ? 2u : 0u;      // coherent-mode records only
        const uint64_t line = pa[k] >> g.log_line;
        set[k] = valid ? (uint32_t)line & (U1 - 1) : U1;             // U1 = no record
        key[k] = ((uint64_t)(uint32_t)(line >> g.log_l2) << 32) | ((j + (j == 0 ? bad_idx : 0u)) << (1 + log_s2)) |
                 ((((uint32_t)line >> g.log_u1) & (S2 - 1)) << 1) | (pm[k] & GG_META_WRITE);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        msk[k] = 0;
        p[k] = 0;
        if (set[k] < U1) {
          __hip_atomic_fetch_or(&pmask[set[k]], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          msk[k] = ld64(&pmask[set[k]]);
          st64(&pmask[set[k]], 0ull);
          p[k] = ld32(&resv[set[k]]);
          __hip_atomic_fetch_add(&resv[set[k]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
#pragma unroll
      for (int k = 0; k < K; ++k) p[k] += (uint32_t)__popcll(msk[k] & lt_mask);
      // per unit: reserved end vs published tail (no deadlock) and consumer head (space)
      uint32_t rn[NCW];
      bool fits = true;
#pragma unroll
      for (int i = 0; i < NCW; ++i) {
        rn[i] = ld32(&resv[lane + GG_WAVE * i]);
        fits = fits && rn[i] - ld32(&tailp[lane + GG_WAVE * i]) <= kRing;
      }
      ++d_batch;
      if (__ballot(!fits) == 0) {
        for (uint32_t spin = 0;; ++spin, ++d_spin) {
          bool ok = true;
#pragma unroll
          for (int i = 0; i < NCW; ++i) ok = ok && rn[i] - ld32(&headp[lane + GG_WAVE * i]) <= kRing;
          if (__ballot(!ok) == 0) break;
          if (spin == kSpinLimit) { hung = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (set[k] < U1) st64(&ring[(p[k] % kRing) * U1 + set[k]], key[k]);
        __builtin_amdgcn_s_waitcnt(kLgkm0);                // slots written before the tails move
#pragma unroll
        for (int i = 0; i < NCW; ++i) st32(&tailp[lane + GG_WAVE * i], rn[i]);
      } else {
        // slow path (a unit with > kRing records in this batch): round by
        // round, at most kRing records of a unit per publication
        ++d_slow;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const uint32_t st = set[k];
          const uint32_t rank = (uint32_t)__popcll(msk[k] & lt_mask), cnt = (uint32_t)__popcll(msk[k]);
          for (uint32_t r0 = 0;; r0 += kRing) {
            const bool act = st < U1 && rank >= r0 && rank < r0 + kRing;
            if (!__ballot(act)) break;
            for (uint32_t spin = 0;; ++spin) {
              const bool ok = !act || (p[k] - ld32(&headp[st]) < kRing);
              if (__ballot(!ok) == 0) break;
              if (spin == kSpinLimit) { hung = true; break; }
              __builtin_amdgcn_s_sleep(1);
            }
            if (act) st64(&ring[(p[k] % kRing) * U1 + st], key[k]);
            __builtin_amdgcn_s_waitcnt(kLgkm0);
            if (act && rank == min(cnt, r0 + kRing) - 1) st32(&tailp[st], p[k] + 1);
          }
        }
      }
    };
    // the loop is unrolled by three so the buffers rotate roles without
    // register moves (a move would wait for the load it copies)
    constexpr uint32_t B = K * GG_WAVE;
    if (n) {
      load(0, pa, pm);
      load(B, na, nm);
    }
    for (uint32_t c = 0; c < n; c += 3 * B) {
      load(c + 2 * B, qa, qm);
      batch(c, pa, pm);
      if (c + B >= n) break;
      load(c + 3 * B, pa, pm);
      batch(c + B, na, nm);
      if (c + 2 * B >= n) break;
      load(c + 4 * B, na, nm);
      batch(c + 2 * B, qa, qm);
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    if (lane == 0) st32(donep, 1u);
    if (__ballot(bad & 1u) && lane == 0) atomicOr(err, GG_DERR_RANGE);
    if (__ballot(bad & 2u) && lane == 0) atomicOr(err, GG_DERR_BARRIER);
    if (hung && lane == 0) atomicOr(err, GG_DERR_CAP);
    if (dbg && lane == 0) {
      atomicAdd(&dbg[0], (unsigned long long)d_batch);
      atomicAdd(&dbg[1], (unsigned long long)d_slow);
      atomicAdd(&dbg[2], (unsigned long long)d_spin);
    }
    return;
  }

  // ---------------- consumers: one unit per lane ----------------
#ifdef GG_CONS_PRIO
  __builtin_amdgcn_s_setprio(GG_CONS_PRIO);
#endif
  // The L1-D set lives in four VGPRs: pos1 (byte w = L2 slot s*A2+w of the
  // line L1-D way w holds, 0xFF = invalid; the L1-D only holds lines its L2
  // holds, checked on entry), mbyt (0x80 in byte w iff way w is MODIFIED),
  // a1 (LRU age nibbles), rr1.  Every per-access decision is a lane mask; the
  // step has no divergent branch: the two possible L2 tag writes go to the
  // real slot or to the lane's dummy word.
  uint32_t mbyt = 0;
#pragma unroll
  for (int w = 0; w < A1; ++w) mbyt |= (((st1 >> (2 * w)) & 3u) == GG_MS_M) ? (0x80u << (8 * w)) : 0u;
  const uint32_t log_line = g.log_line, log_u1 = g.log_u1, log_l2 = g.log_l2;
  uint32_t* res_out = result ? result + base : nullptr;
  uint64_t* ev_out = EV ? evicted + base : nullptr;
  uint32_t* tag0 = reinterpret_cast<uint32_t*>(T) + 4 * u;        // tag (s, w) = tag0[(s*TQ + w/4)*4*U1 + w%4]
  uint32_t* my_dummy = dummy + u;
  // 0x80 flags of a byte mask -> 0xFF bytes
  auto bytes_of = [](uint32_t m) { return m | (m - (m >> 7)); };

  // counters: the result word's eight 1-bit nibble fields summed into byte
  // fields (even / odd nibbles), folded into u32 totals every 128 stepping
  // passes (wave-uniform, so <= 128 per byte); WRITE splits of the two miss fields in
  // two 16-bit halves.
  uint32_t f8[8], c_wr = 0, c_nh1w = 0, c_m2w = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) f8[k] = 0;
  uint32_t acc_lo = 0, acc_hi = 0, acc_w = 0;
  auto flush = [&]() {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f8[2 * k] += (acc_lo >> (8 * k)) & 0xFFu;
      f8[2 * k + 1] += (acc_hi >> (8 * k)) & 0xFFu;
    }
    c_nh1w += acc_w & 0xFFFFu;
    c_m2w += acc_w >> 16;
    acc_lo = acc_hi = acc_w = 0;
  };

  // One access; returns the result word (GG_RES_*), the evicted line through *ev.
  auto step = [&](const uint32_t kl, const uint32_t tag2, uint64_t* ev) -> uint32_t {
    const uint32_t wr = kl & 1u;
    const uint32_t s = __builtin_amdgcn_ubfe(kl, 1, log_s2);
    const uint32_t tq0 = s * TQ * 4 * U1;
    uint32_t tg[4 * TQ];
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const uint4 v = *reinterpret_cast<const uint4*>(tag0 + tq0 + q * 4 * U1);
      tg[4 * q] = v.x; tg[4 * q + 1] = v.y; tg[4 * q + 2] = v.z; tg[4 * q + 3] = v.w;
    }
    const MtT mt = Mt[s * U1 + u];
    AgT ages2 = mt_ages(mt);
    uint32_t st2 = mt_st(mt), rr2 = mt_rr(mt);
    // L2 lookup (valid tags are unique in a set; invalid ways hold the invalid tag)
    bool eq[A2];
#pragma unroll
    for (int w = 0; w < A2; ++w) eq[w] = tg[w] == tag2;
    uint32_t w2 = A2;
#pragma unroll
    for (int w = A2 - 1; w >= 0; --w) w2 = eq[w] ? (uint32_t)w : w2;
    const uint32_t has2m = w2 < A2 ? 0xFFFFFFFFu : 0u;
    // 0 when absent (8 ways and fewer: the bits above the states are 0)
    const uint32_t s2 = W16 ? (__builtin_amdgcn_ubfe(st2, 2 * (w2 & 15u), 2) & has2m) : __builtin_amdgcn_ubfe(st2, 2 * w2, 2);
    // L1-D lookup: the way naming the line's L2 slot; hit = readable (READ) or MODIFIED (WRITE)
    const uint32_t slot = s * A2 + w2;
    const uint32_t zb1 = zero_bytes32(pos1 ^ __builtin_amdgcn_perm(0u, slot, 0u)) & has2m;
    const uint32_t wrm = 0u - wr;
    const uint32_t hitb = zb1 & (~wrm | mbyt);
    const bool hit1 = hitb != 0;
    // no permission: invalidate the L1-D copy first (l1_cache_cntlr.cc:135-137)
    const uint32_t inv1 = hit1 ? 0u : zb1;
    {
      const uint32_t f = bytes_of(inv1);
      pos1 |= f;
      mbyt &= ~f;
    }
    const bool hit2n = s2 > wr;
    const bool hit2 = !hit1 && hit2n;
    const bool miss2 = !hit1 && !hit2n;
    const bool upg = miss2 && wr && s2 == GG_MS_S;
    // upgrade: invalidate the SHARED L2 line (l2_cache_cntlr.cc:260-282)
    st2 = upg ? (st2 & ~(3u << (2 * w2))) : st2;
    *(upg ? tag0 + tq0 + (w2 / 4) * 4 * U1 + (w2 % 4) : my_dummy) = GG_L2_INV_TAG;
    // L2 victim (l2_cache_cntlr.cc:74-116)
    int v2;
    if constexpr (W16) v2 = LRU2 ? victim_nib64(st2, ages2) : (int)rr2;
    else v2 = LRU2 ? victim_nib<A2>(st2, ages2) : (int)rr2;
    errv |= (miss2 && v2 < 0) ? GG_DERR_STATE : 0u;
    const uint32_t vw = (uint32_t)v2 & (A2 - 1);
    const uint32_t sv = __builtin_amdgcn_ubfe(st2, 2 * vw, 2);
    const bool l2ev = miss2 && sv != 0;
    const bool dirty = l2ev && sv == GG_MS_M;
    uint32_t vt = 0;
    if (EV) {
#pragma unroll
      for (int w = 0; w < A2; ++w) vt = (w == (int)vw) ? tg[w] : vt;
    }
    // invalidateCacheLineInL1 (l2_cache_cntlr.cc:124-131) when the L1-D holds the victim
    const uint32_t zbv = zero_bytes32(pos1 ^ __builtin_amdgcn_perm(0u, s * A2 + vw, 0u)) & (l2ev ? 0xFFFFFFFFu : 0u);
    {
      const uint32_t f = bytes_of(zbv);
      pos1 |= f;
      mbyt &= ~f;
    }
    // install (EX_REP -> MODIFIED, SH_REP -> SHARED)
    const uint32_t ns = 1u + wr;
    st2 = miss2 ? ((st2 & ~(3u << (2 * vw))) | (ns << (2 * vw))) : st2;
    *(miss2 ? tag0 + tq0 + (vw / 4) * 4 * U1 + (vw % 4) : my_dummy) = tag2;
    if (!LRU2) rr2 = miss2 ? (rr2 ? rr2 - 1 : (A2 - 1)) : rr2;
    if (LRU2) {
      AgT nb;
      if constexpr (W16) nb = lru_nib64(ages2, miss2 ? vw : (w2 & (A2 - 1)));
      else nb = lru_nib(ages2, miss2 ? vw : (w2 & (A2 - 1)));
      ages2 = (!hit1 || wr) ? nb : ages2;
    }
    Mt[s * U1 + u] = mt_pack(ages2, st2, rr2);
    // L1-D insert (insertCacheLineInL1, l2_cache_cntlr.cc:133-165) after both invalidations
    uint32_t v1;
    bool l1ev;
    if (LRU1) {
      constexpr uint32_t WM1 = (A1 >= 4) ? 0xFFFFFFFFu : ((1u << (8 * A1)) - 1);
      constexpr uint32_t NM1 = (A1 >= 8) ? 0xFFFFFFFFu : ((1u << (4 * A1)) - 1);
      const uint32_t invb = zero_bytes32(~pos1) & WM1;                     // invalid ways
      const uint32_t zn = zero_nibbles(a1 ^ ((uint32_t)(A1 - 1) * 0x11111111u)) & NM1;
      v1 = invb ? ((uint32_t)__builtin_ctz(invb) >> 3) : ((uint32_t)__builtin_ctz(zn | 0x80000000u) >> 2);
      errv |= (!hit1 && !invb && !zn) ? GG_DERR_STATE : 0u;
      l1ev = !hit1 && invb == 0;
    } else {
      v1 = rr1;
      l1ev = !hit1 && ((pos1 >> (8 * v1)) & 0xFFu) != 0xFFu;
    }
    v1 &= A1 - 1;
    {
      const uint32_t sh = 8 * v1;
      const uint32_t islot = s * A2 + (hit2 ? w2 : vw);
      const uint32_t npos = (pos1 & ~(0xFFu << sh)) | (islot << sh);
      const uint32_t nm = (mbyt & ~(0x80u << sh)) | (((hit2 ? s2 : ns) == GG_MS_M) ? (0x80u << sh) : 0u);
      pos1 = hit1 ? pos1 : npos;
      mbyt = hit1 ? mbyt : nm;
    }
    if (!LRU1) rr1 = !hit1 ? (rr1 ? rr1 - 1 : (A1 - 1)) : rr1;
    if (LRU1) a1 = lru_nib(a1, hit1 ? ((uint32_t)__builtin_ctz(hitb) >> 3) : v1);
    if (EV) {
      const uint64_t e2 = ((uint64_t)vt << log_l2) | ((uint64_t)s << log_u1) | l1set;
      *ev = l2ev ? (e2 << log_line) : ~0ull;
    }
    const uint32_t rv = (hit1 ? 0u : GG_RES_L1_MISS) | (miss2 ? GG_RES_L2_MISS : 0u) | (inv1 ? GG_RES_L1_INVAL : 0u) |
                        (l1ev ? GG_RES_L1_EVICT : 0u) | (l2ev ? GG_RES_L2_EVICT : 0u) | (dirty ? GG_RES_L2_EVICT_DIRTY : 0u) |
                        (zbv ? GG_RES_L2_EVICT_INV_L1 : 0u) | (upg ? GG_RES_UPGRADE : 0u);
    return rv;
  };
  auto count = [&](const uint32_t rv, const uint32_t wr) {
    acc_lo += rv & 0x0F0F0F0Fu;
    acc_hi += (rv >> 4) & 0x0F0F0F0Fu;
    const uint32_t x = rv & ((0u - wr) & 0x11u);
    acc_w += (x & 1u) + ((x & 0x10u) << 12);
    c_wr += wr;
  };

#ifdef GG_STREAM_NOSTEP
  const bool nostep = dbg && dbg[7] == 1;               // diagnostics build: hand-off machinery alone
#else
  constexpr bool nostep = false;
#endif
  uint32_t h = 0, idle = 0, d_iter = 0, d_sleep = 0;
  uint32_t t = ld32(&tailp[u]);
  uint64_t kn = ld64(&ring[u]);
  for (;;) {
    bool have = h < t;
    if (!__ballot(have)) {
      const uint32_t d = ld32(donep);                    // before the tails: final once set
      t = ld32(&tailp[u]);
      kn = ld64(&ring[(h % kRing) * U1 + u]);
      have = h < t;
      if (!__ballot(have)) {
        if (d) break;
        if (++idle == kSpinLimit) { errv |= GG_DERR_CAP; break; }
        ++d_sleep;
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
    }
    idle = 0;
    ++d_iter;
    const uint64_t key = kn;
    const uint32_t hn = h + (have ? 1u : 0u);
    t = ld32(&tailp[u]);                                 // next record's tail, then its slot
    kn = ld64(&ring[(hn % kRing) * U1 + u]);
    if (have) {
      const uint32_t kl = (uint32_t)key;
      const uint32_t idx = kl >> (1 + log_s2);
      uint64_t ev = 0;
      const uint32_t rv = nostep ? kl : step(kl, (uint32_t)(key >> 32), &ev);
      st32(&headp[u], hn);
      // a record index outside the tile is a broken hand-off: flagged, never stored
      const bool inr = idx < n;
      errv |= inr ? 0u : GG_DERR_CAP;
      if (res_out && inr) res_out[idx] = rv;
      if (EV && inr) ev_out[idx] = ev;
      count(rv, kl & 1u);
    }
    h = hn;
    // fold the byte fields after every 128 passes that reached here (each adds
    // at most 1 per field); idle passes `continue` above and add nothing
    if ((d_iter & 127u) == 0) flush();
  }
  flush();
  if (dbg && lane == 0) {
    atomicAdd(&dbg[3], (unsigned long long)d_iter);
    atomicAdd(&dbg[4], (unsigned long long)d_sleep);
  }
  if (dbg) atomicAdd(&dbg[5], (unsigned long long)h);

  // ---- store state back in the HBM format ----
  {
    uint64_t m1 = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      if (w < A1) {
        const uint32_t slot = (pos1 >> (8 * w)) & 0xFFu;
        const uint32_t st = slot == 0xFFu ? GG_MS_I : (((mbyt >> (8 * w + 7)) & 1u) ? GG_MS_M : GG_MS_S);
        uint64_t tag1 = GG_L1_INV_TAG;
        if (st) {
          const uint32_t ss = slot / A2, ww = slot % A2;
          tag1 = ((uint64_t)tag_at(ss, ww) << g.log_l2) | ((uint64_t)ss << g.log_u1) | l1set;
        }
        cs.l1_tag[(uint64_t)w * g.units + gu] = tag1;
        m1 |= (uint64_t)GG_M_MAKE(st, 0, (a1 >> (4 * w)) & 0xFu) << (8 * w);
      } else {
        m1 |= 0xF8ull << (8 * w);
      }
    }
    cs.l1_meta[gu] = m1;
    cs.l1_rr[gu] = (uint8_t)rr1;
    for (uint32_t s = 0; s < S2; ++s) {
      const MtT mt = Mt[s * U1 + u];
      const AgT ages = mt_ages(mt);
      const uint32_t sts = mt_st(mt);
      uint64_t mwv[MW];
#pragma unroll
      for (int k = 0; k < MW; ++k) mwv[k] = 0;
#pragma unroll
      for (int w = 0; w < 8 * MW; ++w) {
        if (w < A2) {
          const uint32_t st = (sts >> (2 * w)) & 3u;
          const uint32_t zb = zero_bytes32(pos1 ^ ((s * A2 + w) * 0x01010101u));
          mwv[w / 8] |= (uint64_t)GG_M_MAKE(st, (zb != 0) ? 1u : 0u, (uint32_t)(ages >> (4 * w)) & 0xFu) << (8 * (w % 8));
          cs.l2_tag[(uint64_t)(s * A2 + w) * g.units + gu] = tag_at(s, w);
        } else {
          mwv[w / 8] |= 0xF8ull << (8 * (w % 8));
        }
      }
#pragma unroll
      for (int k = 0; k < MW; ++k) cs.l2_meta[(uint64_t)(s * MW + k) * g.units + gu] = mwv[k];
      if (!LRU2) cs.l2_rr[(uint64_t)s * g.units + gu] = (uint8_t)mt_rr(mt);
    }
  }
  if (errv) atomicOr(err, errv);
  uint32_t cnt[NI];
  cnt[I_WR] = c_wr; cnt[I_NH1] = f8[0]; cnt[I_NH1W] = c_nh1w; cnt[I_M2] = f8[1]; cnt[I_M2W] = c_m2w;
  cnt[I_W1V] = f8[2]; cnt[I_L1EV] = f8[3]; cnt[I_L2EV] = f8[4]; cnt[I_DIRTY] = f8[5]; cnt[I_INVL1] = f8[6];
  cnt[I_UPG] = f8[7];
  replay_counters(cs, g, cnt, h, tile, lane, true);
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
typedef void (*replay_fn)(gg_cache_state, gg_geom, const uint64_t*, const uint32_t*, const uint64_t*,
                          uint32_t*, uint64_t*, uint32_t*);
typedef void (*quartet_fn)(gg_cache_state, gg_geom, QuartetIO*);

struct Kern { int a1, a2; int lru1, lru2; replay_fn replay; quartet_fn quartet; };

// Replay instantiations: every geometry with LRU (the carbon_sim.cfg default),
// all four policy combinations for the reference geometries.
#define GG_KERN(A1, A2, P1, P2) { A1, A2, P1, P2, k_cache_replay<A1, A2, P1, P2>, k_quartet<A1, A2> }
const Kern kKernels[] = {
  GG_KERN(4, 8, 1, 1), GG_KERN(4, 8, 0, 0), GG_KERN(4, 8, 1, 0), GG_KERN(4, 8, 0, 1),
  GG_KERN(4, 16, 1, 1), GG_KERN(4, 16, 0, 0), GG_KERN(4, 16, 1, 0), GG_KERN(4, 16, 0, 1),
  GG_KERN(4, 4, 1, 1), GG_KERN(2, 4, 1, 1), GG_KERN(2, 8, 1, 1), GG_KERN(2, 16, 1, 1),
  GG_KERN(8, 8, 1, 1), GG_KERN(8, 16, 1, 1), GG_KERN(8, 4, 1, 1), GG_KERN(1, 8, 1, 1),
  GG_KERN(4, 2, 1, 1), GG_KERN(4, 32, 1, 1),
};

#define GG_LEAN(A1, A2, P1, P2) { A1, A2, P1, P2, k_cache_replay_lean<A1, A2, P1, P2>, k_quartet<A1, A2> }
const Kern kLean[] = {
  GG_LEAN(4, 8, 1, 1), GG_LEAN(4, 8, 0, 0), GG_LEAN(4, 8, 1, 0), GG_LEAN(4, 8, 0, 1),
  GG_LEAN(4, 4, 1, 1), GG_LEAN(2, 4, 1, 1), GG_LEAN(2, 8, 1, 1), GG_LEAN(4, 2, 1, 1),
};

using stream_fn = void (*)(gg_cache_state, gg_geom, const uint64_t*, const uint32_t*, const uint64_t*,
                           uint32_t*, uint64_t*, uint32_t*, unsigned long long*);
struct StreamKern { int a1, a2, lru1, lru2, ncw; stream_fn plain, ev; };
#define GG_STREAM(A1, A2, P1, P2, W) \
  { A1, A2, P1, P2, W, k_cache_stream<A1, A2, P1, P2, W, false>, k_cache_stream<A1, A2, P1, P2, W, true> }
const StreamKern kStream[] = {
  GG_STREAM(4, 8, 1, 1, 2), GG_STREAM(4, 8, 0, 0, 2), GG_STREAM(4, 8, 1, 0, 2), GG_STREAM(4, 8, 0, 1, 2),
  GG_STREAM(4, 4, 1, 1, 2), GG_STREAM(2, 4, 1, 1, 2), GG_STREAM(2, 8, 1, 1, 2), GG_STREAM(4, 2, 1, 1, 2),
  GG_STREAM(4, 8, 1, 1, 1), GG_STREAM(4, 8, 1, 1, 4),
  GG_STREAM(4, 16, 1, 1, 2), GG_STREAM(4, 16, 0, 0, 2),      // configs[4]: 16-way L2
};

const StreamKern* find_stream(const gg_geom& g)
{
  const int l1 = g.pol1 == GG_POLICY_LRU, l2 = g.pol2 == GG_POLICY_LRU;
  for (const StreamKern& k : kStream)
    if ((uint32_t)k.a1 == g.a1 && (uint32_t)k.a2 == g.a2 && k.lru1 == l1 && k.lru2 == l2 &&
        (uint32_t)k.ncw * GG_WAVE == g.u1)
      return &k;
  return nullptr;
}

const Kern* find_lean(uint32_t a1, uint32_t a2, uint32_t pol1, uint32_t pol2)
{
  const int l1 = pol1 == GG_POLICY_LRU, l2 = pol2 == GG_POLICY_LRU;
  for (const Kern& k : kLean)
    if ((uint32_t)k.a1 == a1 && (uint32_t)k.a2 == a2 && k.lru1 == l1 && k.lru2 == l2) return &k;
  return nullptr;
}

const Kern* find_kernel(uint32_t a1, uint32_t a2, uint32_t pol1, uint32_t pol2)
{
  const int l1 = pol1 == GG_POLICY_LRU, l2 = pol2 == GG_POLICY_LRU;
  for (const Kern& k : kKernels)
    if ((uint32_t)k.a1 == a1 && (uint32_t)k.a2 == a2 && k.lru1 == l1 && k.lru2 == l2) return &k;
  return nullptr;
}

size_t replay_lds_bytes(const gg_geom& g, bool lean)
{
  if (lean) return (size_t)g.s2 * GG_WAVE * ((g.a2 + 3) / 4) * 16 + (size_t)g.s2 * GG_WAVE * 8;
  const size_t tq = (g.a2 + 3) / 4;
  return (size_t)g.s2 * GG_WAVE * tq * 16 + (size_t)g.s2 * GG_WAVE * g.mw * 8 +
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
  if (!find_kernel(g.a1, g.a2, g.pol1, g.pol2))
    return gg_fail(GG_ERR_UNSUPPORTED, "no replay kernel instantiated for L1-D assoc %u / L2 assoc %u / policies %u,%u",
                   g.a1, g.a2, g.pol1, g.pol2);
  if (replay_lds_bytes(g, false) > 64 * 1024)
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
  GG_HIP(hipMalloc((void**)&ctx->total_dev, sizeof(uint64_t)));
  GG_HIP(hipMalloc((void**)&ctx->tile_off_dev, sizeof(uint64_t) * (g.tiles + 1)));
  return GG_OK;
}

void gg_cache_state_free(gg_ctx* ctx)
{
  gg_cache_state& cs = ctx->cs;
  void* ps[] = {cs.l1_tag, cs.l1_meta, cs.l1_rr, cs.l2_tag, cs.l2_meta, cs.l2_rr, cs.counters,
                ctx->sh_key, ctx->sh_res, ctx->sh_ev, ctx->rec_slot, ctx->chunk_cnt, ctx->chunk_tile, ctx->chunk_start,
                ctx->chunk_len, ctx->unit_len, ctx->unit_base, ctx->tile_off_dev, ctx->total_dev};
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
  // ---- default: the single-pass streaming replay ----
  if (ctx->replay_variant == 0) {
    const StreamKern* sk = find_stream(g);
    const size_t lds = stream_lds_bytes(g.u1, g.s2, g.a2);
    uint64_t max_len = 0;
    for (uint32_t t = 0; t < g.tiles; ++t) {
      if (tr->tile_offsets[t + 1] < tr->tile_offsets[t]) return gg_fail(GG_ERR_INVALID, "tile_offsets not monotonic at tile %u", t);
      max_len = std::max<uint64_t>(max_len, tr->tile_offsets[t + 1] - tr->tile_offsets[t]);
    }
    const uint32_t log_s2 = (uint32_t)__builtin_ctz(g.s2);
    if (sk && lds <= 160 * 1024 && g.s2 * g.a2 < 255 && max_len < (1ull << (31 - log_s2))) {
      GG_HIP(hipMemcpyAsync(ctx->tile_off_dev, tr->tile_offsets, sizeof(uint64_t) * (g.tiles + 1), hipMemcpyHostToDevice, s));
      stream_fn fn = evicted ? sk->ev : sk->plain;
      GG_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      gg_timer_begin(ctx, "cache_stream", s);
      // GG_STREAM_DEBUG=1: hand-off counters of the launch on stderr (diagnostics);
      // GG_STREAM_BAD_INDEX=1 (test knob, read per batch): a broken hand-off
      // of each tile's first record (the consumer's guard must flag it)
      static const int dbg_on = getenv("GG_STREAM_DEBUG") ? atoi(getenv("GG_STREAM_DEBUG")) : 0;
      const char* bi = getenv("GG_STREAM_BAD_INDEX");
      const bool bad_index = bi && atoi(bi) == 1;
      unsigned long long* dbg = nullptr;
      if (dbg_on || bad_index) {
        GG_HIP(hipMalloc((void**)&dbg, 8 * sizeof(unsigned long long)));
        GG_HIP(hipMemsetAsync(dbg, 0, 8 * sizeof(unsigned long long), s));
        if (dbg_on == 2) GG_HIP(hipMemsetAsync(dbg + 7, 1, 1, s));   // GG_STREAM_DEBUG=2: skip the cache step (builds with -DGG_STREAM_NOSTEP)
        if (bad_index) GG_HIP(hipMemsetAsync(dbg + 6, 1, 1, s));
      }
      hipLaunchKernelGGL(fn, dim3(g.tiles), dim3((sk->ncw + 1) * GG_WAVE), lds, s, ctx->cs, g, tr->addr_dev,
                         tr->meta_dev, (const uint64_t*)ctx->tile_off_dev, result, evicted,
                         ctx->err_dev, dbg);
      GG_HIP(hipGetLastError());
      gg_timer_end(ctx, "cache_stream", s);
      if (dbg) {
        unsigned long long h[8];
        GG_HIP(hipMemcpyAsync(h, dbg, sizeof(h), hipMemcpyDeviceToHost, s));
        GG_HIP(hipStreamSynchronize(s));
        hipFree(dbg);
        if (dbg_on) fprintf(stderr, "[gg_stream] batches %llu slow %llu producer-spins %llu | consumer wave-iters %llu "
                "idle-sleeps %llu records %llu (lane util %.3f)\n", h[0], h[1], h[2], h[3], h[4], h[5],
                h[3] ? (double)h[5] / (64.0 * h[3]) : 0.0);
      }
      return GG_OK;
    }
  }
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
  // upload tables (chunk_tile doubles as storage for tile_chunk0 after the chunk entries)
  GG_HIP(hipMemcpyAsync(ctx->chunk_tile, ctx->h_chunk_tile.data(), sizeof(uint32_t) * nchunks, hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(ctx->chunk_tile + nchunks, tile_chunk0.data(), sizeof(uint32_t) * (g.tiles + 1), hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(ctx->chunk_start, ctx->h_chunk_start.data(), sizeof(uint64_t) * nchunks, hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(ctx->chunk_len, ctx->h_chunk_len.data(), sizeof(uint32_t) * nchunks, hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(ctx->tile_off_dev, tr->tile_offsets, sizeof(uint64_t) * (g.tiles + 1), hipMemcpyHostToDevice, s));

  if (nchunks) {
    gg_timer_begin(ctx, "cache_hist", s);
    hipLaunchKernelGGL(k_shard_hist, dim3((uint32_t)nchunks), dim3(256), 0, s, tr->addr_dev, tr->meta_dev, ctx->chunk_tile,
                       ctx->chunk_start, ctx->chunk_len, ctx->chunk_cnt, g, ctx->err_dev);
    GG_HIP(hipGetLastError());
  }
  uint32_t scan_threads = 64;
  while (scan_threads < g.u1) scan_threads <<= 1;
  hipLaunchKernelGGL(k_shard_scan, dim3(g.tiles), dim3(scan_threads), 0, s, ctx->chunk_cnt,
                     ctx->chunk_tile + nchunks, ctx->unit_len, g);
  GG_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_unit_scan, dim3(1), dim3(1024), 0, s, ctx->unit_len, g.units, ctx->unit_base, ctx->total_dev);
  GG_HIP(hipGetLastError());
  if (nchunks) gg_timer_end(ctx, "cache_hist", s);
  // size the sharded record buffers (one small device->host read per batch)
  uint64_t total = 0;
  GG_HIP(hipMemcpyAsync(&total, ctx->total_dev, sizeof(total), hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  if (total >= (1ull << 32)) return gg_fail(GG_ERR_RANGE, "batch needs %llu record slots (limit 2^32)", (unsigned long long)total);
  if (gg_status st = grow(&ctx->sh_key, &ctx->sh_cap, total)) return st;
  if (gg_status st = grow(&ctx->rec_slot, &ctx->rec_cap, n)) return st;
  if (result) { if (gg_status st = grow(&ctx->sh_res, &ctx->sh_res_cap, total)) return st; }
  if (evicted) { if (gg_status st = grow(&ctx->sh_ev, &ctx->sh_ev_cap, total)) return st; }
  if (nchunks) {
    gg_timer_begin(ctx, "cache_scatter", s);
    // persistent: 8 one-wave workgroups per CU, a multiple of 8 (measured
    // ahead of one chunk per workgroup, which the template still builds)
    const bool persist = true;
    const uint32_t grid = persist ? (uint32_t)std::min<uint64_t>((nchunks + 7) & ~7ull, (uint64_t)ctx->num_cus * 8)
                                  : (uint32_t)nchunks;
    const uint32_t per = std::max<uint32_t>(1, g.u1 / GG_WAVE);
    auto* fn = persist ? (per == 1 ? k_shard_scatter<1, true> : per == 2 ? k_shard_scatter<2, true> : per == 4 ? k_shard_scatter<4, true>
                          : per == 8 ? k_shard_scatter<8, true> : k_shard_scatter<16, true>)
                       : (per == 1 ? k_shard_scatter<1, false> : per == 2 ? k_shard_scatter<2, false> : per == 4 ? k_shard_scatter<4, false>
                          : per == 8 ? k_shard_scatter<8, false> : k_shard_scatter<16, false>);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(64), scatter_lds_bytes(g), s, tr->addr_dev, tr->meta_dev,
                       ctx->chunk_tile, ctx->chunk_start, ctx->chunk_len, ctx->chunk_cnt, ctx->unit_base,
                       ctx->sh_key, ctx->rec_slot, g, (uint32_t)nchunks);
    GG_HIP(hipGetLastError());
    gg_timer_end(ctx, "cache_scatter", s);
  }
  const Kern* lean = find_lean(g.a1, g.a2, g.pol1, g.pol2);
  const Kern* k = (ctx->replay_variant != 1 && lean) ? lean : find_kernel(g.a1, g.a2, g.pol1, g.pol2);
  const uint32_t groups = (uint32_t)((g.units + GG_WAVE - 1) / GG_WAVE);
  gg_timer_begin(ctx, "cache_replay", s);
  hipLaunchKernelGGL(k->replay, dim3(groups), dim3(GG_WAVE), replay_lds_bytes(g, k == lean), s, ctx->cs, g,
                     (const uint64_t*)ctx->sh_key, (const uint32_t*)ctx->unit_len, (const uint64_t*)ctx->unit_base,
                     result ? ctx->sh_res : nullptr, evicted ? ctx->sh_ev : nullptr, ctx->err_dev);
  GG_HIP(hipGetLastError());
  gg_timer_end(ctx, "cache_replay", s);
  if (n && (result || evicted)) {
    const uint64_t nb = (n + 256 * kUnshardPer - 1) / (256 * kUnshardPer);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nb, 256ull * 16);
    gg_timer_begin(ctx, "cache_unshard", s);
    hipLaunchKernelGGL(k_unshard, dim3(grid), dim3(256), 0, s, (const uint32_t*)ctx->rec_slot,
                       (const uint32_t*)ctx->sh_res, (const uint64_t*)ctx->sh_ev, result, evicted, n);
    GG_HIP(hipGetLastError());
    gg_timer_end(ctx, "cache_unshard", s);
  }
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
  hipLaunchKernelGGL(find_kernel(g.a1, g.a2, g.pol1, g.pol2)->quartet, dim3(1), dim3(1), 0, s, ctx->cs, g, d);
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
