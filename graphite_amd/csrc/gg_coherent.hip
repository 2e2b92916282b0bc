// gg_coherent.hip — the coherent ("Mode C") path on MI355X (gfx950): the
// small kernels (reset, import / export, the round) and the host side of
// gg_coherent_* / the round.  Device code and the design notes: gg_coh_dev.h;
// the step and walker kernels: gg_coh_step.hip, gg_coh_walk.hip.
#include "gg_coh_dev.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace ggc {

__global__ void k_c_import(CP P, CS S, const gg_cmsg* in, uint32_t n)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  import_one(P, S, in[i], &S.imp[0]);
}

// any BARRIER record in the trace (only gg_coherent_run releases barriers)
__global__ void k_has_barrier(const uint32_t* meta, uint64_t n, uint32_t* flag)
{
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (meta[i] == GG_META_BARRIER) { *flag = 1; return; }
}

// Status after a quantum: active / blocked tiles, least next-access start.
__global__ void k_c_status(CP P, CS S, uint64_t* out /* [active, blocked, min_next] */)
{
  const uint32_t lt = blockIdx.x * blockDim.x + threadIdx.x;
  if (lt >= P.L) return;
  const uint64_t r = S.ts[lt].rec;
  if (r >= S.ts[lt].rec_end) return;
  atomicAdd((unsigned long long*)&out[0], 1ull);
  if (S.ts[lt].blocked) { atomicAdd((unsigned long long*)&out[1], 1ull); return; }
  const uint64_t s = S.ts[lt].clk + rec_gap(S.meta[r]) * P.gap_ps;
  atomicMin((unsigned long long*)&out[2], (unsigned long long)s);
}

// constructor state of one owned tile per workgroup (its threads stride the
// tile's arrays); directory sharer words are zeroed when a slot is first used
__global__ void __launch_bounds__(256) k_c_reset(CP P, CS S, const uint64_t* offs)
{
  const uint32_t lt = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  if (lt >= P.L) return;
  const size_t n1 = (size_t)P.s1 * P.a1, n2 = (size_t)P.s2 * P.a2;
  for (size_t i = tid; i < n1; i += nt) { S.l1_tag[lt * n1 + i] = INV_ADDR; S.l1_meta[lt * n1 + i] = (uint8_t)((i % P.a1) << 3); }
  for (size_t i = tid; i < P.s1; i += nt) S.l1_rr[(size_t)lt * P.s1 + i] = (uint8_t)(P.a1 - 1);
  for (size_t i = tid; i < n2; i += nt) { S.l2_tag[lt * n2 + i] = INV_ADDR; S.l2_meta[lt * n2 + i] = (uint8_t)((i % P.a2) << 3); }
  for (size_t i = tid; i < P.s2; i += nt) S.l2_rr[(size_t)lt * P.s2 + i] = (uint8_t)(P.a2 - 1);
  for (size_t i = tid; i < P.E; i += nt) S.dir[(size_t)lt * P.E + i] = DEnt{INV_ADDR, -1, DS_UNCACHED, 0};
  if (tid < 2 * GG_NUM_CACHE_COUNTERS) S.cc[(size_t)lt * 2 * GG_NUM_CACHE_COUNTERS + tid] = 0;
  if (tid < GG_NUM_TILE_STATS) S.st[(size_t)lt * GG_NUM_TILE_STATS + tid] = 0;
  if (P.mosi && tid < GG_NUM_PROTO_STATS) S.ps[(size_t)lt * GG_NUM_PROTO_STATS + tid] = 0;
  if (P.mosi && tid == 0) S.ncdl[lt] = 0;
  if (tid == 0) {
    S.ts[lt].nrep = 0; S.ts[lt].nrq = 0;
    const uint32_t tile = S.gtile[lt];
    S.ts[lt].rec = offs[tile]; S.ts[lt].rec_end = offs[tile + 1];
    S.ts[lt].clk = 0; S.ts[lt].pend_start = 0; S.ts[lt].out_addr = INV_ADDR; S.ts[lt].out_time = 0;
    S.ts[lt].blocked = 0; S.ts[lt].seq = 0;
    reinterpret_cast<uint4*>(S.cnt4)[lt] = make_uint4(0, 0, 0, 0);
    if (P.dram_qm)                                   // QueueModel::create(dram/queue_model/type, min_processing_time)
      hq_init(S.dq + lt, S.dnd + (size_t)lt * P.max_list, P.max_list, P.dram_qtype, P.dram_qaux);
  }
}

__global__ void k_c_final_stats(CP P, CS S)
{
  const uint32_t lt = blockIdx.x * blockDim.x + threadIdx.x;
  if (lt >= P.L || !P.dram_qm) return;
  S.st[(size_t)lt * GG_NUM_TILE_STATS + GG_CT_DRAM_QUEUE_ANALYTICAL] = S.dq[lt].analytical;
  S.st[(size_t)lt * GG_NUM_TILE_STATS + GG_CT_DRAM_QUEUE_UTILIZED_NS] = S.dq[lt].util;
  S.st[(size_t)lt * GG_NUM_TILE_STATS + GG_CT_DRAM_QUEUE_LAST_NS] = S.dq[lt].last_req;
}

// export: group the boundary records by the shard they continue in
__device__ __forceinline__ uint32_t rec_shard(const CS& S, const gg_cmsg& m)
{
  return S.shard[m.hop == GG_HOP_NONE ? m.dst : m.hop];
}
__global__ void k_c_export_count(CS S, const gg_cmsg* b, uint32_t n, uint32_t* counts)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd(&counts[rec_shard(S, b[i])], 1u);
}
__global__ void k_c_export_scatter(CS S, const gg_cmsg* b, uint32_t n, const uint32_t* base, uint32_t* cursor,
                                   gg_cmsg* out)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = rec_shard(S, b[i]);
  out[base[k] + atomicAdd(&cursor[k], 1u)] = b[i];
}

// gg_round_exchange's device side (k_c_round_tail / _commit / _import, k_c_import_slots)
__global__ void k_c_ri_quantum(CS S, uint64_t q)
{
  S.ri[GG_RI_QUANTA]++;
  S.ri[GG_RI_FINAL_QUANTUM] = q;
}
// ---- one round of gg_round_exchange with one host sync (see there) --------
// words of a rank's round status (gathered over the ranks, reduced by each)
enum { RW_SENT = 0, RW_ACTIVE, RW_BLOCKED, RW_ERR, RW_MAXSLOT, RW_MINNEXT, RW_NOTDONE, RW_STEPS, RW_N };
static_assert(RW_N == kRoundWords, "gg_internal.h kRoundWords");
// before RCCL: if the quantum's steps have finished (quiet), the status of the
// owned tiles and the held records scattered into the send slots by owning
// rank; else empty slots and the not-done word.  Nothing here changes the
// context's state: a round another rank has not finished is repeated.
__global__ void __launch_bounds__(1024) k_c_round_tail(CP P, CS S, gg_cmsg* slots, uint32_t world, uint32_t per_rank,
                                                      uint64_t region, const uint32_t* err, uint32_t host_err,
                                                      uint64_t* dv)
{
  __shared__ unsigned long long st[3];                 // active, blocked, least next start
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  const uint32_t quiet = *(volatile uint32_t*)S.quiet;
  for (uint32_t r = tid; r < world; r += nt) slots[(size_t)r * (region + 1)].addr = 0;
  if (tid < 3) st[tid] = tid == 2 ? ~0ull : 0ull;
  __syncthreads();
  if (quiet) {
    for (uint32_t lt = tid; lt < P.L; lt += nt) {      // k_c_status
      const uint64_t r = S.ts[lt].rec;
      if (r >= S.ts[lt].rec_end) continue;
      atomicAdd(&st[0], 1ull);
      if (S.ts[lt].blocked) { atomicAdd(&st[1], 1ull); continue; }
      atomicMin(&st[2], (unsigned long long)(S.ts[lt].clk + rec_gap(S.meta[r]) * P.gap_ps));
    }
    const uint32_t n = *(volatile uint32_t*)S.bnd_cnt;
    for (uint32_t i = tid; i < n; i += nt) {           // the held records, by owning rank
      const uint32_t r = rec_shard(S, S.bnd[i]) / per_rank;
      gg_cmsg* sl = slots + (size_t)r * (region + 1);
      const uint64_t j = atomicAdd((unsigned long long*)&sl[0].addr, 1ull);
      if (j < region) sl[1 + j] = S.bnd[i];
      else atomicOr(S.err, GG_DERR_CAP);
    }
  }
  __threadfence();
  __syncthreads();
  if (tid != 0) return;
  uint64_t sent = 0, mx = 0;
  for (uint32_t r = 0; r < world; ++r) {
    const uint64_t c = __hip_atomic_load(&slots[(size_t)r * (region + 1)].addr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sent += c; mx = c > mx ? c : mx;
  }
  dv[RW_SENT] = sent; dv[RW_ACTIVE] = st[0]; dv[RW_BLOCKED] = st[1];
  dv[RW_ERR] = (uint64_t)(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | host_err);
  dv[RW_MAXSLOT] = mx; dv[RW_MINNEXT] = st[2];
  dv[RW_NOTDONE] = quiet ? 0ull : 1ull; dv[RW_STEPS] = quiet ? quiet - 1 : 0ull;
}
__device__ __forceinline__ bool round_go(const uint64_t* dv_all, uint32_t world)
{
  uint64_t bad = 0;
  for (uint32_t r = 0; r < world; ++r) bad |= dv_all[(size_t)r * RW_N + RW_ERR] | dv_all[(size_t)r * RW_N + RW_NOTDONE];
  return bad == 0;
}
// after RCCL, when every rank finished its quantum with no error: the
// quantum's end on this rank (step counters, held list, run info, record
// pools for the import)
__global__ void k_c_round_commit(CP P, CS S, uint64_t q, const uint64_t* dv_all, uint32_t world)
{
  if (threadIdx.x != 0 || !round_go(dv_all, world)) return;
  for (int i = 0; i < 7; ++i) S.ring[i] = 0;           // ring[4], quiet, imp[2]
  *S.bnd_cnt = 0;
  S.ri[GG_RI_QUANTA]++;
  S.ri[GG_RI_FINAL_QUANTUM] = q;
  S.npool[0] = S.npool[1] = P.L * kChunk;              // the next quantum's first step reads pool 1
}
// the received records [0, min(count, slot)) of every peer (nothing unless
// round_go), and the send / receive slot counts for the host.  The rank's
// own slot is read where the tail wrote it (its records never leave the GPU)
__global__ void k_c_round_import(CP P, CS S, const gg_cmsg* send, const gg_cmsg* recv, uint32_t world, uint32_t self,
                                 uint64_t region, uint64_t slot, const uint64_t* dv_all, uint64_t* counts)
{
  if (blockIdx.x == 0 && blockIdx.y == 0)
    for (uint32_t r = threadIdx.x; r < world; r += blockDim.x) {
      counts[r] = send[(size_t)r * (region + 1)].addr;
      counts[world + r] = (r == self ? send : recv)[(size_t)r * (region + 1)].addr;
    }
  if (!round_go(dv_all, world)) return;
  const gg_cmsg* sl = (blockIdx.y == self ? send : recv) + (size_t)blockIdx.y * (region + 1);
  const uint64_t c = sl[0].addr;
  const uint64_t e = c < slot ? c : slot;
  for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < e; i += (uint64_t)gridDim.x * blockDim.x)
    import_one(P, S, sl[1 + i], &S.imp[0]);
}

__global__ void k_c_import_slots(CP P, CS S, const gg_cmsg* slots, uint64_t region, uint64_t lo, uint64_t hi,
                                 const uint64_t* skip)
{
  if (skip && *skip) return;
  const gg_cmsg* sl = slots + (size_t)blockIdx.y * (region + 1);
  const uint64_t c = sl[0].addr;
  const uint64_t e = c < hi ? c : hi;
  for (uint64_t i = lo + blockIdx.x * blockDim.x + threadIdx.x; i < e; i += (uint64_t)gridDim.x * blockDim.x)
    import_one(P, S, sl[1 + i], &S.imp[0]);
}

}  // namespace ggc

using namespace ggc;
using namespace gg;

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct gg_coh_state {
  CP P{};
  CS S{};
  CP* Pd = nullptr;                  // device copies of P / S (k_c_step reads its launch state through them)
  CS* Sd = nullptr;
  std::vector<void*> allocs;
  uint64_t* status_dev = nullptr;
  uint32_t* ecount_dev = nullptr;    // export counts + cursors
  uint64_t* offs_dev = nullptr;
  uint64_t n_records = 0;
  size_t step_lds = 0, walk_lds = 0;
  uint32_t wtx = 64, wty = 64;          // threads of an X / Y walker workgroup
  bool persist_lc = false;
  bool begun = false;
  uint64_t gen = 0;                     // gg_coherent_begin count: a round in progress belongs to one run
  bool has_barrier = false;             // the bound trace holds BARRIER records (gg_coherent_run only)
  uint32_t* bar_flag = nullptr;
  // live kernel timing (gg_set_timing): an event pair around every
  // kTimeSample-th launch of each kernel (mode 1; a pair around every launch,
  // mode 2, costs ~18 % of a hop-by-hop run), harvested at the batch syncs;
  // since gg_coherent_begin
  std::vector<hipEvent_t> tev;
  std::vector<int> tkind;
  uint32_t tused = 0;
  // mode 2: in-kernel spans, slot s of kind k at kt[2 * (k * kKtRing + s)]
  unsigned long long* kt_dev = nullptr;
  std::vector<unsigned long long> kt_host;
  std::vector<int> kt_kind;             // kind of each slot used since the last harvest
  double kt_tick_ns = 10.0;             // s_memrealtime period
  double ksum[5] = {0, 0, 0, 0, 0};
  uint64_t kcnt[5] = {0, 0, 0, 0, 0};      // timed launches
  uint64_t nlaunch[5] = {0, 0, 0, 0, 0};   // all launches
};
constexpr uint64_t kTimeSample = 16;
constexpr uint32_t kKtRing = 1024;      // in-kernel timing slots between two harvests (a batch is <= 256 steps)
static StepArgs step_args(const gg_coh_state* C) { return StepArgs{C->Pd, C->Sd, C->S.kt, C->S.kt_slot}; }
static void launch_walk(gg_coh_state* C, hipStream_t s, uint32_t blocks, uint32_t threads, uint32_t L, int stage)
{
  ggc::launch_walk(threads > 64, walk_regq(C->P), blocks, threads, C->walk_lds, s, step_args(C), L, stage);
}
constexpr uint32_t kPersistTiles = 64;        // owned tiles up to which gg_coherent_run uses k_c_persist
constexpr uint32_t kPersistLaunches = 16384;  // launch indices per k_c_persist launch
static const char* kKernelNames[5] = {"coherent_step", "coherent_walk_x", "coherent_walk_y", "coherent_persist",
                                     "coherent_unused"};

template <class F> static void timed_launch(gg_ctx* ctx, gg_coh_state* C, hipStream_t s, int kind, F&& fn)
{
  if (ctx->timing >= 2 && !C->kt_dev)
    if (hipMalloc((void**)&C->kt_dev, sizeof(unsigned long long) * (size_t)C->S.kt_stride * kKtRing) == hipSuccess)
      C->allocs.push_back((void*)C->kt_dev);
  if (ctx->timing >= 2 && C->kt_dev && kind < 3 && C->kt_kind.size() < kKtRing) {
    C->nlaunch[kind]++;
    cs_set(C->S.kt, C->kt_dev);
    C->S.kt_slot = (uint32_t)C->kt_kind.size();
    C->kt_kind.push_back(kind);
    fn();
    C->S.kt = nullptr;
    return;
  }
  if (!ctx->timing || C->nlaunch[kind]++ % (ctx->timing >= 2 ? 1 : kTimeSample)) { fn(); return; }
  if (C->tev.size() < 2 * (size_t)(C->tused + 1)) {
    const size_t n0 = C->tev.size();
    C->tev.resize(n0 + 512);
    for (size_t i = n0; i < C->tev.size(); ++i) hipEventCreate(&C->tev[i]);
    C->tkind.resize(C->tev.size() / 2);
  }
  hipEventRecord(C->tev[2 * C->tused], s);
  fn();
  hipEventRecord(C->tev[2 * C->tused + 1], s);
  C->tkind[C->tused++] = kind;
}
static void timed_harvest(gg_coh_state* C)
{
  if (!C->kt_kind.empty()) {
    const size_t n = C->kt_kind.size(), st = C->S.kt_stride;
    C->kt_host.resize(n * st);
    if (hipMemcpy(C->kt_host.data(), C->kt_dev, 8 * n * st, hipMemcpyDeviceToHost) == hipSuccess) {
      for (size_t i = 0; i < n; ++i) {
        const int k = C->kt_kind[i];
        const uint32_t nb = k == 0 ? C->P.L : k == 1 ? C->P.nsx : C->P.nsy;   // every block stamps both words
        unsigned long long a = ~0ull, b = 0;
        for (uint32_t j = 0; j < nb; ++j) {
          a = std::min(a, C->kt_host[i * st + 2 * j]);
          b = std::max(b, C->kt_host[i * st + 2 * j + 1]);
        }
        if (nb && b >= a) { C->ksum[k] += (double)(b - a) * C->kt_tick_ns * 1e-6; C->kcnt[k]++; }
      }
    }
    C->kt_kind.clear();
  }
  for (uint32_t i = 0; i < C->tused; ++i) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, C->tev[2 * i], C->tev[2 * i + 1]) == hipSuccess) {
      C->ksum[C->tkind[i]] += ms;
      C->kcnt[C->tkind[i]]++;
    }
  }
  C->tused = 0;
}

uint64_t gg_coherent_msg_cap(gg_ctx* ctx) { return ctx->coh ? ctx->coh->P.msg_cap : 0; }

gg_status gg_coh_kernel_stats(gg_ctx* ctx, const char* name, double* total_ms, uint64_t* launches)
{
  gg_coh_state* C = ctx->coh;
  for (int k = 0; k < 5; ++k)
    if (C && std::strcmp(name, kKernelNames[k]) == 0) {
      *total_ms = C->kcnt[k] ? C->ksum[k] / (double)C->kcnt[k] * (double)C->nlaunch[k] : 0.0;
      *launches = C->nlaunch[k];
      return GG_OK;
    }
  *total_ms = 0; *launches = 0;
  return GG_ERR_INVALID;
}

static int ilog2(uint64_t v) { int p = -1; while (v) { v >>= 1; ++p; } return p; }
// both record pools empty: their shared parts start above the owned tiles'
// first-chunk slices (Tile::alloc)
__global__ void k_pool_reset(uint32_t* npool, uint32_t base) { if (threadIdx.x < 2) npool[threadIdx.x] = base; }
static hipError_t coh_pool_reset(gg_coh_state* C, hipStream_t s)
{
  hipLaunchKernelGGL(k_pool_reset, dim3(1), dim3(64), 0, s, C->S.npool, C->P.L * kChunk);
  return hipGetLastError();
}
static int clog2(uint64_t v) { int p = ilog2(v); return ((1ull << p) == v) ? p : p + 1; }
static uint64_t lat_ps_host(uint64_t cycles, double f) { return (uint64_t)ceil(((double)1000 * cycles) / f); }

template <class T> static gg_status dalloc(gg_coh_state* C, T** p, uint64_t n)
{
  void* v = nullptr;
  hipError_t e = hipMalloc(&v, sizeof(T) * (n ? n : 1));
  if (e != hipSuccess) return gg_hip_check(e, "hipMalloc(coherent state)");
  *p = (T*)v;
  C->allocs.push_back(v);
  return GG_OK;
}
template <class D, class T> static gg_status dupload(gg_coh_state* C, D* p, const std::vector<T>& v)
{
  T* d = nullptr;
  if (gg_status st = dalloc(C, &d, v.size())) return st;
  if (!v.empty()) GG_HIP(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  cs_set(*p, d);
  return GG_OK;
}

void gg_coh_free(gg_ctx* ctx)
{
  gg_coh_state* C = ctx->coh;
  if (!C) return;
  for (hipEvent_t e : C->tev) hipEventDestroy(e);
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
  CS& S = C->S;
  P.T = c.num_tiles;
  P.K = c.num_shards ? c.num_shards : 1;
  const uint32_t k0 = c.shard_begin, k1 = c.shard_end ? c.shard_end : P.K;
  if (k0 >= k1 || k1 > P.K || P.K > P.T) return gg_fail(GG_ERR_INVALID, "bad shard range [%u, %u) of %u", k0, k1, P.K);
  if (P.T > 4096) return gg_fail(GG_ERR_UNSUPPORTED, "coherent mode: more than 4096 tiles (sharer words per lane)");
  if (c.l1d_assoc > 31 || c.l2_assoc > 31) return gg_fail(GG_ERR_UNSUPPORTED, "coherent mode: associativity above 31");
  if (c.dir_assoc > 64) return gg_fail(GG_ERR_UNSUPPORTED, "coherent mode: directory associativity above 64");
  if (c.line_size != 64)       // AddressHomeLookup and the directory auto sizing use 64-byte lines here and in the oracle
    return gg_fail(GG_ERR_UNSUPPORTED, "coherent mode: line size %u (64 only)", c.line_size);
  // logical shards (the reference's hop-by-hop process blocks) and the owned tiles
  std::vector<uint32_t> shard(P.T);
  if (gg_status st = gg_shard_map(P.T, P.K, shard.data())) return st;
  std::vector<std::vector<uint32_t>> by(P.K);
  for (uint32_t t = 0; t < P.T; ++t) by[shard[t]].push_back(t);
  std::vector<uint32_t> gtile;
  {
    // equal owned shards are interleaved, so blocks b, b + ns, ... of one shard
    // share an XCD under round-robin placement (speed only)
    const uint32_t ns = k1 - k0;
    bool eq = true;
    for (uint32_t s = k0; s < k1; ++s) eq = eq && by[s].size() == by[k0].size();
    if (eq) {
      for (size_t j = 0; j < by[k0].size(); ++j)
        for (uint32_t s = 0; s < ns; ++s) gtile.push_back(by[k0 + s][j]);
    } else {
      for (uint32_t s = k0; s < k1; ++s) gtile.insert(gtile.end(), by[s].begin(), by[s].end());
    }
  }
  P.L = (uint32_t)gtile.size();
  std::vector<int32_t> ltile(P.T, -1);
  for (uint32_t l = 0; l < P.L; ++l) ltile[gtile[l]] = (int32_t)l;
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
  P.bits_ifc = P.bits_req + idb;                 // …mosi/shmem_msg.cc:137-139: + the single receiver
  if (c.protocol > GG_PROTO_SHL2_MESI)
    return gg_fail(GG_ERR_INVALID, "protocol must be GG_PROTO_MSI, _MOSI, _SHL2_MSI or _SHL2_MESI");
  P.mosi = c.protocol == GG_PROTO_MOSI ? 1u : 0u;
  P.shl2 = c.protocol == GG_PROTO_SHL2_MSI || c.protocol == GG_PROTO_SHL2_MESI ? 1u : 0u;
  P.mesi = c.protocol == GG_PROTO_SHL2_MESI ? 1u : 0u;
  if (P.shl2) {
    // pr_l1_sh_l2_msi / _mesi: the directory entries are the L2 slice's lines
    // (ShL2CacheLineInfo); set = L2CacheHashFn (l2_cache_hash_fn.cc:18-34),
    // the directory's XOR fold with log2(L2 sets) bits and no slice bits
    if (P.s2 < 2 || (P.s2 & (P.s2 - 1))) return gg_fail(GG_ERR_UNSUPPORTED, "pr_l1_sh_l2_msi: L2 sets must be a power of two >= 2");
    if (P.a2 > 64) return gg_fail(GG_ERR_UNSUPPORTED, "pr_l1_sh_l2_msi: at most 64 L2 ways");
    if (c.l2_track_miss_types) return gg_fail(GG_ERR_UNSUPPORTED, "pr_l1_sh_l2_msi: L2 miss types are not tracked");
    P.E = P.s2 * P.a2; P.dassoc = P.a2; P.log_dsets = (uint32_t)ilog2(P.s2); P.log_slices = 0;
  }
  P.dram_qm = c.dram_queue_model_enabled;
  P.dram_qtype = c.dram_queue_model_type;
  P.dram_qaux = hq_aux(c.dram_queue_model_type, c.basic_moving_avg, c.history_list_no_interleaving);
  P.max_list = c.max_list_size ? c.max_list_size : 100;
  if (P.dram_qm)
    if (gg_status e = gg_check_queue_model(P.dram_qtype, P.dram_qaux, P.max_list)) return e;
  P.analytical = c.analytical_enabled;
  P.dram_proc = (uint64_t)((float)c.line_size / c.dram_bandwidth) + 1;
  P.dram_cost = (uint64_t)(float)c.dram_latency_ns;
  P.msg_cap = (uint32_t)std::min<uint64_t>((uint64_t)64 * P.T + (uint64_t)kChunk * 2 * P.T + 65536, 0x7FFFFFFFull);
  P.np = gg_noc_params(ctx);
  P.net = c.net_model;
  P.mw = P.np.w; P.mh = P.np.h;
  P.qimg = (uint32_t)((sizeof(HQueue) + (size_t)P.np.max_size * sizeof(HNode) + 15) & ~(size_t)15);
  // hop-by-hop chain segments: the runs of each row / column inside one owned shard
  std::vector<Seg> segx, segy;
  std::vector<uint32_t> tseg((size_t)P.T * 2, ~0u);
  P.seg_xcd = 0;
  if (P.net == GG_NET_EMESH_HOP_BY_HOP) {
    if (P.mw * P.mh != P.T) return gg_fail(GG_ERR_UNSUPPORTED, "emesh_hop_by_hop needs a full W x H mesh (hop_by_hop.cc:55-59)");
    auto owned = [&](uint32_t t) { return ltile[t] >= 0; };
    const uint32_t ns = k1 - k0;
    bool inter = true;                 // every owned shard has the same number of runs per pass
    for (int pass = 0; pass < 2; ++pass) {
      const uint32_t lines = pass == 0 ? P.mh : P.mw, len = pass == 0 ? P.mw : P.mh;
      std::vector<std::vector<Seg>> per(ns);
      for (uint32_t ln = 0; ln < lines; ++ln) {
        auto at = [&](uint32_t pos) { return pass == 0 ? ln * P.mw + pos : pos * P.mw + ln; };
        uint32_t a = 0;
        while (a < len) {
          uint32_t b = a;
          while (b + 1 < len && shard[at(b + 1)] == shard[at(a)]) ++b;
          if (owned(at(a))) per[shard[at(a)] - k0].push_back(Seg{ln, a, b, 0});
          a = b + 1;
        }
      }
      for (uint32_t k = 1; k < ns; ++k) inter = inter && per[k].size() == per[0].size();
      // runs of one shard interleaved (run j of shard k at slot j * ns + k), so
      // with the walker block decode of k_c_walk a shard's walkers share the
      // XCD of its tiles under round-robin placement (speed only)
      std::vector<Seg>& out = pass == 0 ? segx : segy;
      if (inter) {
        for (size_t j = 0; j < per[0].size(); ++j)
          for (uint32_t k = 0; k < ns; ++k) out.push_back(per[k][j]);
      } else {
        for (uint32_t k = 0; k < ns; ++k) out.insert(out.end(), per[k].begin(), per[k].end());
      }
      for (uint32_t i = 0; i < out.size(); ++i) {
        const Seg& g = out[i];
        for (uint32_t q = g.lo; q <= g.hi; ++q) {
          const uint32_t t = pass == 0 ? g.line * P.mw + q : q * P.mw + g.line;
          tseg[(size_t)t * 2 + pass] = i;
        }
      }
    }
    P.seg_xcd = inter ? ns : 0;
  }
  P.nsx = (uint32_t)segx.size() * 2; P.nsy = (uint32_t)segy.size() * 2;
  uint32_t maxrun = 1, mrx = 1, mry = 1;
  for (const Seg& s : segx) mrx = std::max(mrx, s.hi - s.lo + 1);
  for (const Seg& s : segy) mry = std::max(mry, s.hi - s.lo + 1);
  maxrun = std::max(mrx, mry);
  {
    // walkers: one wave per position (the pipeline) when a run has at most
    // kMaxWalkWaves routers, else one wave sweeping the positions
    const char* sw = getenv("GG_COH_WALK_SWEEP");
    const bool sweep = sw && atoi(sw);
    C->wtx = !sweep && mrx <= kMaxWalkWaves ? 64 * mrx : 64;
    C->wty = !sweep && mry <= kMaxWalkWaves ? 64 * mry : 64;
  }
  {
    const size_t fixed = (size_t)maxrun * (P.qimg + kNetCtr * 8) + kWalkSync;
    if (P.net == GG_NET_EMESH_HOP_BY_HOP && fixed + 64 * kWalkPkBytes > kWalkLdsMax)
      return gg_fail(GG_ERR_UNSUPPORTED, "emesh_hop_by_hop: a shard's %u-router run does not fit the LDS of one walker", maxrun);
    P.walk_pk = (uint32_t)std::min<size_t>(4096, (kWalkLdsMax - fixed) / kWalkPkBytes);
    C->walk_lds = fixed + (size_t)P.walk_pk * kWalkPkBytes;
  }
  P.seg_cap = P.msg_cap;
  {
    const char* te = getenv("GG_COH_TOUCH_EACH");
    P.touch_each = te && atoi(te) ? 1u : 0u;
    const char* ww = getenv("GG_COH_WALK_WIDE");
    P.walk_wide = ww && atoi(ww) ? 1u : 0u;
    P.no_hit_runs = 0u;
  }
  C->step_lds = sizeof(StepLds);
  {
    // cache state in LDS for persistent launches of closed-form networks (no walkers)
    const size_t n1 = (size_t)P.s1 * P.a1, n2 = (size_t)P.s2 * P.a2;
    P.cache_lds_off = (uint32_t)((C->step_lds + 15) & ~(size_t)15);
    P.cache_lds_bytes = (uint32_t)(9 * (n1 + n2) + P.s1 + P.s2);
    C->persist_lc = P.net != GG_NET_EMESH_HOP_BY_HOP && (size_t)P.cache_lds_off + P.cache_lds_bytes <= 160 * 1024;
  }
  GG_HIP(step_set_lds(C->step_lds, C->persist_lc ? (size_t)P.cache_lds_off + P.cache_lds_bytes : 0,
                      std::max(C->walk_lds, C->step_lds)));
  if (P.net == GG_NET_EMESH_HOP_BY_HOP) GG_HIP(walk_set_lds(C->walk_lds));
  const uint64_t L = P.L;
  gg_status st = GG_OK;
#define A(ptr, n) if (st == GG_OK) st = dalloc(C, &S.ptr, (n))
  A(l1_tag, L * P.s1 * P.a1); A(l1_meta, L * P.s1 * P.a1); A(l1_rr, L * P.s1);
  A(l2_tag, L * P.s2 * P.a2); A(l2_meta, L * P.s2 * P.a2); A(l2_rr, L * P.s2);
  A(cc, L * 2 * GG_NUM_CACHE_COUNTERS); A(st, L * GG_NUM_TILE_STATS);
  // miss-type tracking (default off): one address table per (tile, cache)
  // (MSI's L1CacheCntlr hands the L1-D the L1-I flag, l1_cache_cntlr.cc:69; MOSI its own, …mosi/l1:68)
  P.mt1 = ((P.mosi || P.shl2) ? ctx->cfg.l1d_track_miss_types : ctx->cfg.l1i_track_miss_types) ? 1u : 0u;   // (sh_l2: its own flag, …sh_l2_msi/l1:67)
  P.mt2 = ctx->cfg.l2_track_miss_types ? 1u : 0u;
  {
    // the fast step instance: every queue it serves a history tree held in
    // registers (or no queue model), no miss types; GG_COH_NO_FAST=1 forces
    // the general instance (A/B)
    const bool rq_net = !P.np.qm || (P.np.qtype == GG_QM_HISTORY_TREE && P.np.max_size <= kQMax);
    const bool rq_dram = !P.dram_qm || (P.dram_qtype == GG_QM_HISTORY_TREE && P.max_list <= kQMax);
    const char* nf = getenv("GG_COH_NO_FAST");
    P.fast = rq_net && rq_dram && !P.mt1 && !P.mt2 && !P.mosi && !P.shl2 && !(nf && atoi(nf)) ? 1u : 0u;
  }
  if (P.mt1 || P.mt2) {
    const uint32_t lines = ctx->cfg.miss_track_lines ? ctx->cfg.miss_track_lines : 65536u;
    if (lines & (lines - 1) || lines < 64) return gg_fail(GG_ERR_INVALID, "miss_track_lines must be a power of two >= 64");
    P.mt_log = (uint32_t)__builtin_ctz(lines);
    A(mtab, (size_t)L * 2 << P.mt_log); A(mtc, L * 2 * GG_NUM_MISS_TYPES);
  }
  A(ts, L);
  A(dir, L * P.E); A(dsh, L * P.E * P.W);
  A(rep, L * P.R); A(rsh, L * P.R * P.W);
  A(rq, L * P.QC);
  if (P.mosi) {
    A(rqx, L * P.QC); A(drng, L * P.E); A(rrng, L * P.R); A(cdl, L * kCdl); A(ncdl, L); A(ps, L * GG_NUM_PROTO_STATS);
  }
  A(dq, L); A(dnd, L * P.max_list);
  A(pool0, P.msg_cap); A(pool1, P.msg_cap); A(npool, 2);
  A(inb0, L * P.IC); A(inb1, L * P.IC); A(cnt4, L * 4);
  const uint64_t al = P.net == GG_NET_EMESH_HOP_BY_HOP ? L * P.IC : 1;
  A(arv0, al); A(arv1, al);
  A(xl, (uint64_t)std::max(P.nsx, 1u) * P.seg_cap); A(nxl, std::max(P.nsx, 1u));
  A(yl, (uint64_t)std::max(P.nsy, 1u) * P.seg_cap); A(nyl, std::max(P.nsy, 1u));
  A(bnd, P.msg_cap); A(bnd_cnt, 1);
  A(ring, 11); A(ri, GG_NUM_RUN_INFO); A(qs, QS_N); A(gbar, 4);
  A(gscr, L * 6 * P.IC);
#undef A
  {
    // in-kernel launch timing slots (timing mode 2): allocated at the first
    // timed launch (timed_launch), not for every context
    S.kt_stride = 2 * std::max(std::max(P.L, P.nsx), std::max(P.nsy, 1u));
    S.kt = nullptr; S.kt_slot = 0;
  }
  S.trs = nullptr; S.trw = nullptr; S.tr_n = 0; S.tr_wb = std::max(std::max(P.nsx, P.nsy), 1u);
  // the diagnostic buffers exist only in a diagnostics build (the product
  // kernels ignore them: no buffers, no dumps of all-zero traces)
  const bool diag = GG_COH_DIAG != 0;
  if (!diag && (getenv("GG_COH_TRACE") || getenv("GG_COH_TRACE_EV") || getenv("GG_COH_PROFILE")))
    fprintf(stderr, "[gg_coh] GG_COH_TRACE / _EV / GG_COH_PROFILE need a diagnostics build "
                    "(tools/build_variant.sh diag -DGG_COH_DIAG=1; GG_LIB=variants/diag/libgraphite_gpu.so); ignored\n");
  if (diag && getenv("GG_COH_TRACE") && atoi(getenv("GG_COH_TRACE")) > 0) {
    S.tr_n = (uint32_t)atoi(getenv("GG_COH_TRACE"));
    if ((st = dalloc(C, &S.trs, (size_t)S.tr_n * P.L * kTrStep))) return st;
    if ((st = dalloc(C, &S.trw, (size_t)S.tr_n * 2 * S.tr_wb * 8))) return st;
  }
  S.tre = nullptr; S.tre_n = 0;
  if (diag && getenv("GG_COH_TRACE_EV") && atoi(getenv("GG_COH_TRACE_EV")) > 0) {
    S.tre_n = (uint32_t)atoi(getenv("GG_COH_TRACE_EV"));
    if ((st = dalloc(C, &S.tre, (size_t)S.tre_n * 2 * S.tr_wb * (kTrEvMax * 4 + 4)))) return st;
  }
  if (diag && getenv("GG_COH_PROFILE") && atoi(getenv("GG_COH_PROFILE"))) {
    if ((st = dalloc(C, &S.prof, 1024 + 8 * 65536))) return st;
    GG_HIP(hipMemset(S.prof, 0, sizeof(unsigned long long) * (1024 + 8 * 65536)));
  }
  if (st) return st;
  S.quiet = S.ring + 4; S.imp = S.ring + 5; S.live = S.ring + 7;
  if ((st = dupload(C, &S.gtile, gtile))) return st;
  if ((st = dupload(C, &S.ltile, ltile))) return st;
  if ((st = dupload(C, &S.shard, shard))) return st;
  if ((st = dupload(C, &S.segx, segx))) return st;
  if ((st = dupload(C, &S.segy, segy))) return st;
  if ((st = dupload(C, &S.tseg, tseg))) return st;
  {
    std::vector<uint4> ti(P.L);
    for (uint32_t l = 0; l < P.L; ++l)
      ti[l] = make_uint4(gtile[l], tseg[(size_t)gtile[l] * 2], tseg[(size_t)gtile[l] * 2 + 1], 0u);
    if ((st = dupload(C, &S.tinfo, ti))) return st;
  }
  if ((st = dalloc(C, &C->status_dev, 4))) return st;
  if ((st = dalloc(C, &C->Pd, 1))) return st;
  if ((st = dalloc(C, &C->Sd, 1))) return st;
  if ((st = dalloc(C, &C->ecount_dev, 2 * (uint64_t)P.K + 2))) return st;
  if ((st = dalloc(C, &C->offs_dev, (uint64_t)P.T + 1))) return st;
  cs_set(S.ctr, gg_noc_ctr(ctx));
  {
    gg::HQueue* q; gg::HNode* nd;
    gg_noc_queues(ctx, &q, &nd);
    cs_set(S.nq, q); cs_set(S.nnd, nd);
  }
  cs_set(S.err, ctx->err_dev);
  return GG_OK;
}

static gg_status coh_check(gg_ctx* ctx)
{
  uint32_t ew[2] = {0, 0};
  GG_HIP(hipMemcpy(ew, ctx->err_dev, sizeof(ew), hipMemcpyDeviceToHost));
  const uint32_t e = ew[0];
  if (e & GG_DERR_CAP) return gg_fail(GG_ERR_UNSUPPORTED, "coherent mode: a device capacity (records / inbox / "
                                      "request queue / replaced entries / call chain / segment, or with miss-type "
                                      "tracking the miss_track_lines address table of a tile) was exceeded");
  if (e & GG_DERR_STATE) return gg_fail(GG_ERR_STATE, "coherent mode: a state the reference would reject "
                                        "(LOG_ASSERT_ERROR / assert; first at gg_coh_dev.h:%u)", ew[1]);
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
  cs_set(C->S.addr, tr->addr_dev); cs_set(C->S.meta, tr->meta_dev); cs_set(C->S.out, access_out_dev);
  GG_HIP(hipMemcpyAsync(C->Pd, &C->P, sizeof(CP), hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(C->Sd, &C->S, sizeof(CS), hipMemcpyHostToDevice, s));
  C->n_records = tr->num_records;
  ++C->gen;
  for (int k = 0; k < 5; ++k) { C->ksum[k] = 0; C->kcnt[k] = 0; C->nlaunch[k] = 0; }
  C->tused = 0;
  GG_HIP(hipMemcpyAsync(C->offs_dev, tr->tile_offsets, sizeof(uint64_t) * (P.T + 1), hipMemcpyHostToDevice, s));
  if (gg_status st = gg_noc_reset(ctx, s)) return st;
  GG_HIP(hipMemsetAsync(ctx->err_dev, 0, 2 * sizeof(uint32_t), s));
  GG_HIP(hipMemsetAsync(C->S.ri, 0, sizeof(uint64_t) * GG_NUM_RUN_INFO, s));
  GG_HIP(coh_pool_reset(C, s));
  GG_HIP(hipMemsetAsync(C->S.ring, 0, sizeof(uint32_t) * 11, s));
  {
    uint64_t q0[QS_N] = {0, 0, 0, 0, 0, 0, ~0ull, 0, (uint64_t)ctx->cfg.quantum_ns * 1000ull, 0, 0, 0};
    GG_HIP(hipMemcpyAsync(C->S.qs, q0, sizeof(q0), hipMemcpyHostToDevice, s));
  }
  GG_HIP(hipMemsetAsync(C->S.bnd_cnt, 0, sizeof(uint32_t), s));
  if (C->S.tre)
    GG_HIP(hipMemsetAsync(C->S.tre, 0, sizeof(unsigned long long) * C->S.tre_n * 2 * C->S.tr_wb * (kTrEvMax * 4 + 4), s));
  if (C->S.trs) {
    GG_HIP(hipMemsetAsync(C->S.trs, 0, sizeof(unsigned long long) * C->S.tr_n * P.L * kTrStep, s));
    GG_HIP(hipMemsetAsync(C->S.trw, 0, sizeof(unsigned long long) * C->S.tr_n * 2 * C->S.tr_wb * 8, s));
  }
  if (C->S.mtab) {                                   // the miss-type address sets start empty
    GG_HIP(hipMemsetAsync(C->S.mtab, 0xFF, sizeof(uint64_t) * ((size_t)P.L * 2 << P.mt_log), s));
    GG_HIP(hipMemsetAsync(C->S.mtc, 0, sizeof(uint64_t) * P.L * 2 * GG_NUM_MISS_TYPES, s));
  }
  GG_HIP(hipMemsetAsync(C->S.nxl, 0, sizeof(uint32_t) * std::max(P.nsx, 1u), s));
  GG_HIP(hipMemsetAsync(C->S.nyl, 0, sizeof(uint32_t) * std::max(P.nsy, 1u), s));
  hipLaunchKernelGGL(k_c_reset, dim3(P.L), dim3(256), 0, s, P, C->S, (const uint64_t*)C->offs_dev);
  GG_HIP(hipGetLastError());
  uint32_t hb = 0;
  if (tr->num_records) {
    if (!C->bar_flag) {
      GG_HIP(hipMalloc((void**)&C->bar_flag, sizeof(uint32_t)));
      C->allocs.push_back(C->bar_flag);
    }
    GG_HIP(hipMemsetAsync(C->bar_flag, 0, sizeof(uint32_t), s));
    const uint64_t nb = std::min<uint64_t>(4096, (tr->num_records + 255) / 256);
    hipLaunchKernelGGL(k_has_barrier, dim3((uint32_t)nb), dim3(256), 0, s, tr->meta_dev, tr->num_records, C->bar_flag);
    GG_HIP(hipGetLastError());
    GG_HIP(hipMemcpyAsync(&hb, C->bar_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  }
  GG_HIP(hipStreamSynchronize(s));
  C->has_barrier = hb != 0;
  C->begun = true;
  return coh_check(ctx);
}

// the steps of quantum q on the owned shards (host-driven batches, one sync
// per batch to look at the quiet flag), then, enqueued without a sync: the
// step counters reset for the next quantum, the status kernel into
// C->status_dev = {active, blocked, min next start, -} and the run-info
// quantum count
static gg_status coh_quantum_steps(gg_ctx* ctx, uint64_t q)
{
  gg_coh_state* C = ctx->coh;
  if (C->has_barrier)
    return gg_fail(GG_ERR_UNSUPPORTED, "BARRIER records are released by gg_coherent_run only (one context)");
  hipStream_t s = ctx->last_stream;
  const CP& P = C->P;
  const uint64_t quantum_ps = (uint64_t)ctx->cfg.quantum_ns * 1000ull;
  const uint64_t barrier = (q + 1) * quantum_ps;
  const bool hbh = P.net == GG_NET_EMESH_HOP_BY_HOP;
  uint32_t k = 0, batch = 8;
  for (;;) {
    for (uint32_t b = 0; b < batch; ++b, ++k) {
      timed_launch(ctx, C, s, 0, [&] { launch_step(P, step_args(C), C->step_lds, s, k, 0u, barrier); });
      if (hbh) {
        if (P.nsx) timed_launch(ctx, C, s, 1, [&] { launch_walk(C, s, P.nsx, C->wtx, k, 0); });
        if (P.nsy) timed_launch(ctx, C, s, 2, [&] { launch_walk(C, s, P.nsy, C->wty, k, 1); });
      }
    }
    GG_HIP(hipGetLastError());
    uint32_t quiet = 0, err = 0;
    GG_HIP(hipMemcpyAsync(&quiet, C->S.quiet, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GG_HIP(hipMemcpyAsync(&err, ctx->err_dev, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    timed_harvest(C);
    if (err) return coh_check(ctx);
    if (quiet) break;
    if (batch < 64) batch *= 2;
  }
  // the next quantum starts from empty step counters (ring, quiet, imported packets)
  GG_HIP(hipMemsetAsync(C->S.ring, 0, sizeof(uint32_t) * 7, s));
  const uint64_t init[4] = {0, 0, ~0ull, 0};
  GG_HIP(hipMemcpyAsync(C->status_dev, init, sizeof(init), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_c_status, dim3((P.L + 63) / 64), dim3(64), 0, s, P, C->S, C->status_dev);
  hipLaunchKernelGGL(k_c_ri_quantum, dim3(1), dim3(1), 0, s, C->S, q);
  GG_HIP(hipGetLastError());
  return GG_OK;
}

gg_status gg_coherent_quantum(gg_ctx* ctx, uint64_t q, gg_coherent_status* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  gg_coh_state* C = ctx->coh;
  if (!C || !C->begun) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  if (gg_status st = coh_quantum_steps(ctx, q)) return st;
  uint64_t res[4];
  uint32_t nb = 0;
  GG_HIP(hipMemcpyAsync(res, C->status_dev, sizeof(res), hipMemcpyDeviceToHost, s));
  GG_HIP(hipMemcpyAsync(&nb, C->S.bnd_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  out->steps = 0;
  out->boundary_msgs = nb;
  out->min_next_ps = res[2];
  out->active_tiles = (uint32_t)res[0];
  out->blocked_tiles = (uint32_t)res[1];
  return coh_check(ctx);
}

// ---- the exchange of gg_round_exchange (gg_round.hip), enqueued on the
// context's stream without a host sync.  Send slots: per destination rank r
// a header record (word 0 = count) and `region` records; the records held at
// the quantum boundary are scattered to the rank that owns their shard (export
// order inside a slot does not matter: import lists them by atomics and every
// consumer orders by the canonical keys).
// Steps [k0, k0 + n) of quantum q (host-indexed launches; the launches after
// the quantum's quiet step return at once)
gg_status gg_coh_steps_async(gg_ctx* ctx, uint64_t q, uint32_t k0, uint32_t n)
{
  gg_coh_state* C = ctx->coh;
  if (!C || !C->begun) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  if (C->has_barrier)
    return gg_fail(GG_ERR_UNSUPPORTED, "BARRIER records are released by gg_coherent_run only (one context)");
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  const CP& P = C->P;
  const uint64_t barrier = (q + 1) * (uint64_t)ctx->cfg.quantum_ns * 1000ull;
  const bool hbh = P.net == GG_NET_EMESH_HOP_BY_HOP;
  for (uint32_t k = k0; k < k0 + n; ++k) {
    timed_launch(ctx, C, s, 0, [&] { launch_step(P, step_args(C), C->step_lds, s, k, 0u, barrier); });
    if (hbh) {
      if (P.nsx) timed_launch(ctx, C, s, 1, [&] { launch_walk(C, s, P.nsx, C->wtx, k, 0); });
      if (P.nsy) timed_launch(ctx, C, s, 2, [&] { launch_walk(C, s, P.nsy, C->wty, k, 1); });
    }
  }
  GG_HIP(hipGetLastError());
  return GG_OK;
}
gg_status gg_coh_round_tail(gg_ctx* ctx, gg_cmsg* slots, uint32_t world, uint32_t per_rank, uint64_t region,
                            uint32_t host_err, uint64_t* dv_own)
{
  gg_coh_state* C = ctx->coh;
  if (!C || !C->begun) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  hipLaunchKernelGGL(k_c_round_tail, dim3(1), dim3(1024), 0, ctx->last_stream, C->P, C->S, slots, world, per_rank, region,
                     (const uint32_t*)ctx->err_dev, host_err, dv_own);
  GG_HIP(hipGetLastError());
  return GG_OK;
}
gg_status gg_coh_round_import(gg_ctx* ctx, uint64_t q, const gg_cmsg* send, const gg_cmsg* recv, uint32_t world,
                              uint32_t self, uint64_t region, uint64_t slot, const uint64_t* dv_all, uint64_t* counts)
{
  gg_coh_state* C = ctx->coh;
  if (!C || !C->begun) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  hipStream_t s = ctx->last_stream;
  hipLaunchKernelGGL(k_c_round_commit, dim3(1), dim3(64), 0, s, C->P, C->S, q, dv_all, world);
  hipLaunchKernelGGL(k_c_round_import, dim3(64, world), dim3(256), 0, s, C->P, C->S, send, recv, world, self, region,
                     slot, dv_all, counts);
  GG_HIP(hipGetLastError());
  return GG_OK;
}
void gg_coh_harvest(gg_ctx* ctx) { if (ctx->coh) timed_harvest(ctx->coh); }

// import records [lo, min(count, hi)) of every received slot; `first`: the
// quantum's first import (the record pools of its first step start empty);
// nothing when *skip_if_dev != 0 (the round's reduced error flag)
gg_status gg_coh_import_slots(gg_ctx* ctx, const gg_cmsg* slots, uint32_t world, uint64_t region, uint64_t lo,
                              uint64_t hi, bool first, const uint64_t* skip_if_dev)
{
  gg_coh_state* C = ctx->coh;
  if (!C || !C->begun) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  hipStream_t s = ctx->last_stream;
  if (first) GG_HIP(coh_pool_reset(C, s));
  hipLaunchKernelGGL(k_c_import_slots, dim3(64, world), dim3(256), 0, s, C->P, C->S, slots, region, lo, hi, skip_if_dev);
  GG_HIP(hipGetLastError());
  return GG_OK;
}

gg_status gg_coh_check(gg_ctx* ctx) { return coh_check(ctx); }
uint64_t gg_coh_generation(gg_ctx* ctx) { return ctx->coh ? ctx->coh->gen : 0; }

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
  if (nb > cap) return gg_fail(GG_ERR_RANGE, "export buffer holds %llu records, %u waiting",
                               (unsigned long long)cap, nb);
  if (nb && !out_dev) return gg_fail(GG_ERR_INVALID, "NULL export buffer");
  std::vector<uint32_t> counts(P.K, 0), base(P.K, 0);
  if (nb) {
    GG_HIP(hipMemsetAsync(C->ecount_dev, 0, sizeof(uint32_t) * 2 * P.K, s));
    hipLaunchKernelGGL(k_c_export_count, dim3((nb + 255) / 256), dim3(256), 0, s, C->S, C->S.bnd, nb, C->ecount_dev);
    GG_HIP(hipMemcpyAsync(counts.data(), C->ecount_dev, sizeof(uint32_t) * P.K, hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    uint32_t a = 0;
    for (uint32_t k = 0; k < P.K; ++k) { base[k] = a; a += counts[k]; }
    GG_HIP(hipMemcpyAsync(C->ecount_dev, base.data(), sizeof(uint32_t) * P.K, hipMemcpyHostToDevice, s));
    GG_HIP(hipMemsetAsync(C->ecount_dev + P.K, 0, sizeof(uint32_t) * P.K, s));
    hipLaunchKernelGGL(k_c_export_scatter, dim3((nb + 255) / 256), dim3(256), 0, s, C->S, C->S.bnd, nb,
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
  if (n > C->P.msg_cap) return gg_fail(GG_ERR_UNSUPPORTED, "import of %llu records beyond the step pool",
                                       (unsigned long long)n);
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  // the quantum's first step reads pool 1 (messages) and walks pool 0 (held packets)
  GG_HIP(coh_pool_reset(C, s));
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
  gg_timer_begin(ctx, "coherent_run", s);
  // the quantum loop on the device (k_c_step's quantum_end): the host only
  // streams launches and looks at the run-over flag once per batch
  const CP& P = C->P;
  const bool hbh = P.net == GG_NET_EMESH_HOP_BY_HOP;
  uint32_t L = 0, batch = 16;
  // small meshes: the whole loop in persistent launches (k_c_persist), one
  // workgroup per owned tile, all resident (<= kPersistTiles << CUs)
  const char* np_env = getenv("GG_COH_NO_PERSIST");
  const char* nl_env = getenv("GG_COH_NO_LDS_CACHE");
  const bool plc = C->persist_lc && !(nl_env && atoi(nl_env));
  bool persist = P.L <= kPersistTiles && !P.mosi && !P.shl2 && !(np_env && atoi(np_env));   // (no persistent MOSI / sh_l2 instance)
  if (persist) {
    // the grid barrier needs every workgroup resident at once (a partitioned
    // device has fewer CUs): else the per-step launches
    const size_t lds = plc ? (size_t)P.cache_lds_off + P.cache_lds_bytes : std::max(C->walk_lds, C->step_lds);
    int per_cu = 0;
    if (persist_occupancy(plc, lds, &per_cu) != hipSuccess ||
        (uint64_t)per_cu * (uint64_t)ctx->num_cus < P.L)
      persist = false;
  }
  while (persist) {
    GG_HIP(hipMemsetAsync(C->S.gbar, 0, 4 * sizeof(uint32_t), s));   // counter + the three stop-vote words
    if (plc) {
      const size_t lds = P.cache_lds_off + P.cache_lds_bytes;
      timed_launch(ctx, C, s, 3, [&] { launch_persist(true, P, step_args(C), lds, s, L, L + kPersistLaunches); });
    } else {
      const size_t lds = std::max(C->walk_lds, C->step_lds);
      timed_launch(ctx, C, s, 3, [&] { launch_persist(false, P, step_args(C), lds, s, L, L + kPersistLaunches); });
    }
    GG_HIP(hipGetLastError());
    L += kPersistLaunches;
    uint64_t done = 0;
    uint32_t err = 0;
    GG_HIP(hipMemcpyAsync(&done, C->S.qs + QS_DONE, sizeof(done), hipMemcpyDeviceToHost, s));
    GG_HIP(hipMemcpyAsync(&err, ctx->err_dev, sizeof(err), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    timed_harvest(C);
    if (err || done) break;
  }
  for (; !persist;) {
    for (uint32_t b = 0; b < batch; ++b, ++L) {
      timed_launch(ctx, C, s, 0, [&] { launch_step(P, step_args(C), C->step_lds, s, L, 1u, (uint64_t)0); });
      if (hbh) {
        if (P.nsx) timed_launch(ctx, C, s, 1, [&] { launch_walk(C, s, P.nsx, C->wtx, L, 0); });
        if (P.nsy) timed_launch(ctx, C, s, 2, [&] { launch_walk(C, s, P.nsy, C->wty, L, 1); });
      }
    }
    GG_HIP(hipGetLastError());
    uint64_t done = 0;
    uint32_t err = 0;
    GG_HIP(hipMemcpyAsync(&done, C->S.qs + QS_DONE, sizeof(done), hipMemcpyDeviceToHost, s));
    GG_HIP(hipMemcpyAsync(&err, ctx->err_dev, sizeof(err), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    timed_harvest(C);
    if (err) break;
    if (done) break;
    if (batch < 256) batch *= 2;
  }
  gg_timer_end(ctx, "coherent_run", s);
  GG_HIP(hipStreamSynchronize(s));
  if (C->S.trs && getenv("GG_COH_TRACE_OUT")) {
    // raw dumps for tools/coh_trace.py: steps [n][L][16], walkers [n][2][wb][8] (u64)
    const std::string pre = getenv("GG_COH_TRACE_OUT");
    const size_t ns = (size_t)C->S.tr_n * P.L * kTrStep, nw = (size_t)C->S.tr_n * 2 * C->S.tr_wb * 8;
    std::vector<unsigned long long> h(std::max(ns, nw));
    for (int k = 0; k < 2; ++k) {
      const size_t cnt = k ? nw : ns;
      GG_HIP(hipMemcpy(h.data(), k ? C->S.trw : C->S.trs, 8 * cnt, hipMemcpyDeviceToHost));
      if (FILE* f = fopen((pre + (k ? ".walk" : ".step")).c_str(), "wb")) { fwrite(h.data(), 8, cnt, f); fclose(f); }
    }
    if (C->S.tre) {
      const size_t ne = (size_t)C->S.tre_n * 2 * C->S.tr_wb * (kTrEvMax * 4 + 4);
      std::vector<unsigned long long> he(ne);
      GG_HIP(hipMemcpy(he.data(), C->S.tre, 8 * ne, hipMemcpyDeviceToHost));
      if (FILE* f = fopen((pre + ".ev").c_str(), "wb")) { fwrite(he.data(), 8, ne, f); fclose(f); }
    }
    if (FILE* f = fopen((pre + ".meta").c_str(), "w")) {
      fprintf(f, "{\"launches\": %u, \"tiles\": %u, \"walk_blocks\": %u, \"nsx\": %u, \"nsy\": %u, \"wtx\": %u, \"wty\": %u, "
              "\"ev_first\": %u, \"ev_launches\": %u, \"ev_max\": %u}\n",
              C->S.tr_n, P.L, C->S.tr_wb, P.nsx, P.nsy, C->wtx, C->wty, kTrEv0, C->S.tre_n, kTrEvMax);
      fclose(f);
    }
  }
  if (C->S.prof) {
    // per-launch maxima in slots L mod 65536
    std::vector<unsigned long long> h(1024 + 8 * 65536);
    GG_HIP(hipMemcpy(h.data(), C->S.prof, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    unsigned long long crit = 0, wx = 0, wy = 0;
    for (int i = 0; i < 65536; ++i) { crit += h[1024 + i]; wx += h[1024 + 65536 + 2 * i]; wy += h[1024 + 65536 + 2 * i + 1]; }
    fprintf(stderr, "[gg_coh] step cycles over tiles: self %llu inbox+handlers %llu (order %llu) trace %llu publish %llu "
            "writeback %llu | slowest tile per launch %llu\n"
            "[gg_coh] walkers: %llu launches, staging %llu events %llu loop %llu handoff %llu, max events X %llu Y %llu | "
            "slowest walker per launch X %llu Y %llu | sweep: batch %llu queue load %llu requests %llu store %llu (s_memtime cycles); requests fast %llu M/G/1 %llu search %llu\n",
            h[0], h[1], h[9], h[2], h[3], h[4], crit, h[22], h[16], h[19], h[17], h[18], h[24], h[25], wx, wy, h[26], h[27], h[28], h[29], h[30], h[31], h[32]);
    {
      unsigned long long mt = 0, mx = 0, my = 0;
      for (int i = 0; i < 65536; ++i) { mt += h[1024 + 3 * 65536 + i]; mx += h[1024 + 4 * 65536 + 2 * i]; my += h[1024 + 4 * 65536 + 2 * i + 1]; }
      fprintf(stderr, "[gg_coh] tiles with SELF arrivals: %llu; cycles prologue %llu, narv %llu, gather %llu, order %llu, queue load %llu, "
              "requests + store %llu | tiles without: %llu, prologue %llu\n", h[96], h[90], h[91], h[92], h[93], h[94], h[95], h[98], h[97]);
      fprintf(stderr, "[gg_coh] per-launch max requests summed: tile (self+sent) %llu walker X %llu Y %llu\n", mt, mx, my);
      unsigned long long sn = 0, sa = 0, ss = 0, c1 = 0, c2 = 0, c3 = 0, ct = 0, nl = 0;
      for (int i = 0; i < 16384; ++i) {
        const unsigned long long* b = &h[1024 + 6 * 65536 + 4 * i];
        if (!b[0]) continue;
        ++nl; ct += b[0] >> 24;
        sn += (b[0] >> 16) & 255; sa += (b[0] >> 8) & 255; ss += b[0] & 255;
        c1 += (b[1] & 0xFFFFFF) << 8; c2 += (b[2] & 0xFFFFFF) << 8; c3 += (b[3] & 0xFFFFFF) << 8;
      }
      fprintf(stderr, "[gg_coh] slowest tile per launch (%llu launches, last 16384 indices): cycles %llu; inbox msgs %llu, SELF arrivals %llu, "
              "sent %llu; cycles self-phase %llu inbox+handlers %llu trace %llu\n", nl, ct, sn, sa, ss, c1, c2, c3);
      const char* kn[3] = {"SELF", "injection", "walker"};
      for (int k = 0; k < 3; ++k)
        fprintf(stderr, "[gg_coh] %s batches, requests by size 1|2-3|4-7|8-15|16-31|32-63|64+: %llu %llu %llu %llu %llu %llu %llu; tail requests %llu\n",
                kn[k], h[50 + 8 * k], h[51 + 8 * k], h[52 + 8 * k], h[53 + 8 * k], h[54 + 8 * k], h[55 + 8 * k], h[56 + 8 * k], h[80 + k]);
    }
    fprintf(stderr, "[gg_coh] trace: hit runs %llu cycles for %llu records (%llu calls, look-up part %llu; %llu row updates: "
            "loop %llu stores %llu); other accesses %llu cycles for %llu\n",
            h[33], h[34], h[38], h[37] - h[39], h[42], h[40] - h[37] + 0, h[41] - h[40], h[35], h[36]);
  }
  if (gg_status e = coh_check(ctx)) return e;
  uint64_t done = 0;
  GG_HIP(hipMemcpy(&done, C->S.qs + QS_DONE, sizeof(done), hipMemcpyDeviceToHost));
  if (done == 2) return gg_fail(GG_ERR_STATE, "coherent run deadlocked: tiles blocked with no message in flight");
  return GG_OK;
}

gg_status gg_coherent_get_miss_types(gg_ctx* ctx, uint64_t* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  gg_coh_state* C = ctx->coh;
  if (!C) return gg_fail(GG_ERR_INVALID, "no coherent run on this context");
  hipSetDevice(ctx->device);
  const CP& P = C->P;
  const size_t per = 2 * GG_NUM_MISS_TYPES;
  std::memset(out, 0, sizeof(uint64_t) * P.T * per);
  if (!C->S.mtc) return GG_OK;
  GG_HIP(hipStreamSynchronize(ctx->last_stream));
  std::vector<uint64_t> v((size_t)P.L * per);
  std::vector<uint32_t> gtile(P.L);
  GG_HIP(hipMemcpy(v.data(), C->S.mtc, sizeof(uint64_t) * v.size(), hipMemcpyDeviceToHost));
  GG_HIP(hipMemcpy(gtile.data(), C->S.gtile, sizeof(uint32_t) * P.L, hipMemcpyDeviceToHost));
  for (uint32_t l = 0; l < P.L; ++l)
    std::memcpy(out + (size_t)gtile[l] * per, v.data() + (size_t)l * per, sizeof(uint64_t) * per);
  return coh_check(ctx);
}

gg_status gg_coherent_get_protocol_stats(gg_ctx* ctx, uint64_t* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  gg_coh_state* C = ctx->coh;
  if (!C) return gg_fail(GG_ERR_INVALID, "no coherent run on this context");
  hipSetDevice(ctx->device);
  const CP& P = C->P;
  std::memset(out, 0, sizeof(uint64_t) * P.T * GG_NUM_PROTO_STATS);
  if (!C->S.ps) return GG_OK;                        // MSI: no MOSI counters
  GG_HIP(hipStreamSynchronize(ctx->last_stream));
  std::vector<uint64_t> v((size_t)P.L * GG_NUM_PROTO_STATS);
  std::vector<uint32_t> gtile(P.L);
  GG_HIP(hipMemcpy(v.data(), C->S.ps, sizeof(uint64_t) * v.size(), hipMemcpyDeviceToHost));
  GG_HIP(hipMemcpy(gtile.data(), C->S.gtile, sizeof(uint32_t) * P.L, hipMemcpyDeviceToHost));
  for (uint32_t l = 0; l < P.L; ++l)
    std::memcpy(out + (size_t)gtile[l] * GG_NUM_PROTO_STATS, v.data() + (size_t)l * GG_NUM_PROTO_STATS,
                sizeof(uint64_t) * GG_NUM_PROTO_STATS);
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
  hipLaunchKernelGGL(k_c_final_stats, dim3((P.L + 63) / 64), dim3(64), 0, s, P, C->S);
  GG_HIP(hipGetLastError());
  GG_HIP(hipStreamSynchronize(s));
  std::vector<uint32_t> gtile(P.L);
  GG_HIP(hipMemcpy(gtile.data(), C->S.gtile, sizeof(uint32_t) * P.L, hipMemcpyDeviceToHost));
  if (tile_stats) {
    std::vector<uint64_t> v((size_t)P.L * GG_NUM_TILE_STATS);
    GG_HIP(hipMemcpy(v.data(), C->S.st, sizeof(uint64_t) * v.size(), hipMemcpyDeviceToHost));
    std::memset(tile_stats, 0, sizeof(uint64_t) * P.T * GG_NUM_TILE_STATS);
    for (uint32_t l = 0; l < P.L; ++l)
      std::memcpy(tile_stats + (size_t)gtile[l] * GG_NUM_TILE_STATS, v.data() + (size_t)l * GG_NUM_TILE_STATS,
                  sizeof(uint64_t) * GG_NUM_TILE_STATS);
  }
  if (cache) {
    const size_t per = 2 * GG_NUM_CACHE_COUNTERS;
    std::vector<uint64_t> v((size_t)P.L * per);
    GG_HIP(hipMemcpy(v.data(), C->S.cc, sizeof(uint64_t) * v.size(), hipMemcpyDeviceToHost));
    std::memset(cache, 0, sizeof(uint64_t) * P.T * per);
    for (uint32_t l = 0; l < P.L; ++l)
      std::memcpy(cache + (size_t)gtile[l] * per, v.data() + (size_t)l * per, sizeof(uint64_t) * per);
  }
  if (run_info) GG_HIP(hipMemcpy(run_info, C->S.ri, sizeof(uint64_t) * GG_NUM_RUN_INFO, hipMemcpyDeviceToHost));
  return coh_check(ctx);
}
