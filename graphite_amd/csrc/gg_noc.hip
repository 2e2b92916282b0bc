// gg_noc.hip — EMesh packet latency on MI355X (gfx950).
//
// emesh_hop_counter (network_model_emesh_hop_counter.cc:143-157): a closed
// form per packet, one thread per packet.
//
// emesh_hop_by_hop (network_model_emesh_hop_by_hop.cc:146-264) with
// RouterModel output-port contention through QueueModelHistoryTree
// (queue_model_history_tree.cc:44-126, interval_tree.cc, queue_model_m_g_1.cc).
// Canonical order: every queue serves its packets in
// (arrival time, packet index) order.  XY routing makes the port graph a DAG
// — injection port -> X chain of the source row (LEFT or RIGHT ports) -> Y
// chain of the destination column (DOWN or UP ports) -> SELF port of the
// destination — so each stage runs its chains independently, one thread per
// chain with a private (time, index) event heap, which reproduces the order of
// one global event queue exactly.
#include "gg_dev.h"

#include <hip/hip_cooperative_groups.h>

#include <algorithm>

// The diagnostic hooks (GG_NOC_PROFILE: phase cycles) are compiled only into
// a diagnostics build (-DGG_NOC_DIAG=1): in the product kernels `prof` is a
// null constant, so the hooks and the registers they hold are gone.
#ifndef GG_NOC_DIAG
#define GG_NOC_DIAG 0
#endif
namespace {
using namespace gg;

enum { P_SELF = 0, P_LEFT, P_RIGHT, P_DOWN, P_UP, NPORTS };   // network_model_emesh_hop_by_hop.h:41-48

// ---------------------------------------------------------------------------
// hop counter / magic: one thread per packet
// ---------------------------------------------------------------------------
__global__ void k_hop_counter(NocParams P, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                              const uint32_t* __restrict__ len, const uint64_t* __restrict__ t0, uint64_t n,
                              uint64_t* arrival, uint64_t* zero_load, uint64_t* contention, uint64_t* ctr)
{
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint64_t zl = 0;
  arrival[k] = route_closed_form(P, src[k], dst[k], len[k], t0[k], zl, ctr);
  zero_load[k] = zl; contention[k] = 0;
}

// ---------------------------------------------------------------------------
// hop-by-hop
// ---------------------------------------------------------------------------
// (time, canonical key, packet): the batch API keys packets by index; the
// coherent path keys a step's messages by (send time, sender, sequence), the
// order the oracle sorts its batch into, so no global sort is needed.
struct Ev { uint64_t t; uint64_t khi; uint64_t klo; uint32_t id; uint32_t pad; };
__device__ __forceinline__ bool ev_lt(const Ev& a, const Ev& b)
{
  return a.t < b.t || (a.t == b.t && (a.khi < b.khi || (a.khi == b.khi && a.klo < b.klo)));
}
__device__ __forceinline__ void heap_push(Ev* h, uint32_t& n, Ev e)
{
  uint32_t i = n++;
  while (i > 0) { uint32_t p = (i - 1) / 2; if (!ev_lt(e, h[p])) break; h[i] = h[p]; i = p; }
  h[i] = e;
}
__device__ __forceinline__ Ev heap_pop(Ev* h, uint32_t& n)
{
  Ev top = h[0], last = h[--n];
  uint32_t i = 0;
  for (;;) {
    uint32_t l = 2 * i + 1, r = l + 1, m = i;
    Ev cand = last;
    if (l < n && ev_lt(h[l], cand)) { m = l; cand = h[l]; }
    if (r < n && ev_lt(h[r], cand)) m = r;
    if (m == i) break;
    h[i] = h[m]; i = m;
  }
  if (n) h[i] = last;
  return top;
}

struct NocDev {
  NocParams P;
  HQueue* q; HNode* nd;                // queue (tile*6 + port): ports 0..4 mesh, 5 injection
  uint64_t* ctr;
  uint32_t* err;
  __device__ HTree tree(uint32_t tile, int port) const
  {
    const uint64_t qi = (uint64_t)tile * 6 + port;
    HTree t{q + qi, nd + qi * P.max_size, 1, P.analytical != 0};
    return t;
  }
};

struct PktState {   // per-packet working state of the current batch
  uint64_t* t; uint64_t* zl; uint64_t* ct; uint32_t* cur;
  const uint64_t* khi; const uint64_t* klo;   // canonical keys, or NULL (key = packet index)
};
__device__ __forceinline__ Ev mkev(const PktState& S, uint64_t t, uint32_t k)
{
  return Ev{t, S.khi ? S.khi[k] : 0ull, S.klo ? S.klo[k] : (uint64_t)k, k, 0};
}

// Stage ids of a packet's chains
__device__ __forceinline__ uint32_t xchain_of(const NocParams& P, uint32_t s, uint32_t d)
{
  const uint32_t sx = s % P.w, sy = s / P.w, dx = d % P.w;
  if (dx == sx) return ~0u;
  return sy * 2 + (dx > sx ? 1u : 0u);        // [row][LEFT=0, RIGHT=1]
}
__device__ __forceinline__ uint32_t ychain_of(const NocParams& P, uint32_t s, uint32_t d)
{
  const uint32_t sy = s / P.w, dx = d % P.w, dy = d / P.w;
  if (dy == sy) return ~0u;
  return dx * 2 + (dy > sy ? 1u : 0u);        // [col][DOWN=0, UP=1]
}

// one mesh router hop (RouterModel::processPacket + ElectricalLinkModel::processPacket + Hop)
// through the output-port queue `tr` of `tile`
__device__ __forceinline__ void mesh_hop_q(const NocDev& D, uint32_t tile, HTree& tr, uint32_t bits, uint64_t& t, uint64_t& zl, uint64_t& ct,
                           uint64_t* lc = nullptr)
{
  // counters: straight to HBM, or to the workgroup's LDS block of this tile (lc, flushed at the end)
  auto add = [&](int k, uint64_t v) { if (lc) lc[k] += v; else cadd(D.ctr, tile, k, v); };
  const NocParams& P = D.P;
  const uint64_t nf = nflits(P, bits);
  uint64_t zlc = P.router_delay, qd = 0;
  if (P.qm) {
    qd = tr.delay(time_to_cycles(t, P.f), nf, D.err);
    add(GG_NC_ROUTER_CONTENTION_CYCLES, qd);
    add(GG_NC_ROUTER_PACKETS, 1);
  }
  add(GG_NC_BUFFER_WRITES, nf); add(GG_NC_BUFFER_READS, nf);
  add(GG_NC_SWITCH_ALLOC, 1); add(GG_NC_CROSSBAR, nf);
  zlc += P.link_delay;
  add(GG_NC_LINK_TRAVERSALS, nf);
  const uint64_t zps = lat_to_ps(zlc, P.f), cps = lat_to_ps(qd, P.f);
  t += zps + cps; zl += zps; ct += cps;
}
__device__ void mesh_hop(const NocDev& D, uint32_t tile, int port, uint32_t bits, uint64_t& t, uint64_t& zl, uint64_t& ct)
{
  HTree tr = D.tree(tile, port);
  mesh_hop_q(D, tile, tr, bits, t, zl, ct);
}

// ---------------------------------------------------------------------------
// LDS-staged queues.  A stage walks its packets in event order and every
// queue operation is a chain of dependent node accesses (AVL search, insert,
// rebalance); from HBM/L2 each costs a memory round trip.  The staged
// kernels copy the queues a workgroup owns (a chain's w or h ports, or 16
// tiles' injection / SELF ports) into LDS once per launch, run the same code
// on the LDS image and write it back.  Image = HQueue | max_size HNode.
// ---------------------------------------------------------------------------
__host__ __device__ inline uint32_t qimg_bytes(uint32_t ms)
{
  return (uint32_t)((sizeof(HQueue) + ms * sizeof(HNode) + 15) & ~15u);
}
__device__ inline HTree qimg_tree(uint8_t* img, uint32_t ms, bool analytical)
{
  HTree t{reinterpret_cast<HQueue*>(img), reinterpret_cast<HNode*>(img + sizeof(HQueue)), 1, analytical};
  return t;
}
static_assert(sizeof(HQueue) % 8 == 0 && sizeof(HNode) % 8 == 0, "8-byte images");
// Cooperative copy (all threads of the block) between HBM and the LDS images
// of n queues (image slot s <- queue qid(s)), slots with skip(s) left alone.
// One flat index space over all images, 8 independent loads in flight per
// thread before their stores (a per-queue word loop waits one memory round
// trip per 8-byte word, which dominated the short per-step launches of the
// coherent hop-by-hop path).
template <bool TO_LDS, class Qid, class Skip>
__device__ void qimg_copy_set(const NocDev& D, uint32_t n, Qid qid, Skip skip, uint8_t* base, uint32_t qb)
{
  const uint32_t ms = D.P.max_size, tid = threadIdx.x, nt = blockDim.x;
  constexpr uint32_t QW = sizeof(HQueue) / 8;
  const uint32_t NW = ms * (uint32_t)(sizeof(HNode) / 8);
  const uint32_t per = QW + NW;                    // 8-byte words of queue + nodes
  const uint32_t total = n * per;
  constexpr uint32_t U = 8;
  for (uint32_t i0 = tid; i0 < total; i0 += U * nt) {
    uint64_t v[U];
    #pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * nt;
      if (i >= total) break;
      const uint32_t s = i / per, w = i % per;
      if (skip(s)) continue;
      const uint64_t qi = qid(s);
      uint8_t* img = base + (size_t)s * qb;
      if (w < QW) v[u] = TO_LDS ? reinterpret_cast<const uint64_t*>(D.q + qi)[w] : reinterpret_cast<uint64_t*>(img)[w];
      else {
        const uint32_t j = w - QW;
        v[u] = TO_LDS ? reinterpret_cast<const uint64_t*>(D.nd + qi * ms)[j]
                      : reinterpret_cast<uint64_t*>(img + sizeof(HQueue))[j];
      }
    }
    #pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * nt;
      if (i >= total) break;
      const uint32_t s = i / per, w = i % per;
      if (skip(s)) continue;
      const uint64_t qi = qid(s);
      uint8_t* img = base + (size_t)s * qb;
      if (w < QW) {
        if (TO_LDS) reinterpret_cast<uint64_t*>(img)[w] = v[u]; else reinterpret_cast<uint64_t*>(D.q + qi)[w] = v[u];
      } else {
        const uint32_t j = w - QW;
        if (TO_LDS) reinterpret_cast<uint64_t*>(img + sizeof(HQueue))[j] = v[u];
        else reinterpret_cast<uint64_t*>(D.nd + qi * ms)[j] = v[u];
      }
    }
  }
}

// Stage 0: injection port of each source tile, packets in (time, index) order.
__device__ void inject_tile(const NocDev& D, uint32_t tile, const uint32_t* __restrict__ len,
                            const uint64_t* __restrict__ bucket_off, const uint32_t* __restrict__ bucket_ids, Ev* heap,
                            const PktState& S)
{
  const uint64_t b = bucket_off[tile], e = bucket_off[tile + 1];
  Ev* h = heap + b;
  uint32_t n = 0;
  for (uint64_t i = b; i < e; ++i) { uint32_t k = bucket_ids[i]; heap_push(h, n, mkev(S, S.t[k], k)); }
  HTree tr = D.tree(tile, 5);
  while (n) {
    Ev ev = heap_pop(h, n);
    const uint32_t k = ev.id;
    const uint64_t nf = nflits(D.P, len[k]);
    cadd(D.ctr, tile, GG_NC_PACKETS_SENT, 1); cadd(D.ctr, tile, GG_NC_FLITS_SENT, nf);
    cadd(D.ctr, tile, GG_NC_BITS_SENT, len[k]);
    uint64_t qd = 0;
    if (D.P.qm) qd = tr.delay(time_to_cycles(S.t[k], D.P.f), nf, D.err);   // injection router: delay 0
    const uint64_t cps = lat_to_ps(qd, D.P.f);
    S.t[k] += lat_to_ps(0, D.P.f) + cps;
    S.ct[k] += cps;
  }
}
// Stages X and Y, chains whose queue images do not fit LDS (large
// max_list_size): one thread per chain, ports along the chain in (time,
// index) order, queues in HBM.
__global__ void k_chain(NocDev D, int stage, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                        const uint32_t* __restrict__ len, const uint64_t* __restrict__ bucket_off,
                        const uint32_t* __restrict__ bucket_ids, Ev* heap, PktState S, uint32_t nchains)
{
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchains) return;
  const NocParams& P = D.P;
  const uint64_t b = bucket_off[c], e = bucket_off[c + 1];
  Ev* h = heap + b;
  uint32_t n = 0;
  for (uint64_t i = b; i < e; ++i) { uint32_t k = bucket_ids[i]; heap_push(h, n, mkev(S, S.t[k], k)); }
  while (n) {
    Ev ev = heap_pop(h, n);
    const uint32_t k = ev.id;
    const uint32_t cur = S.cur[k], d = dst[k];
    const uint32_t cx = cur % P.w, cy = cur / P.w, dx = d % P.w, dy = d / P.w;
    int port; uint32_t next; bool done;
    if (stage == 0) {                       // X: LEFT / RIGHT until the destination column
      port = (cx > dx) ? P_LEFT : P_RIGHT;
      next = (cx > dx) ? cur - 1 : cur + 1;
      done = (next % P.w) == dx;
    } else {                                // Y: DOWN / UP until the destination row
      port = (cy > dy) ? P_DOWN : P_UP;
      next = (cy > dy) ? cur - P.w : cur + P.w;
      done = (next / P.w) == dy;
    }
    uint64_t t = S.t[k], zl = S.zl[k], ct = S.ct[k];
    mesh_hop(D, cur, port, len[k], t, zl, ct);
    S.t[k] = t; S.zl[k] = zl; S.ct[k] = ct; S.cur[k] = next;
    if (!done) heap_push(h, n, mkev(S, t, k));
    (void)cx; (void)cy;
  }
}

// Final stage: SELF port of each destination + receive (processReceivedPacket).
__device__ void self_tile(const NocDev& D, uint32_t tile, const uint32_t* __restrict__ len,
                          const uint64_t* __restrict__ bucket_off, const uint32_t* __restrict__ bucket_ids, Ev* heap,
                          const PktState& S)
{
  const uint64_t b = bucket_off[tile], e = bucket_off[tile + 1];
  Ev* h = heap + b;
  uint32_t n = 0;
  for (uint64_t i = b; i < e; ++i) { uint32_t k = bucket_ids[i]; heap_push(h, n, mkev(S, S.t[k], k)); }
  while (n) {
    Ev ev = heap_pop(h, n);
    const uint32_t k = ev.id;
    uint64_t t = S.t[k], zl = S.zl[k], ct = S.ct[k];
    mesh_hop(D, tile, P_SELF, len[k], t, zl, ct);
    const uint64_t nf = nflits(D.P, len[k]);
    const uint64_t ser = lat_to_ps(nf, D.P.f);
    t += ser; zl += ser;
    cadd(D.ctr, tile, GG_NC_PACKETS_RECEIVED, 1); cadd(D.ctr, tile, GG_NC_FLITS_RECEIVED, nf);
    cadd(D.ctr, tile, GG_NC_BITS_RECEIVED, len[k]);
    cadd(D.ctr, tile, GG_NC_TOTAL_LATENCY_PS, zl + ct); cadd(D.ctr, tile, GG_NC_TOTAL_CONTENTION_PS, ct);
    S.t[k] = t; S.zl[k] = zl; S.ct[k] = ct;
  }
}
// Staged packets: a workgroup's packets (a contiguous bucket range [B, E))
// gathered into LDS next to its queues — the event heap, the working times
// and the canonical keys — so the serial event walk touches no HBM; written
// back at the end.  Used when they fit (kPktLdsBytes per packet), else the
// walk keeps its heap and packet state in HBM.
constexpr size_t kStageLdsMax = 160 * 1024 - 64;   // leaves room for k_chain_staged's static position range
constexpr uint32_t kPktLdsBytes = sizeof(Ev) + 5 * 8 + 4 * 4;
constexpr uint32_t kCtrBytes = GG_NUM_NET_COUNTERS * 8;   // a tile's counter block in LDS
__device__ void lctr_zero(uint64_t* lc, uint32_t ntiles)
{
  for (uint32_t i = threadIdx.x; i < ntiles * GG_NUM_NET_COUNTERS; i += blockDim.x) lc[i] = 0;
}
template <class TileAt>
__device__ void lctr_flush(const NocDev& D, const uint64_t* lc, uint32_t ntiles, TileAt tile_at)
{
  for (uint32_t i = threadIdx.x; i < ntiles * GG_NUM_NET_COUNTERS; i += blockDim.x)
    if (lc[i]) cadd(D.ctr, tile_at(i / GG_NUM_NET_COUNTERS), (int)(i % GG_NUM_NET_COUNTERS), lc[i]);
}
struct LPk {
  Ev* heap; uint64_t *t, *zl, *ct, *khi, *klo; uint32_t *cur, *dst, *len, *gid;
  __device__ LPk(uint8_t* base, uint32_t np)
  {
    heap = reinterpret_cast<Ev*>(base);
    t = reinterpret_cast<uint64_t*>(heap + np); zl = t + np; ct = zl + np; khi = ct + np; klo = khi + np;
    cur = reinterpret_cast<uint32_t*>(klo + np); dst = cur + np; len = dst + np; gid = len + np;
  }
  __device__ Ev ev(uint32_t i) const { return Ev{t[i], khi[i], klo[i], i, 0}; }
};
__device__ void lpk_load(LPk& L, uint64_t B, uint32_t np, const uint32_t* bucket_ids, const PktState& S,
                         const uint32_t* dst, const uint32_t* len)
{
  for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
    const uint32_t k = bucket_ids[B + i];
    L.gid[i] = k; L.t[i] = S.t[k]; L.zl[i] = S.zl[k]; L.ct[i] = S.ct[k]; L.cur[i] = S.cur[k];
    L.dst[i] = dst[k]; L.len[i] = len[k];
    L.khi[i] = S.khi ? S.khi[k] : 0ull; L.klo[i] = S.klo ? S.klo[k] : (uint64_t)k;
  }
}
__device__ void lpk_store(const LPk& L, uint32_t np, const PktState& S)
{
  for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
    const uint32_t k = L.gid[i];
    S.t[k] = L.t[i]; S.zl[k] = L.zl[i]; S.ct[k] = L.ct[i]; S.cur[k] = L.cur[i];
  }
}

// Staged stages X / Y, the general form: one workgroup per chain (row or
// column, direction), the chain's w (or h) output-port queues in LDS; thread
// 0 walks the events.  k_chain_sweep falls back to it for chains outside its
// limits (any queue model, any batch size or time range).
__device__ void chain_staged(NocDev D, int stage, const uint32_t* __restrict__ dst,
    const uint32_t* __restrict__ len, const uint64_t* __restrict__ bucket_off,
    const uint32_t* __restrict__ bucket_ids, Ev* heap, PktState S, uint32_t c)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t qlds[];
  const NocParams& P = D.P;
  const uint32_t line = c / 2, dir = c % 2;
  const uint64_t b = bucket_off[c], e = bucket_off[c + 1];
  if (b == e) return;
  const uint32_t ms = P.max_size, qb = qimg_bytes(ms);
  const uint32_t Lq = stage == 0 ? P.w : P.h;
  const uint32_t np = (uint32_t)(e - b);
  const bool lp = (size_t)Lq * (qb + kCtrBytes) + (size_t)np * kPktLdsBytes <= kStageLdsMax;
  uint64_t* lcb = reinterpret_cast<uint64_t*>(qlds + Lq * qb);
  LPk L(qlds + Lq * (qb + kCtrBytes), lp ? np : 0u);
  const int port = stage == 0 ? (dir ? P_RIGHT : P_LEFT) : (dir ? P_UP : P_DOWN);   // xchain_of / ychain_of
  auto tile_at = [&](uint32_t i) -> uint32_t { return stage == 0 ? line * P.w + i : i * P.w + line; };
  // only the ports between a packet's current and destination position can be
  // visited: stage the chain's queues in that position range
  __shared__ uint32_t s_lo, s_hi;
  if (threadIdx.x == 0) { s_lo = ~0u; s_hi = 0; }
  if (lp) lpk_load(L, b, np, bucket_ids, S, dst, len);
  if (lp) lctr_zero(lcb, Lq);
  __syncthreads();
  {
    auto pos_of = [&](uint32_t tile) { return stage == 0 ? tile % P.w : tile / P.w; };
    uint32_t lo = ~0u, hi = 0;
    for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
      const uint32_t cur = lp ? L.cur[i] : S.cur[bucket_ids[b + i]];
      const uint32_t d = lp ? L.dst[i] : dst[bucket_ids[b + i]];
      const uint32_t a = pos_of(cur), z = pos_of(d);
      lo = min(lo, min(a, z)); hi = max(hi, max(a, z));
    }
    if (lo <= hi) { atomicMin(&s_lo, lo); atomicMax(&s_hi, hi); }
  }
  __syncthreads();
  const uint32_t plo = s_lo, phi = s_hi;
  auto cq = [&](uint32_t i) { return (uint64_t)tile_at(i) * 6 + port; };
  auto cskip = [&](uint32_t i) { return i < plo || i > phi; };
  qimg_copy_set<true>(D, Lq, cq, cskip, qlds, qb);
  __syncthreads();
  if (threadIdx.x == 0) {
    // one hop of packet (cur, d) along the chain; returns whether it left the chain
    auto hop = [&](uint32_t cur, uint32_t d, uint32_t bits, uint64_t& t, uint64_t& zl, uint64_t& ct,
                   uint32_t& next) -> bool {
      uint32_t pos;
      bool done;
      if (stage == 0) { next = dir ? cur + 1 : cur - 1; done = (next % P.w) == d % P.w; pos = cur % P.w; }
      else { next = dir ? cur + P.w : cur - P.w; done = (next / P.w) == d / P.w; pos = cur / P.w; }
      HTree tr = qimg_tree(qlds + pos * qb, ms, P.analytical != 0);
      mesh_hop_q(D, cur, tr, bits, t, zl, ct, lp ? lcb + pos * GG_NUM_NET_COUNTERS : nullptr);
      return done;
    };
    uint32_t n = 0;
    if (lp) {
      Ev* h = L.heap;
      for (uint32_t i = 0; i < np; ++i) heap_push(h, n, L.ev(i));
      while (n) {
        const uint32_t i = heap_pop(h, n).id;
        uint32_t next;
        uint64_t t = L.t[i], zl = L.zl[i], ct = L.ct[i];
        const bool done = hop(L.cur[i], L.dst[i], L.len[i], t, zl, ct, next);
        L.t[i] = t; L.zl[i] = zl; L.ct[i] = ct; L.cur[i] = next;
        if (!done) heap_push(h, n, L.ev(i));
      }
    } else {
      Ev* h = heap + b;
      for (uint64_t i = b; i < e; ++i) { uint32_t k = bucket_ids[i]; heap_push(h, n, mkev(S, S.t[k], k)); }
      while (n) {
        const uint32_t k = heap_pop(h, n).id;
        uint32_t next;
        uint64_t t = S.t[k], zl = S.zl[k], ct = S.ct[k];
        const bool done = hop(S.cur[k], dst[k], len[k], t, zl, ct, next);
        S.t[k] = t; S.zl[k] = zl; S.ct[k] = ct; S.cur[k] = next;
        if (!done) heap_push(h, n, mkev(S, t, k));
      }
    }
  }
  __syncthreads();
  if (lp) lpk_store(L, np, S);
  if (lp) lctr_flush(D, lcb, Lq, tile_at);
  qimg_copy_set<false>(D, Lq, cq, cskip, qlds, qb);
}

// ---------------------------------------------------------------------------
// Stages X / Y as a position sweep (the default): one workgroup per chain.
// In a chain the packets move one way, so the requests a port sees depend
// only on the ports before it: the sweep visits the positions in the
// direction of travel; the batch of a position = the packets that left the
// position before it + those whose route starts there, sorted by (arrival
// time, packet index) — the order of the global event queue at that port —
// by the workgroup's threads (bitonic, LDS); one wave serves the batch
// through the port's history tree held in its registers (RegQueue); the
// lanes then split the batch into packets leaving the chain (time, zero-load
// / contention parts and position written back) and the next position's
// arrivals.  A batch entry is (time, i), i the packet's rank by index among
// the chain's packets (their ids sorted first).  Limits (else chain_staged):
// <= kSweepPk packets, <= kSweepPos positions, history_tree queues of <=
// kQMaxNoc intervals (or no queue model), flits < 2^16.
// ---------------------------------------------------------------------------
constexpr uint32_t kSweepPk = 6144, kSweepSort = 8192, kSweepPos = 256, kSweepThreads = 256, kQMaxNoc = 128;
struct SK { uint64_t t; uint32_t i, pad; };
static_assert(sizeof(SK) == 16 && sizeof(Ev) >= 2 * sizeof(SK), "start runs + arrivals fit a bucket's Ev scratch");
constexpr size_t kSweepLds = (size_t)kSweepSort * sizeof(SK) + (size_t)kSweepPk * 4 + kSweepPos * 8 + 64;
__device__ __forceinline__ bool sk_lt(const SK& a, const SK& b) { return a.t < b.t || (a.t == b.t && a.i < b.i); }
__device__ __forceinline__ void nsync()   // LDS ordering between the lanes of one wave of a multi-wave workgroup
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ uint64_t wave_sum64n(uint64_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((long long)v, o);
  return v;
}

// ascending bitonic sort of a[0, M), M a power of two, all threads of the block
template <class T, class Lt>
__device__ void block_bitonic(T* a, uint32_t M, Lt lt)
{
  for (uint32_t k = 2; k <= M; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < M; i += blockDim.x) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const T x = a[i], y = a[l];
          if (((i & k) == 0) == lt(y, x)) { a[i] = y; a[l] = x; }
        }
      }
      __syncthreads();
    }
}

__device__ void chain_sweep(NocDev D, int stage, const uint32_t* __restrict__ dst,
    const uint32_t* __restrict__ len, const uint64_t* __restrict__ bucket_off, uint32_t* __restrict__ bucket_ids,
    Ev* heap, PktState S, unsigned long long* prof, uint32_t c)
{
  // prof (GG_NOC_PROFILE=1, diagnostics): shader-clock cycles of the setup, the
  // per-position sorts, serves and hand-offs, requests served, over the chains
  const uint64_t c_0 = prof ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t c_sort = 0, c_serve = 0, c_part = 0, c_set = 0, nreq = 0;
  extern __shared__ __attribute__((aligned(16))) uint8_t qlds[];
  const NocParams& P = D.P;
  const uint32_t line = c / 2, dir = c % 2, tid = threadIdx.x, ln = tid & 63;
  const uint64_t b = bucket_off[c], e = bucket_off[c + 1];
  if (b == e) return;
  const uint32_t n = (uint32_t)min<uint64_t>(e - b, 0xFFFFFFFFull);
  const uint32_t npos = stage == 0 ? P.w : P.h;
  const bool regq = P.qtype == GG_QM_HISTORY_TREE && P.max_size <= kQMaxNoc;
  __shared__ uint32_t s_bad, s_na;
  if (tid == 0) s_bad = 0;
  __syncthreads();
  if (n > kSweepPk || npos > kSweepPos || (P.qm && !regq)) { chain_staged(D, stage, dst, len, bucket_off, bucket_ids, heap, S, c); return; }
  SK* A = reinterpret_cast<SK*>(qlds);                                   // [kSweepSort] the batch being sorted / served
  uint32_t* info = reinterpret_cast<uint32_t*>(A + kSweepSort);          // [kSweepPk] flits | exit position << 16
  uint64_t* pc = reinterpret_cast<uint64_t*>(info + kSweepPk);           // [kSweepPos + 1] start-run offsets
  uint32_t* ids = bucket_ids + b;
  SK* G = reinterpret_cast<SK*>(heap + b);                               // [n] start runs (HBM: the bucket's Ev scratch)
  SK* Bq = G + n;                                                        // [n] arrivals for the next position
  // 1. the chain's packet ids in index order (i = rank by index), then their info
  uint32_t M = 1;
  while (M < n) M <<= 1;
  uint32_t* ia = reinterpret_cast<uint32_t*>(A);
  for (uint32_t i = tid; i < M; i += blockDim.x) ia[i] = i < n ? ids[i] : 0xFFFFFFFFu;
  __syncthreads();
  block_bitonic(ia, M, [](uint32_t x, uint32_t y) { return x < y; });
  auto pos_of = [&](uint32_t tile) { return stage == 0 ? tile % P.w : tile / P.w; };
  auto tile_at = [&](uint32_t pos) -> uint32_t { return stage == 0 ? line * P.w + pos : pos * P.w + line; };
  for (uint32_t i = tid; i < n; i += blockDim.x) {
    const uint32_t k = ia[i];
    ids[i] = k;
    const uint64_t nf = nflits(P, len[k]);
    if (nf >= (1u << 16)) atomicOr(&s_bad, 1u);
    info[i] = (uint32_t)nf | (pos_of(dst[k]) << 16);
  }
  for (uint32_t p = tid; p <= npos; p += blockDim.x) pc[p] = 0;
  __syncthreads();
  if (s_bad) { chain_staged(D, stage, dst, len, bucket_off, bucket_ids, heap, S, c); return; }
  // 2. start runs: the packets bucketed by start position (counting sort into G)
  for (uint32_t i = tid; i < n; i += blockDim.x) atomicAdd((unsigned long long*)&pc[pos_of(S.cur[ids[i]]) + 1], 1ull);
  __syncthreads();
  if (tid == 0) for (uint32_t p = 0; p < npos; ++p) pc[p + 1] += pc[p];
  __syncthreads();
  for (uint32_t i = tid; i < n; i += blockDim.x) {
    const uint32_t k = ids[i];
    const uint64_t j = atomicAdd((unsigned long long*)&pc[pos_of(S.cur[k])], 1ull);   // pc[p] ends at run p's end
    G[j] = SK{S.t[k], i, 0};
  }
  __syncthreads();
  // run p = [p ? pc[p - 1] : 0, pc[p])
  const uint64_t zps = lat_to_ps((uint64_t)P.router_delay + P.link_delay, P.f);
  const int port = stage == 0 ? (dir ? P_RIGHT : P_LEFT) : (dir ? P_UP : P_DOWN);
  uint32_t nb = 0;                                                       // arrivals waiting in Bq
  if (prof) c_set = __builtin_amdgcn_s_memtime() - c_0;
  for (uint32_t s_ = 0; s_ < npos; ++s_) {
    const uint64_t c_a = prof ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t pos = dir ? s_ : npos - 1 - s_;
    const uint64_t r0 = pos ? pc[pos - 1] : 0, r1 = pc[pos];
    const uint32_t m = nb + (uint32_t)(r1 - r0);
    if (m == 0) continue;
    M = 1;
    while (M < m) M <<= 1;
    for (uint32_t i = tid; i < M; i += blockDim.x)
      A[i] = i < nb ? Bq[i] : i < m ? G[r0 + (i - nb)] : SK{~0ull, ~0u, 0};
    __syncthreads();
    block_bitonic(A, M, sk_lt);
    const uint64_t c_b = prof ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t tile = tile_at(pos);
    if (tid < 64) {
      // one wave serves the batch in order through the port's queue (registers)
      RegQueue rq;
      HQueue* q = D.q + (uint64_t)tile * 6 + port;
      HNode* nd = D.nd + ((uint64_t)tile * 6 + port) * P.max_size;
      if (P.qm) rq.load(q, nd, 1, P.analytical != 0, ln);
      uint64_t cq = 0, cf = 0;
      for (uint32_t j0 = 0; j0 < m; j0 += 64) {
        const uint32_t cnt = min(64u, m - j0);
        const uint64_t myt = ln < cnt ? A[j0 + ln].t : 0;
        const uint32_t myinfo = ln < cnt ? info[A[j0 + ln].i] : 0;
        uint64_t out = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
          const uint64_t t = rl64(myt, j);
          const uint32_t nf = (uint32_t)__builtin_amdgcn_readlane((int)myinfo, (int)j) & 0xFFFFu;
          const uint64_t qd = P.qm ? rq.request<true>(time_to_cycles(t, P.f), nf, D.err) : 0;
          cq += qd; cf += nf;
          if (ln == j) out = t + zps + lat_to_ps(qd, P.f);
        }
        if (ln < cnt) A[j0 + ln].t = out;
      }
      if (P.qm) rq.store(q, nd);
      if (ln == 0) {
        if (P.qm) { cadd(D.ctr, tile, GG_NC_ROUTER_CONTENTION_CYCLES, cq); cadd(D.ctr, tile, GG_NC_ROUTER_PACKETS, m); }
        cadd(D.ctr, tile, GG_NC_BUFFER_WRITES, cf); cadd(D.ctr, tile, GG_NC_BUFFER_READS, cf);
        cadd(D.ctr, tile, GG_NC_SWITCH_ALLOC, m); cadd(D.ctr, tile, GG_NC_CROSSBAR, cf);
        cadd(D.ctr, tile, GG_NC_LINK_TRAVERSALS, cf);
        s_na = 0;
      }
    }
    __syncthreads();
    const uint64_t c_c = prof ? __builtin_amdgcn_s_memtime() : 0;
    // the served batch: packets leaving the chain are written back, the rest arrive at the next position
    const uint32_t nx = dir ? pos + 1 : pos - 1;
    for (uint32_t j = tid; j < m; j += blockDim.x) {
      const SK x = A[j];
      if ((info[x.i] >> 16) == nx) {
        const uint32_t k = ids[x.i];
        const uint64_t t0 = S.t[k];
        const uint32_t a = pos_of(S.cur[k]);
        const uint64_t hz = (uint64_t)(dir ? nx - a : a - nx) * zps;   // zero-load part: router + link per hop
        S.zl[k] += hz;
        S.ct[k] += x.t - t0 - hz;
        S.t[k] = x.t;
        S.cur[k] = tile_at(nx);
      } else {
        Bq[atomicAdd(&s_na, 1u)] = x;
      }
    }
    __syncthreads();
    nb = s_na;
    if (prof) { c_sort += c_b - c_a; c_serve += c_c - c_b; c_part += __builtin_amdgcn_s_memtime() - c_c; nreq += m; }
  }
  if (prof && tid == 0) {
    atomicAdd(&prof[8 * stage + 0], (unsigned long long)c_set); atomicAdd(&prof[8 * stage + 1], (unsigned long long)c_sort);
    atomicAdd(&prof[8 * stage + 2], (unsigned long long)c_serve); atomicAdd(&prof[8 * stage + 3], (unsigned long long)c_part);
    atomicAdd(&prof[8 * stage + 4], (unsigned long long)nreq); atomicAdd(&prof[8 * stage + 5], 1ull);
    atomicMax(&prof[8 * stage + 6], (unsigned long long)(__builtin_amdgcn_s_memtime() - c_0));
  }
}
__global__ __launch_bounds__(kSweepThreads) void k_chain_sweep(NocDev D, int stage, const uint32_t* __restrict__ dst,
    const uint32_t* __restrict__ len, const uint64_t* __restrict__ bucket_off, uint32_t* __restrict__ bucket_ids,
    Ev* heap, PktState S, unsigned long long* prof)
{
  if (!GG_NOC_DIAG) prof = nullptr;
  chain_sweep(D, stage, dst, len, bucket_off, bucket_ids, heap, S, prof, blockIdx.x);
}

// ---------------------------------------------------------------------------
// Stages X / Y as a pipeline of time slabs (the default for chains of <=
// kPipePos positions): the positions of a chain serve concurrently, one wave
// per kPipeK positions.  Time is cut into slabs [T_{r-1}, T_r); at diagonal
// step d the position of travel index s serves its pending packets of slab
// r = d - s in (time, index) order.  That is the global event order at the
// port: a packet reaching position s before T_r left position s - 1 before
// T_r (a hop takes >= router + link delay >= 0), so position s - 1 served it
// in a slab <= r, at a step <= d - 1; and every packet still to come to s
// arrives at T_r or later.  Each position keeps its pending packets in an HBM
// pool (only its wave touches it) and receives the packets of the position
// before it through a two-parity incoming list (written at step d, taken at
// step d + 1); the slab's packets are sorted in the wave's LDS (bitonic) and
// served through the port's history tree held in the wave's registers
// (RegQueue) for the whole chain.  A slab part too large for the LDS batch
// is cut at a lower time bound (bisection) and served in parts: the order is
// unchanged.  Chains beyond the limits take the position sweep.
// ---------------------------------------------------------------------------
constexpr uint32_t kPipePos = 32, kPipeK = 2, kPipeWaves = kPipePos / kPipeK, kPipeBatch = 256, kPipePk = 6144;
constexpr size_t kPipeLds = (size_t)kPipeWaves * kPipeBatch * sizeof(SK) + (size_t)kPipePk * 4 + 3 * kPipePos * 4 + 64;
static_assert(kPipeLds <= kStageLdsMax, "pipeline LDS");

// one position of a pipelined chain, held by a wave across the slabs
struct PipePos {
  RegQueue rq;
  uint64_t cq, cf, m;       // contention cycles, flits, requests (wave-uniform)
};

__device__ __forceinline__ bool sk_below(const SK& x, uint64_t bt, uint32_t bi) { return x.t < bt || (x.t == bt && x.i < bi); }

__global__ __launch_bounds__(64 * kPipeWaves) void k_chain_pipe(NocDev D, int stage, const uint32_t* __restrict__ dst,
    const uint32_t* __restrict__ len, const uint64_t* __restrict__ bucket_off, uint32_t* __restrict__ bucket_ids,
    Ev* heap, PktState S, SK* pscr, uint64_t pstride, unsigned long long* prof)
{
  if (!GG_NOC_DIAG) prof = nullptr;
  extern __shared__ __attribute__((aligned(16))) uint8_t qlds[];
  const NocParams& P = D.P;
  const uint32_t c = blockIdx.x, line = c / 2, dir = c % 2, tid = threadIdx.x, ln = tid & 63, wv = tid >> 6;
  const uint64_t b = bucket_off[c], e = bucket_off[c + 1];
  if (b == e) return;
  const uint32_t npos = stage == 0 ? P.w : P.h;
  const bool regq = P.qtype == GG_QM_HISTORY_TREE && P.max_size <= kQMaxNoc;
  if (e - b > kPipePk || npos > kPipePos || (P.qm && !regq)) {
    chain_sweep(D, stage, dst, len, bucket_off, bucket_ids, heap, S, prof, c);
    return;
  }
  const uint32_t n = (uint32_t)(e - b);
  SK* A = reinterpret_cast<SK*>(qlds);                                         // [waves][kPipeBatch] slab batches
  uint32_t* info = reinterpret_cast<uint32_t*>(A + (size_t)kPipeWaves * kPipeBatch);   // [n] flits | exit position << 16
  uint32_t* npool = info + kPipePk;                                            // [npos] pool counts
  uint32_t* ninc = npool + kPipePos;                                           // [2][npos] incoming counts
  __shared__ uint32_t s_bad, s_left;
  __shared__ uint64_t s_tmin, s_tmax;
  uint32_t* ids = bucket_ids + b;
  // per position (travel index s) in HBM: pool [n], incoming [2][n]
  SK* base = pscr + (size_t)b * pstride;
  auto pool = [&](uint32_t s) { return base + (size_t)s * 3 * n; };
  auto inc = [&](uint32_t s, uint32_t par) { return base + (size_t)s * 3 * n + (size_t)(1 + par) * n; };
  auto pos_of = [&](uint32_t tile) { return stage == 0 ? tile % P.w : tile / P.w; };
  auto tile_at = [&](uint32_t pos) -> uint32_t { return stage == 0 ? line * P.w + pos : pos * P.w + line; };
  auto sidx = [&](uint32_t pos) { return dir ? pos : npos - 1 - pos; };        // travel index of a position
  auto pos_at = [&](uint32_t s) { return dir ? s : npos - 1 - s; };
  if (tid == 0) { s_bad = 0; s_left = n; s_tmin = ~0ull; s_tmax = 0; }
  for (uint32_t i = tid; i < kPipePos; i += blockDim.x) { npool[i] = 0; ninc[i] = 0; ninc[kPipePos + i] = 0; }
  __syncthreads();
  // 1. the chain's ids in index order (i = rank by index), info, start pools
  uint32_t M = 1;
  while (M < n) M <<= 1;
  uint32_t* ia = reinterpret_cast<uint32_t*>(A);                               // n <= kPipePk <= waves * batch * 4
  for (uint32_t i = tid; i < M; i += blockDim.x) ia[i] = i < n ? ids[i] : 0xFFFFFFFFu;
  __syncthreads();
  block_bitonic(ia, M, [](uint32_t x, uint32_t y) { return x < y; });
  for (uint32_t i = tid; i < n; i += blockDim.x) {
    const uint32_t k = ia[i];
    ids[i] = k;
    const uint64_t nf = nflits(P, len[k]);
    if (nf >= (1u << 16)) atomicOr(&s_bad, 1u);
    info[i] = (uint32_t)nf | (pos_of(dst[k]) << 16);
  }
  __syncthreads();
  if (s_bad) { chain_sweep(D, stage, dst, len, bucket_off, bucket_ids, heap, S, prof, c); return; }
  uint64_t tmn = ~0ull, tmx = 0;
  for (uint32_t i = tid; i < n; i += blockDim.x) {
    const uint32_t k = ids[i];
    const uint64_t t = S.t[k];
    const uint32_t s = sidx(pos_of(S.cur[k]));
    pool(s)[atomicAdd(&npool[s], 1u)] = SK{t, i, 0};
    tmn = t < tmn ? t : tmn; tmx = t > tmx ? t : tmx;
  }
  atomicMin((unsigned long long*)&s_tmin, (unsigned long long)tmn);
  atomicMax((unsigned long long*)&s_tmax, (unsigned long long)tmx);
  __syncthreads();
  // slab width: about 64 packets of the chain's start times per slab
  const uint64_t t0 = s_tmin;
  const uint64_t delta = max<uint64_t>(1, (s_tmax - s_tmin) / max<uint32_t>(1, n / 64) + 1);
  const uint64_t zps = lat_to_ps((uint64_t)P.router_delay + P.link_delay, P.f);
  const int port = stage == 0 ? (dir ? P_RIGHT : P_LEFT) : (dir ? P_UP : P_DOWN);
  // this wave's positions: travel indices wv + j * waves
  PipePos pp[kPipeK];
#pragma unroll
  for (uint32_t j = 0; j < kPipeK; ++j) {
    const uint32_t s = wv + j * kPipeWaves;
    pp[j].cq = 0; pp[j].cf = 0; pp[j].m = 0;
    if (s < npos && P.qm) {
      const uint32_t tile = tile_at(pos_at(s));
      pp[j].rq.load(D.q + (uint64_t)tile * 6 + port, D.nd + ((uint64_t)tile * 6 + port) * P.max_size, 1,
                    P.analytical != 0, ln);
    }
  }
  SK* mine = A + (size_t)wv * kPipeBatch;
  constexpr uint64_t kMaxSteps = 1ull << 24;
  for (uint64_t d = 0;; ++d) {
    const uint32_t par = (uint32_t)(d & 1);
#pragma unroll
    for (uint32_t j = 0; j < kPipeK; ++j) {
      const uint32_t s = wv + j * kPipeWaves;
      if (s >= npos || d < s) continue;
      const uint64_t r = d - s;
      const uint64_t Tr = (r + 1 >= (~0ull - t0) / delta) ? ~0ull : t0 + (r + 1) * delta;   // slab r = [.., Tr)
      // take the incoming packets of the last step into the pool
      SK* pl = pool(s);
      uint32_t np = npool[s];
      {
        const uint32_t q = par ^ 1u;                                           // the parity written at step d - 1
        uint32_t* cnt = &ninc[q * kPipePos + s];
        const uint32_t k_in = *cnt;
        const SK* src = inc(s, q);
        for (uint32_t i = ln; i < k_in; i += 64) pl[np + i] = src[i];
        np += k_in;
        nsync();
        if (ln == 0) *cnt = 0;
      }
      // serve every pending packet below (Tr, 0), in parts of <= kPipeBatch: a part ends at a
      // lower bound (time, index) found by bisection (on the time, then on the index)
      const uint32_t pos = pos_at(s), nx = dir ? pos + 1 : pos - 1;
      const uint32_t tile = tile_at(pos);
      (void)tile;
      for (;;) {
        auto count_below = [&](uint64_t bt, uint32_t bi) {
          uint32_t cm = 0;
          for (uint32_t i = ln; i < np; i += 64) cm += sk_below(pl[i], bt, bi);
          return (uint32_t)wave_sum64n(cm);
        };
        const uint32_t cntb = count_below(Tr, 0);
        if (cntb == 0) break;
        uint64_t bt = Tr;
        uint32_t bi = 0;
        if (cntb > kPipeBatch) {
          uint64_t lo = 0, hi = Tr;                                           // count(< lo) <= batch < count(< hi)
          while (hi - lo > 1) {
            const uint64_t mid = lo + (hi - lo) / 2;
            if (count_below(mid, 0) <= kPipeBatch) lo = mid; else hi = mid;
          }
          bt = lo;
          if (count_below(lo, 0) == 0) {                                      // > batch packets at time lo: by index
            uint32_t ilo = 0, ihi = n;                                        // count(< (lo, ilo)) <= batch < count(< (lo, ihi))
            while (ihi - ilo > 1) {
              const uint32_t mid = ilo + (ihi - ilo) / 2;
              if (count_below(lo, mid) <= kPipeBatch) ilo = mid; else ihi = mid;
            }
            bi = ilo;
          }
        }
        // split the pool: the part below bound to LDS, the rest compacted in place
        uint32_t m = 0, keep = 0;
        for (uint32_t i0 = 0; i0 < np; i0 += 64) {
          const uint32_t i = i0 + ln;
          SK x{~0ull, ~0u, 0};
          if (i < np) x = pl[i];
          const bool take = i < np && sk_below(x, bt, bi);
          const bool kp = i < np && !take;
          const uint64_t bt = __ballot(take), bk = __ballot(kp);
          const uint64_t below = (1ull << ln) - 1;
          if (take) mine[m + __builtin_popcountll(bt & below)] = x;
          nsync();
          if (kp) pl[keep + __builtin_popcountll(bk & below)] = x;
          m += (uint32_t)__builtin_popcountll(bt);
          keep += (uint32_t)__builtin_popcountll(bk);
        }
        np = keep;
        uint32_t Mb = 1;
        while (Mb < m) Mb <<= 1;
        for (uint32_t i = m + ln; i < Mb; i += 64) mine[i] = SK{~0ull, ~0u, 0};
        nsync();
        for (uint32_t kk = 2; kk <= Mb; kk <<= 1)
          for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
            for (uint32_t i = ln; i < Mb; i += 64) {
              const uint32_t l = i ^ jj;
              if (l > i) {
                const SK x = mine[i], y = mine[l];
                if (((i & kk) == 0) == sk_lt(y, x)) { mine[i] = y; mine[l] = x; }
              }
            }
            nsync();
          }
        // serve in order
        for (uint32_t j0 = 0; j0 < m; j0 += 64) {
          const uint32_t cnt = min(64u, m - j0);
          const bool ok = ln < cnt;
          const SK x = ok ? mine[j0 + ln] : SK{0, 0, 0};
          const uint32_t inf = ok ? info[x.i] : 0u;
          uint64_t out = 0;
          for (uint32_t jj = 0; jj < cnt; ++jj) {
            const uint64_t t = rl64(x.t, jj);
            const uint32_t nf = (uint32_t)__builtin_amdgcn_readlane((int)inf, (int)jj) & 0xFFFFu;
            uint64_t qd = 0;
            if (P.qm) qd = j == 0 ? pp[0].rq.request<true>(time_to_cycles(t, P.f), nf, D.err)
                                  : pp[kPipeK - 1].rq.request<true>(time_to_cycles(t, P.f), nf, D.err);
            if (j == 0) { pp[0].cq += qd; pp[0].cf += nf; } else { pp[kPipeK - 1].cq += qd; pp[kPipeK - 1].cf += nf; }
            if (ln == jj) out = t + zps + lat_to_ps(qd, P.f);
          }
          // hand the served packets on: leave the chain, or arrive at the next position
          if (ok) {
            if ((inf >> 16) == nx) {
              const uint32_t k = ids[x.i];
              const uint64_t ts = S.t[k];
              const uint32_t a = pos_of(S.cur[k]);
              const uint64_t hz = (uint64_t)(dir ? nx - a : a - nx) * zps;
              S.zl[k] += hz;
              S.ct[k] += out - ts - hz;
              S.t[k] = out;
              S.cur[k] = tile_at(nx);
              atomicSub(&s_left, 1u);
            } else {
              const uint32_t s2 = s + 1;
              inc(s2, par)[atomicAdd(&ninc[par * kPipePos + s2], 1u)] = SK{out, x.i, 0};
            }
          }
          nsync();
        }
        if (j == 0) pp[0].m += m; else pp[kPipeK - 1].m += m;
        if (bt == Tr && bi == 0) break;
      }
      if (ln == 0) npool[s] = np;
    }
    __syncthreads();
    if (s_left == 0) break;
    if (d + 1 >= kMaxSteps) { if (tid == 0) atomicOr(D.err, GG_DERR_STATE); break; }
  }
  // write the queues back, the counters once per position
#pragma unroll
  for (uint32_t j = 0; j < kPipeK; ++j) {
    const uint32_t s = wv + j * kPipeWaves;
    if (s >= npos) continue;
    const uint32_t tile = tile_at(pos_at(s));
    if (P.qm) pp[j].rq.store(D.q + (uint64_t)tile * 6 + port, D.nd + ((uint64_t)tile * 6 + port) * P.max_size);
    if (ln == 0 && pp[j].m) {
      const uint64_t m = pp[j].m, cf = pp[j].cf;
      if (P.qm) { cadd(D.ctr, tile, GG_NC_ROUTER_CONTENTION_CYCLES, pp[j].cq); cadd(D.ctr, tile, GG_NC_ROUTER_PACKETS, m); }
      cadd(D.ctr, tile, GG_NC_BUFFER_WRITES, cf); cadd(D.ctr, tile, GG_NC_BUFFER_READS, cf);
      cadd(D.ctr, tile, GG_NC_SWITCH_ALLOC, m); cadd(D.ctr, tile, GG_NC_CROSSBAR, cf);
      cadd(D.ctr, tile, GG_NC_LINK_TRAVERSALS, cf);
    }
  }
}

// ---------------------------------------------------------------------------
// Stages 0 / 3 (injection ports / SELF ports + receive), the default: one
// wave per tile (kPortWaves tiles per workgroup).  The tile's packets sorted
// by (time, packet index) in the wave's LDS (bitonic), served in order by the
// wave through the port's history tree held in its registers (RegQueue), the
// per-packet results and the tile's counters written by the lanes.  Tiles
// beyond kPortPk packets or with another queue model: the lane-serial walk
// (inject_tile / self_tile).
// ---------------------------------------------------------------------------
constexpr uint32_t kPortWaves = 4, kPortPk = 2048;
constexpr size_t kPortLds = (size_t)kPortWaves * kPortPk * sizeof(SK);

template <bool SELF>
__global__ __launch_bounds__(64 * kPortWaves) void k_port_sweep(NocDev D, const uint32_t* __restrict__ len,
    const uint64_t* __restrict__ bucket_off, const uint32_t* __restrict__ bucket_ids, Ev* heap, PktState S)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t qlds[];
  const NocParams& P = D.P;
  const uint32_t ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t tile = blockIdx.x * kPortWaves + wv;
  if (tile >= P.tiles) return;
  const uint64_t b = bucket_off[tile], e = bucket_off[tile + 1];
  if (b == e) return;
  const uint32_t n = (uint32_t)min<uint64_t>(e - b, 0xFFFFFFFFull);
  const bool regq = P.qtype == GG_QM_HISTORY_TREE && P.max_size <= kQMaxNoc;
  if (n > kPortPk || (P.qm && !regq)) {
    if (ln == 0) {
      if (SELF) self_tile(D, tile, len, bucket_off, bucket_ids, heap, S);
      else inject_tile(D, tile, len, bucket_off, bucket_ids, heap, S);
    }
    return;
  }
  SK* A = reinterpret_cast<SK*>(qlds) + (size_t)wv * kPortPk;
  uint32_t M = 1;
  while (M < n) M <<= 1;
  // (time, packet index) keys; i = the packet id itself (unique)
  for (uint32_t i = ln; i < M; i += 64) {
    if (i < n) { const uint32_t k = bucket_ids[b + i]; A[i] = SK{S.t[k], k, 0}; }
    else A[i] = SK{~0ull, ~0u, 0};
  }
  nsync();
  for (uint32_t kk = 2; kk <= M; kk <<= 1)
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      for (uint32_t i = ln; i < M; i += 64) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const SK x = A[i], y = A[l];
          if (((i & kk) == 0) == sk_lt(y, x)) { A[i] = y; A[l] = x; }
        }
      }
      nsync();
    }
  const int port = SELF ? P_SELF : 5;
  HQueue* q = D.q + (uint64_t)tile * 6 + port;
  HNode* nd = D.nd + ((uint64_t)tile * 6 + port) * P.max_size;
  RegQueue rq;
  if (P.qm) rq.load(q, nd, 1, P.analytical != 0, ln);
  const uint64_t zps = lat_to_ps((uint64_t)P.router_delay + P.link_delay, P.f);
  uint64_t cq = 0;                                         // uniform: contention cycles of the port
  uint64_t sf = 0, sb = 0, sl = 0, sc = 0;                  // this lane's packets: flits, bits, latency, contention
  for (uint32_t j0 = 0; j0 < n; j0 += 64) {
    const uint32_t cnt = min(64u, n - j0);
    const bool mine = ln < cnt;
    const uint32_t k = mine ? A[j0 + ln].i : 0u;
    const uint32_t bits = mine ? len[k] : 0u;
    const uint64_t myt = mine ? A[j0 + ln].t : 0;
    const uint32_t mynf = mine ? (uint32_t)nflits(P, bits) : 0u;
    uint64_t qmine = 0;
    for (uint32_t j = 0; j < cnt; ++j) {
      const uint64_t t = rl64(myt, j);
      const uint32_t nf = (uint32_t)__builtin_amdgcn_readlane((int)mynf, (int)j);
      const uint64_t qd = P.qm ? rq.request<true>(time_to_cycles(t, P.f), nf, D.err) : 0;
      cq += qd;
      if (ln == j) qmine = qd;
    }
    if (mine) {
      const uint64_t cps = lat_to_ps(qmine, P.f);
      if (!SELF) {                                          // injection router: delay 0 + queue delay
        S.t[k] = myt + lat_to_ps(0, P.f) + cps;
        S.ct[k] += cps;
        sf += mynf; sb += bits;
      } else {                                              // SELF hop + serialization + receive
        const uint64_t ser = lat_to_ps(mynf, P.f);
        const uint64_t t2 = myt + zps + cps + ser, z2 = S.zl[k] + zps + ser, c2 = S.ct[k] + cps;
        S.t[k] = t2; S.zl[k] = z2; S.ct[k] = c2;
        sf += mynf; sb += bits; sl += z2 + c2; sc += c2;
      }
    }
  }
  if (P.qm) rq.store(q, nd);
  sf = wave_sum64n(sf); sb = wave_sum64n(sb); sl = wave_sum64n(sl); sc = wave_sum64n(sc);
  if (ln == 0) {
    if (!SELF) {
      cadd(D.ctr, tile, GG_NC_PACKETS_SENT, n); cadd(D.ctr, tile, GG_NC_FLITS_SENT, sf); cadd(D.ctr, tile, GG_NC_BITS_SENT, sb);
    } else {
      if (P.qm) { cadd(D.ctr, tile, GG_NC_ROUTER_CONTENTION_CYCLES, cq); cadd(D.ctr, tile, GG_NC_ROUTER_PACKETS, n); }
      cadd(D.ctr, tile, GG_NC_BUFFER_WRITES, sf); cadd(D.ctr, tile, GG_NC_BUFFER_READS, sf);
      cadd(D.ctr, tile, GG_NC_SWITCH_ALLOC, n); cadd(D.ctr, tile, GG_NC_CROSSBAR, sf);
      cadd(D.ctr, tile, GG_NC_LINK_TRAVERSALS, sf);
      cadd(D.ctr, tile, GG_NC_PACKETS_RECEIVED, n); cadd(D.ctr, tile, GG_NC_FLITS_RECEIVED, sf);
      cadd(D.ctr, tile, GG_NC_BITS_RECEIVED, sb);
      cadd(D.ctr, tile, GG_NC_TOTAL_LATENCY_PS, sl); cadd(D.ctr, tile, GG_NC_TOTAL_CONTENTION_PS, sc);
    }
  }
}

// bucket keys: 0 = injection (src tile), 1 = X chain, 2 = Y chain, 3 = SELF (dst tile); ~0 = not in stage
__device__ __forceinline__ uint64_t batch_n(uint64_t n, const uint32_t* n_dev) { return n_dev ? min((uint64_t)*n_dev, n) : n; }

__global__ void k_keys(NocParams P, int stage, const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                       uint64_t cap, const uint32_t* n_dev, uint32_t* keys, uint32_t* counts, uint32_t* err)
{
  const uint64_t n = batch_n(cap, n_dev);
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t s = src[k], d = dst[k];
  if (s >= P.tiles || d >= P.tiles) { atomicOr(err, GG_DERR_RANGE); keys[k] = ~0u; return; }
  uint32_t key = ~0u;
  if (s != d) {
    if (stage == 0) key = s;
    else if (stage == 1) key = xchain_of(P, s, d);
    else if (stage == 2) key = ychain_of(P, s, d);
    else key = d;
  }
  keys[k] = key;
  if (key != ~0u) atomicAdd(&counts[key], 1u);
}

__global__ void k_scan_counts(const uint32_t* counts, uint32_t nb, uint64_t* off, uint32_t* cursor)
{
  // single block; nb is small (<= 2 * 4096)
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x, per = (nb + blockDim.x - 1) / blockDim.x;
  uint64_t s = 0;
  for (uint32_t i = t * per; i < min(nb, (t + 1) * per); ++i) s += counts[i];
  part[t] = s;
  __syncthreads();
  if (t == 0) { uint64_t a = 0; for (uint32_t i = 0; i < blockDim.x; ++i) { uint64_t v = part[i]; part[i] = a; a += v; } off[nb] = a; }
  __syncthreads();
  uint64_t a = part[t];
  for (uint32_t i = t * per; i < min(nb, (t + 1) * per); ++i) { off[i] = a; cursor[i] = 0; a += counts[i]; }
}

__global__ void k_bucket(const uint32_t* __restrict__ keys, uint64_t cap, const uint32_t* n_dev,
                         const uint64_t* __restrict__ off, uint32_t* cursor, uint32_t* ids)
{
  const uint64_t n = batch_n(cap, n_dev);
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t key = keys[k];
  if (key == ~0u) return;
  ids[off[key] + atomicAdd(&cursor[key], 1u)] = (uint32_t)k;
}

__global__ void k_init_pkts(const uint32_t* __restrict__ src, const uint64_t* __restrict__ t0, uint64_t cap,
                            const uint32_t* n_dev, PktState S)
{
  const uint64_t n = batch_n(cap, n_dev);
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  S.t[k] = t0[k]; S.zl[k] = 0; S.ct[k] = 0; S.cur[k] = src[k];
}

__global__ void k_htree_reset(HQueue* q, HNode* nd, uint64_t nq, uint32_t max_size, uint32_t type, uint32_t aux)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  hq_init(q + i, nd + i * max_size, max_size, type, aux);
}

// processing times of 0 are outside the reference's call sites (flits >= 1,
// DRAM 13) and outside the interval argument of gg_dev.h: rejected
// One wave: the queue image in LDS and every request on the whole wave
// (HTree::delay_w, the path of the coherent walkers); one lane on the HBM
// image beyond 128 slots.
__global__ void __launch_bounds__(64) k_htree_seq(HQueue* q, HNode* nd, uint64_t min_proc, uint32_t analytical,
                                                  const uint64_t* t, const uint64_t* p, uint64_t n, uint64_t* d,
                                                  uint32_t* err)
{
  __shared__ __attribute__((aligned(16))) uint8_t img[sizeof(HQueue) + 128 * sizeof(HNode)];
  const uint32_t ln = threadIdx.x, ms = q->max_size;
  if (ms > 128) {
    if (ln != 0) return;
    HTree tr{q, nd, min_proc, analytical != 0};
    for (uint64_t i = 0; i < n; ++i) {
      if (p[i] == 0) { atomicOr(err, GG_DERR_RANGE); d[i] = 0; continue; }
      d[i] = tr.delay(t[i], p[i], err);
    }
    return;
  }
  HQueue* lq = reinterpret_cast<HQueue*>(img);
  HNode* lnd = reinterpret_cast<HNode*>(img + sizeof(HQueue));
  for (uint32_t w = ln; w < sizeof(HQueue) / 16 + ms; w += 64)
    reinterpret_cast<uint4*>(img)[w] = w < sizeof(HQueue) / 16 ? reinterpret_cast<const uint4*>(q)[w]
                                                              : reinterpret_cast<const uint4*>(nd)[w - sizeof(HQueue) / 16];
  __syncthreads();
  HTree tr{lq, lnd, min_proc, analytical != 0};
  // a history tree lives in the wave's registers for the whole stream (RegQueue)
  const bool reg = lq->type == GG_QM_HISTORY_TREE;
  RegQueue rq;
  if (reg) rq.load(lq, lnd, min_proc, analytical != 0, ln);
  __shared__ uint64_t ct[512], cp[512], cd[512];          // requests staged 512 at a time
  for (uint64_t b = 0; b < n; b += 512) {
    const uint32_t m = (uint32_t)min<uint64_t>(512, n - b);
    for (uint32_t k = ln; k < m; k += 64) { ct[k] = t[b + k]; cp[k] = p[b + k]; }
    __syncthreads();
    for (uint32_t k = 0; k < m; ++k) {
      const uint64_t ti = ct[k], pi = cp[k];
      uint64_t r = 0;
      if (pi == 0) { if (ln == 0) atomicOr(err, GG_DERR_RANGE); }
      else r = reg ? rq.request(ti, pi, err) : tr.delay_w(ti, pi, err, ln);
      cd[k] = r;
    }
    __syncthreads();
    for (uint32_t k = ln; k < m; k += 64) d[b + k] = cd[k];
    __syncthreads();
  }
  if (reg) rq.store(lq, lnd);
  for (uint32_t w = ln; w < sizeof(HQueue) / 16 + ms; w += 64) {
    const uint4 v = reinterpret_cast<const uint4*>(img)[w];
    if (w < sizeof(HQueue) / 16) reinterpret_cast<uint4*>(q)[w] = v;
    else reinterpret_cast<uint4*>(nd)[w - sizeof(HQueue) / 16] = v;
  }
}

__global__ void k_analytical(const HQueue* q, uint32_t tiles, uint64_t* ctr)
{
  const uint32_t tile = blockIdx.x * blockDim.x + threadIdx.x;
  if (tile >= tiles) return;
  uint64_t a = 0;
  for (int p = 0; p < NPORTS; ++p) a += q[(uint64_t)tile * 6 + p].analytical;
  ctr[(uint64_t)tile * GG_NUM_NET_COUNTERS + GG_NC_ANALYTICAL_REQUESTS] = a;
  for (int p = 0; p < NPORTS; ++p) {
    ctr[(uint64_t)tile * GG_NUM_NET_COUNTERS + GG_NC_PORT_UTILIZED_CYCLES + p] = q[(uint64_t)tile * 6 + p].util;
    ctr[(uint64_t)tile * GG_NUM_NET_COUNTERS + GG_NC_PORT_LAST_CYCLES + p] = q[(uint64_t)tile * 6 + p].last_req;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// Broadcast tree (gg_noc_route_tree): NetworkModelEMeshHopByHop::routePacket's
// broadcast branch (network_model_emesh_hop_by_hop.cc:163-221).  A broadcast
// event at router c asks all its listed output-port queues at one time and
// forwards every copy with the max delay (RouterModel::processPacket over a
// port list, router_model.cc:71-108), so the row (X) and column (Y) port
// chains are no longer independent stages: the walk is one global
// (time, packet index) event order — injection events (SEND_TILE, :151-159)
// and router events in one heap, an event being the packet, its router and
// its time (zero-load = XY distance from the sender + 1 hops x router+link
// delay, every tree path being a shortest path; contention = the rest).  One
// lane walks; the heap lives in LDS when its bound (packets + broadcasts x
// tiles) fits, else in HBM.
// ---------------------------------------------------------------------------
struct TEv { uint64_t t; uint32_t id, at; };   // at: router tile, | kInjBit = injection port of src
constexpr uint32_t kTreeLdsEv = 160 * 1024 / sizeof(TEv);
constexpr uint32_t kInjBit = 0x80000000u;
__device__ __forceinline__ bool tev_lt(const TEv& a, const TEv& b) { return a.t < b.t || (a.t == b.t && a.id < b.id); }
__device__ __forceinline__ void theap_push(TEv* h, uint64_t& n, const TEv& e)
{
  uint64_t i = n++;
  while (i > 0) { uint64_t p = (i - 1) / 2; if (!tev_lt(e, h[p])) break; h[i] = h[p]; i = p; }
  h[i] = e;
}
__device__ __forceinline__ TEv theap_pop(TEv* h, uint64_t& n)
{
  TEv top = h[0], last = h[--n];
  uint64_t i = 0;
  for (;;) {
    uint64_t l = 2 * i + 1, r = l + 1, m = i;
    TEv cand = last;
    if (l < n && tev_lt(h[l], cand)) { m = l; cand = h[l]; }
    if (r < n && tev_lt(h[r], cand)) m = r;
    if (m == i) break;
    h[i] = h[m]; i = m;
  }
  if (n) h[i] = last;
  return top;
}

// GG_TREE_DBG (diagnostic builds only, results not valid): 1 = no counter
// atomics, 2 = no queue requests in the tree walk
#ifndef GG_TREE_DBG
#define GG_TREE_DBG 0
#endif
__device__ __forceinline__ void tcadd(uint64_t* c, uint32_t tile, int k, uint64_t v)
{
  if (!(GG_TREE_DBG & 1)) cadd(c, tile, k, v);
}
// a router's event counters, summed in registers over its events and added
// to HBM once (the windowed walk: one thread owns a router)
constexpr uint32_t kNetCtrTree = 15;   // TreeAcc's fields: rcc rpk buf sw xb[5] link prcv frcv brcv lat con
struct TreeAcc {
  uint64_t rcc = 0, rpk = 0, buf = 0, sw = 0, xb[5] = {0, 0, 0, 0, 0}, link = 0, prcv = 0, frcv = 0, brcv = 0, lat = 0, con = 0;
  __device__ __forceinline__ void crossbar(int np, uint64_t nf)
  {
    // constant indices only (a dynamically indexed private array would go to scratch)
    if (np == 1) xb[0] += nf; else if (np == 2) xb[1] += nf; else if (np == 3) xb[2] += nf;
    else if (np == 4) xb[3] += nf; else xb[4] += nf;
  }
  __device__ __forceinline__ void flush(uint64_t* c, uint32_t tile)
  {
    tcadd(c, tile, GG_NC_ROUTER_CONTENTION_CYCLES, rcc); tcadd(c, tile, GG_NC_ROUTER_PACKETS, rpk);
    tcadd(c, tile, GG_NC_BUFFER_WRITES, buf); tcadd(c, tile, GG_NC_BUFFER_READS, buf);
    tcadd(c, tile, GG_NC_SWITCH_ALLOC, sw); tcadd(c, tile, GG_NC_CROSSBAR, xb[0]);
    tcadd(c, tile, GG_NC_CROSSBAR_MULTI + 0, xb[1]); tcadd(c, tile, GG_NC_CROSSBAR_MULTI + 1, xb[2]);
    tcadd(c, tile, GG_NC_CROSSBAR_MULTI + 2, xb[3]); tcadd(c, tile, GG_NC_CROSSBAR_MULTI + 3, xb[4]);
    tcadd(c, tile, GG_NC_LINK_TRAVERSALS, link); tcadd(c, tile, GG_NC_PACKETS_RECEIVED, prcv);
    tcadd(c, tile, GG_NC_FLITS_RECEIVED, frcv); tcadd(c, tile, GG_NC_BITS_RECEIVED, brcv);
    tcadd(c, tile, GG_NC_TOTAL_LATENCY_PS, lat); tcadd(c, tile, GG_NC_TOTAL_CONTENTION_PS, con);
    *this = TreeAcc();
  }
};
struct TreeIO {
  const uint32_t* src; const uint32_t* dst; const uint32_t* len; const uint64_t* t0;
  uint32_t* bidx; gg_packet_out out, bout;
};

// SEND_TILE: the injection router (delay 0, port 0) -> the router event at the source
__device__ __forceinline__ TEv tree_inject(const NocDev& D, const TreeIO& IO, const TEv& e)
{
  const NocParams& P = D.P;
  const uint32_t k = e.id, s = IO.src[k], bits = IO.len[k];
  const uint64_t nf = nflits(P, bits);
  tcadd(D.ctr, s, GG_NC_PACKETS_SENT, 1); tcadd(D.ctr, s, GG_NC_FLITS_SENT, nf); tcadd(D.ctr, s, GG_NC_BITS_SENT, bits);
  if (IO.dst[k] == GG_BROADCAST) {                 // updateSendCounters (network_model.cc:244-250)
    tcadd(D.ctr, s, GG_NC_PACKETS_BROADCASTED, 1); tcadd(D.ctr, s, GG_NC_FLITS_BROADCASTED, nf);
    tcadd(D.ctr, s, GG_NC_BITS_BROADCASTED, bits);
  }
  uint64_t qd = 0;
  if (P.qm && !(GG_TREE_DBG & 2)) { HTree tr = D.tree(s, 5); qd = tr.delay(time_to_cycles(e.t, P.f), nf, D.err); }
  return TEv{e.t + lat_to_ps(0, P.f) + lat_to_ps(qd, P.f), k, s};
}

// EMESH: one router event (unicast XY or broadcast fork); forwarded copies go to push(TEv)
template <class Push>
__device__ __forceinline__ void tree_router(const NocDev& D, const TreeIO& IO, const TEv& e, Push push, TreeAcc& A)
{
  const NocParams& P = D.P;
  const uint32_t W = P.w, H = P.h;
  const uint32_t k = e.id, s = IO.src[k], d = IO.dst[k], bits = IO.len[k];
  const uint64_t nf = nflits(P, bits);
  const uint32_t c = e.at, cx = c % W, cy = c / W, sx = s % W, sy = s / W;
  int ports[5]; uint32_t nxt[5]; int np = 0;
  if (d != GG_BROADCAST) {                         // XY (:223-256)
    const uint32_t dx = d % W, dy = d / W;
    if (cx > dx)      { ports[0] = P_LEFT;  nxt[0] = c - 1; }
    else if (cx < dx) { ports[0] = P_RIGHT; nxt[0] = c + 1; }
    else if (cy > dy) { ports[0] = P_DOWN;  nxt[0] = c - W; }
    else if (cy < dy) { ports[0] = P_UP;    nxt[0] = c + W; }
    else              { ports[0] = P_SELF;  nxt[0] = c; }
    np = 1;
  } else {                                         // broadcast tree (:163-221), next_dest_list order
    if (cy >= sy && cy + 1 < H) { ports[np] = P_UP;   nxt[np++] = c + W; }
    if (cy <= sy && cy >= 1)    { ports[np] = P_DOWN; nxt[np++] = c - W; }
    if (cy == sy) {
      if (cx >= sx && cx + 1 < W) { ports[np] = P_RIGHT; nxt[np++] = c + 1; }
      if (cx <= sx && cx >= 1)    { ports[np] = P_LEFT;  nxt[np++] = c - 1; }
    }
    ports[np] = P_SELF; nxt[np++] = c;
  }
  uint64_t qd = 0;
  if (P.qm && !(GG_TREE_DBG & 2)) {
    for (int i = 0; i < np; ++i) {
      HTree tr = D.tree(c, ports[i]);
      qd = max(qd, tr.delay(time_to_cycles(e.t, P.f), nf, D.err));
    }
    A.rcc += qd * (uint64_t)np;                    // updateContentionCounters, per listed port
    A.rpk += (uint64_t)np;
  }
  A.buf += nf; A.sw += 1; A.crossbar(np, nf);
  A.link += nf * (uint64_t)np;
  const uint64_t zps = lat_to_ps((uint64_t)P.router_delay + P.link_delay, P.f), cps = lat_to_ps(qd, P.f);
  const uint64_t hops = (uint64_t)((cx > sx ? cx - sx : sx - cx) + (cy > sy ? cy - sy : sy - cy)) + 1;
  const uint64_t t = e.t + zps + cps, zl = hops * zps, ct = t - IO.t0[k] - zl;
  for (int i = 0; i < np; ++i) {
    if (ports[i] != P_SELF) { push(TEv{t, k, nxt[i]}); continue; }
    const uint64_t ser = lat_to_ps(nf, P.f);       // receive at c (network_model.cc:118-150,253-272)
    A.prcv += 1; A.frcv += nf; A.brcv += bits;
    A.lat += zl + ser + ct; A.con += ct;
    if (d == GG_BROADCAST) {
      const uint64_t o = (uint64_t)IO.bidx[k] * P.tiles + c;
      IO.bout.arrival_ps_dev[o] = t + ser; IO.bout.zero_load_ps_dev[o] = zl + ser; IO.bout.contention_ps_dev[o] = ct;
    } else {
      IO.out.arrival_ps_dev[k] = t + ser; IO.out.zero_load_ps_dev[k] = zl + ser; IO.out.contention_ps_dev[k] = ct;
    }
  }
}

// The serial form: one lane, one heap (zero router + link delay, where the
// windowed form below has no lookahead, or meshes beyond kTreeMaxT).
template <bool LDS>
__global__ __launch_bounds__(64) void k_tree_walk(NocDev D, TreeIO IO, uint64_t n, uint64_t nb, TEv* gheap, uint64_t hcap)
{
  extern __shared__ __align__(16) uint8_t tree_lds[];
  TEv* heap = LDS ? reinterpret_cast<TEv*>(tree_lds) : gheap;
  if (threadIdx.x != 0) return;
  const NocParams& P = D.P;
  // validate, number the broadcasts in batch order, seed the injection events
  uint64_t m = 0, hn = 0;
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t s = IO.src[k], d = IO.dst[k];
    if (s >= P.tiles || (d >= P.tiles && d != GG_BROADCAST)) { atomicOr(D.err, GG_DERR_RANGE); return; }
    IO.bidx[k] = d == GG_BROADCAST ? (uint32_t)m++ : ~0u;
  }
  if (m != nb || n + nb * P.tiles > hcap) { atomicOr(D.err, GG_DERR_CAP); return; }
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t s = IO.src[k], d = IO.dst[k];
    if (s == d) { IO.out.arrival_ps_dev[k] = IO.t0[k]; IO.out.zero_load_ps_dev[k] = 0; IO.out.contention_ps_dev[k] = 0; continue; }
    theap_push(heap, hn, TEv{IO.t0[k], (uint32_t)k, s | kInjBit});
  }
  while (hn) {
    const TEv e = theap_pop(heap, hn);
    if (e.at & kInjBit) { theap_push(heap, hn, tree_inject(D, IO, e)); continue; }
    TreeAcc A;
    tree_router(D, IO, e, [&](const TEv& x) { theap_push(heap, hn, x); }, A);
    A.flush(D.ctr, e.at);
  }
}

constexpr uint32_t kTreeMaxT = 4096;                  // the windowed walk's per-router LDS arrays
// exclusive block-wide scan of one value per thread (DPP-free shuffles within
// the wave, the wave totals through LDS); *total = the block sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total)
{
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  uint32_t x = v;
  #pragma unroll
  for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(x, o, 64); if (lane >= (uint32_t)o) x += y; }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) { uint32_t a = 0; for (uint32_t i = 0; i < nw; ++i) { const uint32_t t = wsum[i]; wsum[i] = a; a += t; } wsum[nw] = a; }
  __syncthreads();
  const uint32_t r = wsum[wid] + x - v;
  *total = wsum[nw];
  __syncthreads();
  return r;
}
// ---------------------------------------------------------------------------
// The windowed walk (k_tree_pool, one workgroup): a router event at time t
// forwards its copies at t + router + link delay (zps > 0) or later, so in a
// window [t_min, t_min + zps) every router's events depend only on that
// router's own queues: the routers serve their window events in (time, index)
// order in parallel.  The per-window work is kept off HBM:
// * injection ports are served once at the start; each tile's router events
//   are a (time, index)-sorted run in HBM whose head time sits in LDS, so a
//   window takes the due heads instead of rescanning every pending injection;
// * the pending forwarded copies live in an LDS pool (two buffers, one per
//   window parity), continued in HBM beyond its capacity;
// * the window's due events are LDS records holding their packet's fields,
//   linked per router and sorted there by (time, index);
// * a router's listed output ports are separate queues whose requests come in
//   the router's event order, so every (router, port) with requests is a task
//   of its own and an event's delay is the max over its ports (an LDS atomic
//   max): the memory round trips of one event's ports overlap.
// Beyond the LDS capacities the due records and the pool continue in HBM, so
// results never depend on them (only the speed).
constexpr uint32_t kTpThreads = 1024;
constexpr uint32_t kTpNil = 0xFFFFFFFFu;
constexpr size_t kTpLds = 160 * 1024 - 256;
struct TGe {                                     // a due router event of the window
  uint64_t t, t0, q;                             // time at the router, injection time, max port delay (cycles)
  uint32_t k, at, src, dst, len, bidx, next, mask;   // next: the router's list; mask: listed ports (1 << P_*)
};
__device__ __forceinline__ uint64_t tp_wave_min64(uint64_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const uint64_t u = (uint64_t)__shfl_xor((long long)v, o); v = u < v ? u : v; }
  return v;
}
// listed output ports of packet (s, d) at router c (hop_by_hop.cc:163-256)
__device__ __forceinline__ uint32_t tree_ports(const NocParams& P, uint32_t c, uint32_t s, uint32_t d)
{
  const uint32_t W = P.w, H = P.h, cx = c % W, cy = c / W, sx = s % W, sy = s / W;
  if (d != GG_BROADCAST) {
    const uint32_t dx = d % W, dy = d / W;
    return 1u << (cx > dx ? P_LEFT : cx < dx ? P_RIGHT : cy > dy ? P_DOWN : cy < dy ? P_UP : P_SELF);
  }
  uint32_t m = 1u << P_SELF;
  if (cy >= sy && cy + 1 < H) m |= 1u << P_UP;
  if (cy <= sy && cy >= 1) m |= 1u << P_DOWN;
  if (cy == sy) {
    if (cx >= sx && cx + 1 < W) m |= 1u << P_RIGHT;
    if (cx <= sx && cx >= 1) m |= 1u << P_LEFT;
  }
  return m;
}
__device__ __forceinline__ uint32_t tree_next(const NocParams& P, uint32_t c, int port)
{
  return port == P_LEFT ? c - 1 : port == P_RIGHT ? c + 1 : port == P_DOWN ? c - P.w : port == P_UP ? c + P.w : c;
}
struct TpBufs {
  TEv* run;        // [n] the tiles' injection router events, (time, index)-sorted per tile
  TEv* heap;       // [n] setup scratch
  TEv* hp[2];      // [hcap] the pool buffers beyond their LDS part
  TGe* gh;         // [hcap] due records beyond their LDS part
};
// LDS bytes of k_tree_pool for T tiles, gcap due records and ecap pool events per buffer
__host__ __device__ inline size_t tp_lds_bytes(uint32_t T, uint32_t gcap, uint32_t ecap)
{
  return 8ull * T + 2ull * ecap * sizeof(TEv) + (size_t)gcap * sizeof(TGe) + 4ull * (T + 1) + 12ull * T + T;
}

__global__ __launch_bounds__(kTpThreads) void k_tree_pool(NocDev D, TreeIO IO, uint64_t n, uint64_t nb, TpBufs B,
                                                         uint64_t hcap, uint32_t gcap, uint32_t ecap,
                                                         unsigned long long* prof)
{
  if (!GG_NOC_DIAG) prof = nullptr;
  extern __shared__ __align__(16) uint8_t tp_lds[];
  __shared__ uint32_t wsum[kTpThreads / 64 + 1];
  __shared__ unsigned long long s_tmin, s_pmin, s_pmin1;
  __shared__ uint32_t s_n0, s_n1, s_nd, s_na, s_err;
  const NocParams& P = D.P;
  const uint32_t T = P.tiles, tid = threadIdx.x, nt = blockDim.x, ln = tid & 63;
  const uint64_t zps = lat_to_ps((uint64_t)P.router_delay + P.link_delay, P.f);
  uint64_t* hd = reinterpret_cast<uint64_t*>(tp_lds);                   // [T] head time of each tile's injection run
  TEv* El[2] = {reinterpret_cast<TEv*>(hd + T), reinterpret_cast<TEv*>(hd + T) + ecap};
  TGe* Gl = reinterpret_cast<TGe*>(El[1] + ecap);                       // [gcap]
  uint32_t* off = reinterpret_cast<uint32_t*>(Gl + gcap);               // [T + 1] run offsets
  uint32_t* cur = off + T + 1;                                          // [T] run cursors
  uint32_t* head = cur + T;                                             // [T] the router's due list
  uint32_t* act = head + T;                                             // [na] routers with due events
  uint8_t* um = reinterpret_cast<uint8_t*>(act + T);                    // [na] union of their events' ports
  // the due records and the pool buffers: LDS part, then HBM
  auto with_g = [&](uint32_t i, auto f) { if (i < gcap) f(Gl[i]); else f(B.gh[i - gcap]); };
  auto with_e = [&](uint32_t b, uint32_t i, auto f) { if (i < ecap) f(El[b][i]); else f(B.hp[b][i - ecap]); };
  unsigned long long pc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pw = 0, pn = 0, pt = __builtin_amdgcn_s_memtime();
  auto lap = [&](int i) { if (prof) { const unsigned long long x = __builtin_amdgcn_s_memtime(); pc[i] += x - pt; pt = x; } };

  // 1. validate; broadcast ordinals; the packets bucketed by source
  if (tid == 0) { s_err = 0; s_n0 = 0; s_pmin = ~0ull; }
  for (uint32_t i = tid; i < T; i += nt) { cur[i] = 0; head[i] = kTpNil; }
  __syncthreads();
  const uint64_t per = (n + nt - 1) / nt, k0 = min(n, tid * per), k1 = min(n, k0 + per);
  uint32_t mine = 0;
  for (uint64_t k = k0; k < k1; ++k) {
    const uint32_t s = IO.src[k], d = IO.dst[k];
    if (s >= T || (d >= T && d != GG_BROADCAST)) atomicOr(&s_err, GG_DERR_RANGE);
    mine += d == GG_BROADCAST;
    if (s < T && s != d) atomicAdd(&cur[s], 1u);
  }
  uint32_t nbc;
  mine = block_excl_scan(mine, wsum, &nbc);
  if (tid == 0 && (nbc != nb || n + nb * T > hcap)) s_err |= GG_DERR_CAP;
  __syncthreads();
  if (s_err) { if (tid == 0) atomicOr(D.err, s_err); return; }
  for (uint64_t k = k0; k < k1; ++k) IO.bidx[k] = IO.dst[k] == GG_BROADCAST ? mine++ : ~0u;
  {
    const uint32_t pt_ = (T + nt - 1) / nt;
    uint32_t a = 0, tot;
    for (uint32_t i = tid * pt_; i < min(T, (tid + 1) * pt_); ++i) a += cur[i];
    a = block_excl_scan(a, wsum, &tot);
    for (uint32_t i = tid * pt_; i < min(T, (tid + 1) * pt_); ++i) { off[i] = a; a += cur[i]; cur[i] = 0; }
    if (tid == 0) off[T] = tot;
    __syncthreads();
  }
  for (uint64_t k = k0; k < k1; ++k) {
    const uint32_t s = IO.src[k], d = IO.dst[k];
    if (s == d) { IO.out.arrival_ps_dev[k] = IO.t0[k]; IO.out.zero_load_ps_dev[k] = 0; IO.out.contention_ps_dev[k] = 0; continue; }
    B.heap[off[s] + atomicAdd(&cur[s], 1u)] = TEv{IO.t0[k], (uint32_t)k, s | kInjBit};
  }
  __syncthreads();
  // 2. injection ports: each tile's packets in (time, index) order; the router
  //    events they produce re-sorted into the tile's run
  for (uint32_t r = tid; r < T; r += nt) {
    TEv* h = B.heap + off[r];
    TEv* h2 = B.run + off[r];
    const uint64_t m = off[r + 1] - off[r];
    uint64_t hn = 0, hn2 = 0;
    for (uint64_t i = 0; i < m; ++i) { const TEv e = h[i]; theap_push(h, hn, e); }
    while (hn) { const TEv e = theap_pop(h, hn); theap_push(h2, hn2, tree_inject(D, IO, e)); }
    for (uint64_t i = 0; i < m; ++i) h[i] = theap_pop(h2, hn2);     // sorted run into the scratch half ...
    for (uint64_t i = 0; i < m; ++i) h2[i] = h[i];                  // ... and back
    cur[r] = off[r];
    hd[r] = m ? h2[0].t : ~0ull;
  }
  __syncthreads();
  lap(0);
  // 3. windows
  uint32_t pb = 0;                                   // pool buffer holding the pending events
  for (;;) {
    if (tid == 0) s_tmin = s_pmin;
    __syncthreads();
    {
      unsigned long long lm = ~0ull;
      for (uint32_t r = tid; r < T; r += nt) lm = min(lm, (unsigned long long)hd[r]);
      lm = tp_wave_min64(lm);
      if (ln == 0 && lm != ~0ull) atomicMin(&s_tmin, lm);
    }
    __syncthreads();
    const uint64_t tmin = s_tmin;
    if (tmin == ~0ull) break;
    const uint64_t wend = tmin + zps;
    const uint32_t n0 = s_n0;
    pw++; pn += n0;
    __syncthreads();
    if (tid == 0) { s_n1 = 0; s_nd = 0; s_na = 0; s_pmin1 = ~0ull; }
    __syncthreads();
    lap(1);
    // due events -> records linked per router; the rest carried to the other pool buffer
    auto add_due = [&](const TEv& e) {
      const uint32_t slot = atomicAdd(&s_nd, 1u), k = e.id, c = e.at;
      const uint32_t s = IO.src[k], d = IO.dst[k];
      const TGe g{e.t, IO.t0[k], 0, k, c, s, d, IO.len[k], d == GG_BROADCAST ? IO.bidx[k] : 0u, 0u,
                  tree_ports(P, c, s, d)};
      const uint32_t nx = atomicExch(&head[c], slot);
      if (nx == kTpNil) act[atomicAdd(&s_na, 1u)] = c;
      with_g(slot, [&](TGe& x) { x = g; x.next = nx; });
    };
    unsigned long long cm = ~0ull;
    for (uint32_t i = tid; i < n0; i += nt) {
      TEv e;
      with_e(pb, i, [&](TEv& x) { e = x; });
      if (e.t < wend) add_due(e);
      else { with_e(pb ^ 1u, atomicAdd(&s_n1, 1u), [&](TEv& x) { x = e; }); cm = min(cm, (unsigned long long)e.t); }
    }
    for (uint32_t r = tid; r < T; r += nt) {
      while (hd[r] < wend) {
        const uint32_t c = cur[r], e1 = off[r + 1];
        const TEv e = B.run[c];
        hd[r] = c + 1 < e1 ? B.run[c + 1].t : ~0ull;
        cur[r] = c + 1;
        add_due(e);
      }
    }
    cm = tp_wave_min64(cm);
    if (ln == 0 && cm != ~0ull) atomicMin(&s_pmin1, cm);
    __syncthreads();
    lap(2);
    const uint32_t na = s_na;
    // each router's due list sorted by (time, index); the union of its ports
    for (uint32_t i = tid; i < na; i += nt) {
      const uint32_t c = act[i];
      uint32_t sorted = kTpNil, x = head[c], u = 0;
      while (x != kTpNil) {
        TGe gx;
        with_g(x, [&](TGe& g) { gx = g; });
        const uint32_t nx = gx.next;
        u |= gx.mask;
        auto lt = [&](uint32_t y) { uint64_t ty; uint32_t ky; with_g(y, [&](TGe& g) { ty = g.t; ky = g.k; });
                                    return gx.t < ty || (gx.t == ty && gx.k < ky); };
        if (sorted == kTpNil || lt(sorted)) { with_g(x, [&](TGe& g) { g.next = sorted; }); sorted = x; }
        else {
          uint32_t y = sorted;
          for (;;) {
            uint32_t yn;
            with_g(y, [&](TGe& g) { yn = g.next; });
            if (yn == kTpNil || lt(yn)) { with_g(x, [&](TGe& g) { g.next = yn; }); with_g(y, [&](TGe& g) { g.next = x; }); break; }
            y = yn;
          }
        }
        x = nx;
      }
      head[c] = sorted;
      um[i] = (uint8_t)u;
    }
    __syncthreads();
    lap(3);
    // (router, port) tasks: the port's requests in the router's event order
    if (P.qm) {
      for (uint32_t j = tid; j < NPORTS * na; j += nt) {
        const uint32_t i = j % na, port = j / na;
        if (!((um[i] >> port) & 1u)) continue;
        const uint32_t c = act[i];
        HTree tr = D.tree(c, (int)port);
        uint32_t x = head[c];
        while (x != kTpNil) {
          with_g(x, [&](TGe& g) {
            if ((g.mask >> port) & 1u) {
              const uint64_t qd = tr.delay(time_to_cycles(g.t, P.f), nflits(P, g.len), D.err);
              if (qd) atomicMax((unsigned long long*)&g.q, (unsigned long long)qd);
            }
            x = g.next;
          });
        }
      }
      __syncthreads();
    }
    lap(4);
    // each router's events in order: counters, forwarded copies, deliveries
    {
      unsigned long long fm = ~0ull;
      for (uint32_t i = tid; i < na; i += nt) {
        const uint32_t c = act[i], cx = c % P.w, cy = c / P.w;
        TreeAcc A;
        uint32_t x = head[c];
        while (x != kTpNil) {
          TGe g;
          with_g(x, [&](TGe& y) { g = y; });
          x = g.next;
          const uint64_t nf = nflits(P, g.len), qd = g.q;
          const int np = __builtin_popcount(g.mask);
          if (P.qm) { A.rcc += qd * (uint64_t)np; A.rpk += (uint64_t)np; }
          A.buf += nf; A.sw += 1; A.crossbar(np, nf);
          A.link += nf * (uint64_t)np;
          const uint32_t sx = g.src % P.w, sy = g.src / P.w;
          const uint64_t cps = lat_to_ps(qd, P.f);
          const uint64_t hops = (uint64_t)((cx > sx ? cx - sx : sx - cx) + (cy > sy ? cy - sy : sy - cy)) + 1;
          const uint64_t t = g.t + zps + cps, zl = hops * zps, ct = t - g.t0 - zl;
          for (int port = P_LEFT; port < NPORTS; ++port) {
            if (!((g.mask >> port) & 1u)) continue;
            const TEv f{t, g.k, tree_next(P, c, port)};
            with_e(pb ^ 1u, atomicAdd(&s_n1, 1u), [&](TEv& y) { y = f; });
            fm = min(fm, (unsigned long long)t);
          }
          if (g.mask & (1u << P_SELF)) {
            const uint64_t ser = lat_to_ps(nf, P.f);   // receive at c (network_model.cc:118-150,253-272)
            A.prcv += 1; A.frcv += nf; A.brcv += g.len;
            A.lat += zl + ser + ct; A.con += ct;
            if (g.dst == GG_BROADCAST) {
              const uint64_t o = (uint64_t)g.bidx * P.tiles + c;
              IO.bout.arrival_ps_dev[o] = t + ser; IO.bout.zero_load_ps_dev[o] = zl + ser; IO.bout.contention_ps_dev[o] = ct;
            } else {
              IO.out.arrival_ps_dev[g.k] = t + ser; IO.out.zero_load_ps_dev[g.k] = zl + ser; IO.out.contention_ps_dev[g.k] = ct;
            }
          }
        }
        A.flush(D.ctr, c);
        head[c] = kTpNil;
      }
      fm = tp_wave_min64(fm);
      if (ln == 0 && fm != ~0ull) atomicMin(&s_pmin1, fm);
    }
    __syncthreads();
    lap(5);
    if (tid == 0) { s_n0 = s_n1; s_pmin = s_pmin1; }
    pb ^= 1u;
    __syncthreads();
  }
  if (prof && tid == 0) {
    for (int i = 0; i < 6; ++i) prof[i] += pc[i];
    prof[6] += pw; prof[7] += pn;
  }
}

// ---------------------------------------------------------------------------
// The windowed walk over the whole chip (k_tree_grid, the default where its
// LDS fits): the same windows as k_tree_pool, with the routers spread over
// G workgroups (one per CU), each owning a block of R consecutive routers
// and their six output-port queues as LDS images for the whole batch, so a
// queue request costs LDS latency instead of HBM round trips.  Per window:
//   grid barrier -> the window start (min over every pending event, kept in
//   three rotating words) -> the copies other blocks pushed during the last
//   window drained from the block's inbox into its pool -> the due events
//   (pool and the tiles' injection runs) linked per router, sorted by
//   (time, index) -> one task per (router, output port) -> per router:
//   counters, deliveries, forwarded copies (to the own pool, or appended to
//   the owner block's inbox for the next window) -> the next window's start
//   contributed by atomic min.
// One grid barrier per window (cooperative launch: every workgroup
// resident).  k_tree_setup (one workgroup) validates and buckets the packets
// by source first.
// ---------------------------------------------------------------------------
constexpr uint32_t kTgThreads = 256;
constexpr uint32_t kTgBarShards = 32;                // grid barrier counter shards
constexpr uint32_t kTgBarFlags = 8;                  // grid barrier release flag replicas
struct TgBufs {
  uint32_t* off;             // [T + 1] packets per source (k_tree_setup)
  TEv* pk;                   // [n] the packets bucketed by source; heap scratch
  TEv* run;                  // [n] each tile's injection router events, (time, index)-sorted
  TEv* spill;                // [2][G][bwg] the pool buffers beyond LDS
  TEv* inbox;                // [2][G][bwg] copies pushed by other blocks, per window parity
  TGe* gh;                   // [G][bwg] due records beyond LDS
  uint32_t* icnt;            // [2][G] inbox counts
  unsigned long long* gmin;  // [3] window starts (rotating)
  uint32_t* flag;            // [1] nonzero: setup rejected the batch
  uint32_t* bar;             // [kTgBarShards + kTgBarFlags][32] barrier arrival shards, release flags (128-B lines)
};

__global__ __launch_bounds__(1024) void k_tree_setup(NocDev D, TreeIO IO, uint64_t n, uint64_t nb, TgBufs B, uint64_t hcap)
{
  __shared__ uint32_t wsum[1024 / 64 + 1];
  __shared__ uint32_t s_err;
  extern __shared__ __align__(16) uint8_t ts_lds[];
  uint32_t* cnt = reinterpret_cast<uint32_t*>(ts_lds);          // [T]
  const NocParams& P = D.P;
  const uint32_t T = P.tiles, tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) s_err = 0;
  for (uint32_t i = tid; i < T; i += nt) cnt[i] = 0;
  __syncthreads();
  const uint64_t per = (n + nt - 1) / nt, k0 = min(n, tid * per), k1 = min(n, k0 + per);
  uint32_t mine = 0;
  for (uint64_t k = k0; k < k1; ++k) {
    const uint32_t s = IO.src[k], d = IO.dst[k];
    if (s >= T || (d >= T && d != GG_BROADCAST)) atomicOr(&s_err, GG_DERR_RANGE);
    mine += d == GG_BROADCAST;
    if (s < T && s != d) atomicAdd(&cnt[s], 1u);
  }
  uint32_t nbc;
  mine = block_excl_scan(mine, wsum, &nbc);
  if (tid == 0 && (nbc != nb || n + nb * T > hcap)) s_err |= GG_DERR_CAP;
  __syncthreads();
  if (s_err) { if (tid == 0) { atomicOr(D.err, s_err); *B.flag = 1; } return; }
  if (tid == 0) *B.flag = 0;
  for (uint64_t k = k0; k < k1; ++k) IO.bidx[k] = IO.dst[k] == GG_BROADCAST ? mine++ : ~0u;
  {
    const uint32_t pt = (T + nt - 1) / nt;
    uint32_t a = 0, tot;
    for (uint32_t i = tid * pt; i < min(T, (tid + 1) * pt); ++i) a += cnt[i];
    a = block_excl_scan(a, wsum, &tot);
    for (uint32_t i = tid * pt; i < min(T, (tid + 1) * pt); ++i) { B.off[i] = a; a += cnt[i]; cnt[i] = 0; }
    if (tid == 0) B.off[T] = tot;
    __syncthreads();
  }
  for (uint64_t k = k0; k < k1; ++k) {
    const uint32_t s = IO.src[k], d = IO.dst[k];
    if (s == d) { IO.out.arrival_ps_dev[k] = IO.t0[k]; IO.out.zero_load_ps_dev[k] = 0; IO.out.contention_ps_dev[k] = 0; continue; }
    B.pk[B.off[s] + atomicAdd(&cnt[s], 1u)] = TEv{IO.t0[k], (uint32_t)k, s | kInjBit};
  }
}

// LDS bytes of k_tree_grid: R routers' six queue images, run heads, two pool
// buffers of ecap events, gcap due records, per-router lists and counters
constexpr uint32_t kTgStage = 512;                   // staged copies for other blocks per window
__host__ __device__ inline size_t tg_stage_off(uint32_t R, uint32_t qb, uint32_t ecap, uint32_t gcap)
{
  return ((size_t)R * 6 * qb + 8ull * R + 8ull * R * kNetCtrTree + 2ull * ecap * sizeof(TEv) + (size_t)gcap * sizeof(TGe) +
          20ull * R + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t tg_lds_bytes(uint32_t R, uint32_t qb, uint32_t ecap, uint32_t gcap)
{
  return tg_stage_off(R, qb, ecap, gcap) + (size_t)kTgStage * (sizeof(TEv) + 8);
}

__global__ __launch_bounds__(kTgThreads) void k_tree_grid(NocDev D, TreeIO IO, TgBufs B, uint32_t R, uint32_t qb,
                                                         uint64_t bwg, uint32_t ecap, uint32_t gcap,
                                                         unsigned long long* prof)
{
  if (!GG_NOC_DIAG) prof = nullptr;
  // prof (GG_NOC_PROFILE=1, diagnostics): block 0's shader clocks per phase
  unsigned long long pc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pw = 0, pt = __builtin_amdgcn_s_memtime();
  auto lap = [&](int i) { if (prof) { const unsigned long long x = __builtin_amdgcn_s_memtime(); pc[i] += x - pt; pt = x; } };
  if (*B.flag) return;                                   // rejected in setup: every block leaves before a barrier
  extern __shared__ __align__(16) uint8_t tg_lds[];
  __shared__ unsigned long long s_pmin;
  __shared__ uint32_t s_n0, s_n1, s_nd, s_na, s_ns;
  const NocParams& P = D.P;
  const uint32_t T = P.tiles, g = blockIdx.x, G = gridDim.x, tid = threadIdx.x, nt = blockDim.x, ln = tid & 63;
  const uint32_t r0 = g * R, nr = r0 < T ? min(R, T - r0) : 0u;
  const uint64_t zps = lat_to_ps((uint64_t)P.router_delay + P.link_delay, P.f);
  uint8_t* img = tg_lds;                                                        // [R][6] queue images
  uint64_t* hd = reinterpret_cast<uint64_t*>(img + (size_t)R * 6 * qb);          // [R] run head times
  uint64_t* lctr = hd + R;                                                      // [R][kNetCtrTree] router counters
  TEv* El[2] = {reinterpret_cast<TEv*>(lctr + (size_t)R * kNetCtrTree), reinterpret_cast<TEv*>(lctr + (size_t)R * kNetCtrTree) + ecap};
  TGe* Gl = reinterpret_cast<TGe*>(El[1] + ecap);                               // [gcap]
  uint32_t* cur = reinterpret_cast<uint32_t*>(Gl + gcap);                       // [R] run cursors
  uint32_t* end = cur + R;                                                      // [R]
  uint32_t* head = end + R;                                                     // [R] due list per local router
  uint32_t* act = head + R;                                                     // [R] local routers with due events
  uint32_t* um = act + R;                                                       // [R] their ports
  TEv* stg = reinterpret_cast<TEv*>(tg_lds + tg_stage_off(R, qb, ecap, gcap));     // [kTgStage] copies for other blocks
  uint32_t* stg_og = reinterpret_cast<uint32_t*>(stg + kTgStage);               // [kTgStage] their block
  uint32_t* stg_base = stg_og + kTgStage;                                       // [kTgStage] slot of a block's first copy
  TEv* const sp[2] = {B.spill + (size_t)g * bwg, B.spill + ((size_t)G + g) * bwg};
  TGe* const gh = B.gh + (size_t)g * bwg;
  auto with_g = [&](uint32_t i, auto f) { if (i < gcap) f(Gl[i]); else f(gh[i - gcap]); };
  auto with_e = [&](uint32_t b, uint32_t i, auto f) { if (i < ecap) f(El[b][i]); else f(sp[b][i - ecap]); };
  // Cross-block data (inbox records and counts, window starts) moves with
  // agent-scope (sc1) stores / loads and atomics only, so the grid barrier
  // needs no L2 write-back or invalidate: every wave waits for its stores,
  // the workgroup meets, one lane adds to the arrival counter and polls it
  // with sc1 loads (MI355X_MICROARCH.md, inter-workgroup hand-offs, row 1).
  // Arrivals: each block adds 1 to its shard of a sharded counter
  // (kTgBarShards words, one 128-B line each, so the adds do not serialize on
  // one address); block 0 polls every shard and then publishes the
  // generation in kTgBarFlags replicated flags; every other block polls its
  // replica (one line read by G / kTgBarFlags blocks, not by all G).
  unsigned long long pbw = 0, pbp = 0, pbn = 0;
  uint32_t* const flags = B.bar + kTgBarShards * 32;
  auto gbar = [&](uint32_t gen) {
    const unsigned long long b0 = prof ? __builtin_amdgcn_s_memtime() : 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long b1 = prof ? __builtin_amdgcn_s_memtime() : 0;
    if (tid < 64) {
      if (tid == 0) atomicAdd(&B.bar[(g % kTgBarShards) * 32], 1u);
      uint32_t spin = 0;
      if (g == 0) {
        const uint32_t target = gen * G;
        for (;; ++spin) {
          const uint32_t v = tid < kTgBarShards ? __hip_atomic_load(&B.bar[tid * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
          uint32_t sum = v;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) sum += (uint32_t)__shfl_xor((int)sum, o);
          if (sum >= target) break;
          if (spin > (1u << 26)) { if (tid == 0) atomicOr(D.err, GG_DERR_STATE); break; }
          __builtin_amdgcn_s_sleep(1);
          ++pbn;
        }
        if (tid < kTgBarFlags) __hip_atomic_store(&flags[tid * 32], gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (tid == 0) {
        uint32_t* f = &flags[(g % kTgBarFlags) * 32];
        for (; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen; ++spin) {
          if (spin > (1u << 26)) { atomicOr(D.err, GG_DERR_STATE); break; }
          __builtin_amdgcn_s_sleep(1);
          ++pbn;
        }
      }
    }
    __syncthreads();
    if (prof) { const unsigned long long b2 = __builtin_amdgcn_s_memtime(); pbw += b1 - b0; pbp += b2 - b1; }
  };
  auto ld_ev = [](const TEv* p) {
    const uint64_t a = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t b = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return TEv{a, (uint32_t)b, (uint32_t)(b >> 32)};
  };
  auto st_ev = [](TEv* p, const TEv& e) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), e.t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p) + 1, (uint64_t)e.id | ((uint64_t)e.at << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  };
  auto qtree = [&](uint32_t lr, int port) {
    uint8_t* q = img + ((size_t)lr * 6 + port) * qb;
    return HTree{reinterpret_cast<HQueue*>(q), reinterpret_cast<HNode*>(q + sizeof(HQueue)), 1, P.analytical != 0};
  };
  // the block's queue images into LDS; counters zero
  {
    const uint32_t words = qb / 16, per_q = words;
    for (uint32_t i = tid; i < nr * 6 * per_q; i += nt) {
      const uint32_t qi = i / per_q, wd = i % per_q, lr = qi / 6, port = qi % 6;
      const uint64_t gq = (uint64_t)(r0 + lr) * 6 + port;
      uint4 v;
      if (wd * 16 < sizeof(HQueue)) v = reinterpret_cast<const uint4*>(D.q + gq)[wd];
      else v = reinterpret_cast<const uint4*>(D.nd + gq * P.max_size)[wd - sizeof(HQueue) / 16];
      reinterpret_cast<uint4*>(img + (size_t)qi * qb)[wd] = v;
    }
    for (uint32_t i = tid; i < nr * kNetCtrTree; i += nt) lctr[i] = 0;
    for (uint32_t i = tid; i < nr; i += nt) head[i] = kTpNil;
    if (tid == 0) { s_n0 = 0; s_pmin = ~0ull; }
  }
  __syncthreads();
  // injection ports of the block's tiles: each tile's packets in (time, index)
  // order through its injection queue; the router events re-sorted into its run
  for (uint32_t lr = tid; lr < nr; lr += nt) {
    const uint32_t r = r0 + lr, o = B.off[r], m = B.off[r + 1] - o;
    TEv* h = B.pk + o;
    TEv* h2 = B.run + o;
    uint64_t hn = 0, hn2 = 0;
    for (uint32_t i = 0; i < m; ++i) { const TEv e = h[i]; theap_push(h, hn, e); }
    HTree tq = qtree(lr, 5);
    while (hn) {
      const TEv e = theap_pop(h, hn);
      const uint32_t k = e.id, bits = IO.len[k];
      const uint64_t nf = nflits(P, bits);
      tcadd(D.ctr, r, GG_NC_PACKETS_SENT, 1); tcadd(D.ctr, r, GG_NC_FLITS_SENT, nf); tcadd(D.ctr, r, GG_NC_BITS_SENT, bits);
      if (IO.dst[k] == GG_BROADCAST) {                 // updateSendCounters (network_model.cc:244-250)
        tcadd(D.ctr, r, GG_NC_PACKETS_BROADCASTED, 1); tcadd(D.ctr, r, GG_NC_FLITS_BROADCASTED, nf);
        tcadd(D.ctr, r, GG_NC_BITS_BROADCASTED, bits);
      }
      const uint64_t qd = P.qm ? tq.delay(time_to_cycles(e.t, P.f), nf, D.err) : 0;
      theap_push(h2, hn2, TEv{e.t + lat_to_ps(0, P.f) + lat_to_ps(qd, P.f), k, r});
    }
    for (uint32_t i = 0; i < m; ++i) h[i] = theap_pop(h2, hn2);
    for (uint32_t i = 0; i < m; ++i) h2[i] = h[i];
    cur[lr] = o; end[lr] = o + m;
    hd[lr] = m ? h2[0].t : ~0ull;
    if (m) atomicMin(&B.gmin[0], (unsigned long long)h2[0].t);
  }
  // 3. windows
  lap(0);
  for (uint32_t w = 0;; ++w) {
    gbar(w + 1);
    lap(1);
    const uint64_t tmin = __hip_atomic_load(&B.gmin[w % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tmin == ~0ull) break;
    ++pw;
    if (g == 0 && tid == 0) __hip_atomic_store(&B.gmin[(w + 2) % 3], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t wend = tmin + zps;
    const uint32_t pin = w & 1u, pout = pin ^ 1u, pb = w & 1u;      // pool buffer pb holds the pending events
    // the copies other blocks pushed in the last window join the pool
    const uint32_t nin = __hip_atomic_load(&B.icnt[pin * G + g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const TEv* inb = B.inbox + ((size_t)pin * G + g) * bwg;
    const uint32_t n0 = s_n0;
    for (uint32_t i = tid; i < nin; i += nt) { const TEv e = ld_ev(inb + i); with_e(pb, n0 + i, [&](TEv& x) { x = e; }); }
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_store(&B.icnt[pin * G + g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_n0 = n0 + nin; s_n1 = 0; s_nd = 0; s_na = 0; s_ns = 0; s_pmin = ~0ull;
    }
    __syncthreads();
    const uint32_t np0 = s_n0;
    auto add_due = [&](const TEv& e) {
      const uint32_t slot = atomicAdd(&s_nd, 1u), k = e.id, c = e.at, lr = c - r0;
      const uint32_t s = IO.src[k], d = IO.dst[k];
      const TGe gr{e.t, IO.t0[k], 0, k, c, s, d, IO.len[k], d == GG_BROADCAST ? IO.bidx[k] : 0u, 0u,
                   tree_ports(P, c, s, d)};
      const uint32_t nx = atomicExch(&head[lr], slot);
      if (nx == kTpNil) act[atomicAdd(&s_na, 1u)] = lr;
      with_g(slot, [&](TGe& x) { x = gr; x.next = nx; });
    };
    unsigned long long cm = ~0ull;
    for (uint32_t i = tid; i < np0; i += nt) {
      TEv e;
      with_e(pb, i, [&](TEv& x) { e = x; });
      if (e.t < wend) add_due(e);
      else { with_e(pb ^ 1u, atomicAdd(&s_n1, 1u), [&](TEv& x) { x = e; }); cm = min(cm, (unsigned long long)e.t); }
    }
    for (uint32_t lr = tid; lr < nr; lr += nt) {
      while (hd[lr] < wend) {
        const uint32_t c = cur[lr];
        const TEv e = B.run[c];
        hd[lr] = c + 1 < end[lr] ? B.run[c + 1].t : ~0ull;
        cur[lr] = c + 1;
        add_due(e);
      }
      cm = min(cm, (unsigned long long)hd[lr]);
    }
    cm = tp_wave_min64(cm);
    if (ln == 0 && cm != ~0ull) atomicMin(&s_pmin, cm);
    __syncthreads();
    lap(2);
    const uint32_t na = s_na;
    // each router's due list sorted by (time, index); the union of its ports
    for (uint32_t i = tid; i < na; i += nt) {
      const uint32_t lr = act[i];
      uint32_t sorted = kTpNil, x = head[lr], u = 0;
      while (x != kTpNil) {
        TGe gx;
        with_g(x, [&](TGe& y) { gx = y; });
        const uint32_t nx = gx.next;
        u |= gx.mask;
        auto lt = [&](uint32_t y) { uint64_t ty; uint32_t ky; with_g(y, [&](TGe& z) { ty = z.t; ky = z.k; });
                                    return gx.t < ty || (gx.t == ty && gx.k < ky); };
        if (sorted == kTpNil || lt(sorted)) { with_g(x, [&](TGe& y) { y.next = sorted; }); sorted = x; }
        else {
          uint32_t y = sorted;
          for (;;) {
            uint32_t yn;
            with_g(y, [&](TGe& z) { yn = z.next; });
            if (yn == kTpNil || lt(yn)) { with_g(x, [&](TGe& z) { z.next = yn; }); with_g(y, [&](TGe& z) { z.next = x; }); break; }
            y = yn;
          }
        }
        x = nx;
      }
      head[lr] = sorted;
      um[i] = u;
    }
    __syncthreads();
    lap(3);
    // (router, port) tasks on the LDS queue images
    if (P.qm) {
      for (uint32_t j = tid; j < NPORTS * na; j += nt) {
        const uint32_t i = j % na, port = j / na;
        if (!((um[i] >> port) & 1u)) continue;
        const uint32_t lr = act[i];
        HTree tr = qtree(lr, (int)port);
        uint32_t x = head[lr];
        while (x != kTpNil) {
          with_g(x, [&](TGe& gx) {
            if ((gx.mask >> port) & 1u) {
              const uint64_t qd = tr.delay(time_to_cycles(gx.t, P.f), nflits(P, gx.len), D.err);
              if (qd) atomicMax((unsigned long long*)&gx.q, (unsigned long long)qd);
            }
            x = gx.next;
          });
        }
      }
      __syncthreads();
    }
    lap(4);
    // per router, in order: counters, deliveries, forwarded copies
    {
      unsigned long long fm = ~0ull, rm = ~0ull;
      for (uint32_t i = tid; i < na; i += nt) {
        const uint32_t lr = act[i], c = r0 + lr, cx = c % P.w, cy = c / P.w;
        uint64_t* L = lctr + (size_t)lr * kNetCtrTree;
        uint32_t x = head[lr];
        while (x != kTpNil) {
          TGe gx;
          with_g(x, [&](TGe& y) { gx = y; });
          x = gx.next;
          const uint64_t nf = nflits(P, gx.len), qd = gx.q;
          const int np = __builtin_popcount(gx.mask);
          if (P.qm) { L[0] += qd * (uint64_t)np; L[1] += (uint64_t)np; }
          L[2] += nf; L[3] += 1; L[4 + min(np, 5) - 1] += nf; L[9] += nf * (uint64_t)np;
          const uint32_t sx = gx.src % P.w, sy = gx.src / P.w;
          const uint64_t cps = lat_to_ps(qd, P.f);
          const uint64_t hops = (uint64_t)((cx > sx ? cx - sx : sx - cx) + (cy > sy ? cy - sy : sy - cy)) + 1;
          const uint64_t t = gx.t + zps + cps, zl = hops * zps, ct = t - gx.t0 - zl;
          for (int port = P_LEFT; port < NPORTS; ++port) {
            if (!((gx.mask >> port) & 1u)) continue;
            const uint32_t nc = tree_next(P, c, port), og = nc / R;
            const TEv f{t, gx.k, nc};
            if (og == g) { with_e(pb ^ 1u, atomicAdd(&s_n1, 1u), [&](TEv& y) { y = f; }); fm = min(fm, (unsigned long long)t); }
            else {
              rm = min(rm, (unsigned long long)t);
              const uint32_t j = atomicAdd(&s_ns, 1u);
              if (j < kTgStage) { stg[j] = f; stg_og[j] = og; continue; }
              const uint32_t slot = atomicAdd(&B.icnt[pout * G + og], 1u);   // staging full: one by one
              if (slot >= bwg) { atomicOr(D.err, GG_DERR_CAP); continue; }
              st_ev(B.inbox + ((size_t)pout * G + og) * bwg + slot, f);
            }
          }
          if (gx.mask & (1u << P_SELF)) {
            const uint64_t ser = lat_to_ps(nf, P.f);   // receive at c (network_model.cc:118-150,253-272)
            L[10] += 1; L[11] += nf; L[12] += gx.len; L[13] += zl + ser + ct; L[14] += ct;
            if (gx.dst == GG_BROADCAST) {
              const uint64_t o = (uint64_t)gx.bidx * P.tiles + c;
              IO.bout.arrival_ps_dev[o] = t + ser; IO.bout.zero_load_ps_dev[o] = zl + ser; IO.bout.contention_ps_dev[o] = ct;
            } else {
              IO.out.arrival_ps_dev[gx.k] = t + ser; IO.out.zero_load_ps_dev[gx.k] = zl + ser; IO.out.contention_ps_dev[gx.k] = ct;
            }
          }
        }
        head[lr] = kTpNil;
      }
      fm = tp_wave_min64(fm);
      if (ln == 0 && fm != ~0ull) atomicMin(&s_pmin, fm);
      rm = tp_wave_min64(rm);
      if (ln == 0 && rm != ~0ull) atomicMin(&B.gmin[(w + 1) % 3], rm);
    }
    __syncthreads();
    // the staged copies: one slot reservation per destination block (its
    // first copy's thread adds the block's count), then every copy stored
    {
      const uint32_t ns = min(s_ns, kTgStage);
      for (uint32_t j = tid; j < ns; j += nt) {
        const uint32_t og = stg_og[j];
        bool first = true;
        uint32_t tot = 0;
        for (uint32_t k = 0; k < ns; ++k) { const bool same = stg_og[k] == og; tot += same; first = first && !(same && k < j); }
        if (first) stg_base[j] = atomicAdd(&B.icnt[pout * G + og], tot);
      }
      __syncthreads();
      for (uint32_t j = tid; j < ns; j += nt) {
        const uint32_t og = stg_og[j];
        uint32_t lead = j, rank = 0;
        for (uint32_t k = 0; k < j; ++k) if (stg_og[k] == og) { ++rank; lead = min(lead, k); }
        const uint32_t slot = stg_base[lead] + rank;
        if (slot >= bwg) { atomicOr(D.err, GG_DERR_CAP); continue; }
        st_ev(B.inbox + ((size_t)pout * G + og) * bwg + slot, stg[j]);
      }
    }
    __syncthreads();
    if (tid == 0) {
      if (s_pmin != ~0ull) atomicMin(&B.gmin[(w + 1) % 3], s_pmin);
      s_n0 = s_n1;
    }
    lap(5);
  }
  if (prof && g == 0 && tid == 0) {               // slots 16..: the chain sweep uses 0..15
    for (int i = 0; i < 6; ++i) prof[16 + i] += pc[i];
    prof[22] += pw;
  }
  if (prof && tid == 0) {                        // the busiest block: most work, least barrier wait
    atomicMax(&prof[24], pc[2] + pc[3] + pc[4] + pc[5]);
    atomicMin(&prof[25], pc[1]);
    if (g == 0) { prof[26] += pbw; prof[27] += pbp; prof[28] += pbn; }
  }
  // the queue images and the counters back to HBM
  {
    const uint32_t per_q = qb / 16;
    for (uint32_t i = tid; i < nr * 6 * per_q; i += nt) {
      const uint32_t qi = i / per_q, wd = i % per_q, lr = qi / 6, port = qi % 6;
      const uint64_t gq = (uint64_t)(r0 + lr) * 6 + port;
      const uint4 v = reinterpret_cast<const uint4*>(img + (size_t)qi * qb)[wd];
      if (wd * 16 < sizeof(HQueue)) reinterpret_cast<uint4*>(D.q + gq)[wd] = v;
      else reinterpret_cast<uint4*>(D.nd + gq * P.max_size)[wd - sizeof(HQueue) / 16] = v;
    }
    for (uint32_t lr = tid; lr < nr; lr += nt) {
      const uint64_t* L = lctr + (size_t)lr * kNetCtrTree;
      const uint32_t c = r0 + lr;
      tcadd(D.ctr, c, GG_NC_ROUTER_CONTENTION_CYCLES, L[0]); tcadd(D.ctr, c, GG_NC_ROUTER_PACKETS, L[1]);
      tcadd(D.ctr, c, GG_NC_BUFFER_WRITES, L[2]); tcadd(D.ctr, c, GG_NC_BUFFER_READS, L[2]);
      tcadd(D.ctr, c, GG_NC_SWITCH_ALLOC, L[3]); tcadd(D.ctr, c, GG_NC_CROSSBAR, L[4]);
      tcadd(D.ctr, c, GG_NC_CROSSBAR_MULTI + 0, L[5]); tcadd(D.ctr, c, GG_NC_CROSSBAR_MULTI + 1, L[6]);
      tcadd(D.ctr, c, GG_NC_CROSSBAR_MULTI + 2, L[7]); tcadd(D.ctr, c, GG_NC_CROSSBAR_MULTI + 3, L[8]);
      tcadd(D.ctr, c, GG_NC_LINK_TRAVERSALS, L[9]); tcadd(D.ctr, c, GG_NC_PACKETS_RECEIVED, L[10]);
      tcadd(D.ctr, c, GG_NC_FLITS_RECEIVED, L[11]); tcadd(D.ctr, c, GG_NC_BITS_RECEIVED, L[12]);
      tcadd(D.ctr, c, GG_NC_TOTAL_LATENCY_PS, L[13]); tcadd(D.ctr, c, GG_NC_TOTAL_CONTENTION_PS, L[14]);
    }
  }
}

struct gg_noc_state {
  NocParams P;
  HQueue* q = nullptr; HNode* nd = nullptr; uint64_t nq = 0;
  uint64_t* ctr = nullptr;
  // batch scratch
  uint64_t cap = 0;
  uint64_t *t = nullptr, *zl = nullptr, *ct = nullptr;
  uint32_t *cur = nullptr, *keys = nullptr, *ids = nullptr;
  Ev* heap = nullptr;
  uint32_t* counts = nullptr; uint32_t* cursor = nullptr; uint64_t* off = nullptr; uint32_t nb_cap = 0;
  TEv* theap = nullptr; uint32_t* bidx = nullptr; uint64_t tcap = 0, bcap = 0;   // broadcast-tree walk scratch
  unsigned long long* prof = nullptr;             // GG_NOC_PROFILE=1: k_chain_sweep phase cycles (diagnostics)
  SK* pscr = nullptr; uint64_t pscr_cap = 0;       // k_chain_pipe: per packet 3 x positions pool / incoming slots
  uint8_t* tp = nullptr; uint64_t tp_bytes = 0;     // k_tree_pool: TpBufs
  uint8_t* tg = nullptr; uint64_t tg_bytes = 0;     // k_tree_setup / k_tree_grid: TgBufs
};

gg_status gg_noc_alloc(gg_ctx* ctx)
{
  gg_noc_state* S = new gg_noc_state();
  ctx->noc = S;
  const gg_config& c = ctx->cfg;
  NocParams& P = S->P;
  P.tiles = c.num_tiles;
  P.w = (uint32_t)floor(sqrt((double)c.num_tiles));               // hop_counter.cc:18-19
  P.h = (uint32_t)ceil(1.0 * c.num_tiles / P.w);
  P.flit_width = c.flit_width ? c.flit_width : 64;
  P.router_delay = c.router_delay;
  P.link_delay = c.link_delay;
  P.qm = c.queue_model_enabled;
  P.analytical = c.analytical_enabled;
  P.max_size = c.max_list_size ? c.max_list_size : 100;
  P.net_model = c.net_model;
  P.f = c.frequency_ghz;
  if (P.max_size > 32767) return gg_fail(GG_ERR_UNSUPPORTED, "max_list_size too large");
  P.qtype = c.queue_model_type;
  P.qaux = hq_aux(c.queue_model_type, c.basic_moving_avg, c.history_list_no_interleaving);
  if (gg_status e = gg_check_queue_model(c.queue_model_type, P.qaux, P.max_size)) return e;
  if (getenv("GG_NOC_PROFILE") && atoi(getenv("GG_NOC_PROFILE"))) {
    if (!GG_NOC_DIAG) fprintf(stderr, "[gg_noc] GG_NOC_PROFILE needs a diagnostics build (-DGG_NOC_DIAG=1)\n");
    GG_HIP(hipMalloc((void**)&S->prof, 32 * sizeof(unsigned long long)));
    GG_HIP(hipMemset(S->prof, 0, 32 * sizeof(unsigned long long)));
    GG_HIP(hipMemset(S->prof + 25, 0xFF, sizeof(unsigned long long)));
  }
  GG_HIP(hipFuncSetAttribute((const void*)k_chain_sweep, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStageLdsMax));
  GG_HIP(hipFuncSetAttribute((const void*)k_chain_pipe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStageLdsMax));
  GG_HIP(hipFuncSetAttribute((const void*)k_port_sweep<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPortLds));
  GG_HIP(hipFuncSetAttribute((const void*)k_port_sweep<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPortLds));
  static_assert(kSweepLds <= kStageLdsMax, "the sweep's LDS arrays fit the stage budget");
  GG_HIP(hipFuncSetAttribute((const void*)k_tree_pool, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTpLds));
  GG_HIP(hipFuncSetAttribute((const void*)k_tree_grid, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTpLds));
  GG_HIP(hipFuncSetAttribute((const void*)k_tree_walk<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)(kTreeLdsEv * sizeof(TEv))));
  GG_HIP(hipMalloc((void**)&S->ctr, sizeof(uint64_t) * c.num_tiles * GG_NUM_NET_COUNTERS));
  // one history tree per mesh output port (5) + the injection port, per tile; the
  // stand-alone gg_queue_delay_batch queue lives at index tiles*6
  S->nq = (uint64_t)c.num_tiles * 6 + 1;
  GG_HIP(hipMalloc((void**)&S->q, sizeof(HQueue) * S->nq));
  GG_HIP(hipMalloc((void**)&S->nd, sizeof(HNode) * S->nq * P.max_size));
  return GG_OK;
}

void gg_noc_free(gg_ctx* ctx)
{
  gg_noc_state* S = ctx->noc;
  if (!S) return;
  void* ps[] = {S->q, S->nd, S->ctr, S->t, S->zl, S->ct, S->cur, S->keys, S->ids, S->heap,
                S->counts, S->cursor, S->off, S->theap, S->bidx, S->prof, S->pscr, S->tp, S->tg};
  for (void* p : ps) if (p) hipFree(p);
  delete S;
  ctx->noc = nullptr;
}

gg_status gg_noc_reset(gg_ctx* ctx, hipStream_t s)
{
  gg_noc_state* S = ctx->noc;
  GG_HIP(hipMemsetAsync(S->ctr, 0, sizeof(uint64_t) * S->P.tiles * GG_NUM_NET_COUNTERS, s));
  hipLaunchKernelGGL(k_htree_reset, dim3((uint32_t)((S->nq + 255) / 256)), dim3(256), 0, s, S->q, S->nd,
                     S->nq, S->P.max_size, S->P.qtype, S->P.qaux);
  GG_HIP(hipGetLastError());
  return GG_OK;
}

static gg_status noc_grow(gg_noc_state* S, uint64_t n, uint32_t nb)
{
  if (n > S->cap) {
    void* ps[] = {S->t, S->zl, S->ct, S->cur, S->keys, S->ids, S->heap};
    for (void* p : ps) if (p) hipFree(p);
    uint64_t c = n + n / 4 + 1024;
    GG_HIP(hipMalloc((void**)&S->t, 8 * c)); GG_HIP(hipMalloc((void**)&S->zl, 8 * c));
    GG_HIP(hipMalloc((void**)&S->ct, 8 * c)); GG_HIP(hipMalloc((void**)&S->cur, 4 * c));
    GG_HIP(hipMalloc((void**)&S->keys, 4 * c)); GG_HIP(hipMalloc((void**)&S->ids, 4 * c));
    GG_HIP(hipMalloc((void**)&S->heap, sizeof(Ev) * c));
    S->cap = c;
  }
  if (nb > S->nb_cap) {
    if (S->counts) { hipFree(S->counts); hipFree(S->cursor); hipFree(S->off); }
    GG_HIP(hipMalloc((void**)&S->counts, 4 * (nb + 1)));
    GG_HIP(hipMalloc((void**)&S->cursor, 4 * (nb + 1)));
    GG_HIP(hipMalloc((void**)&S->off, 8 * (nb + 1)));
    S->nb_cap = nb;
  }
  return GG_OK;
}

gg_status gg_noc_run(gg_ctx* ctx, const gg_packets* pk, const gg_packet_out* out, hipStream_t s)
{
  gg_noc_state* S = ctx->noc;
  const NocParams& P = S->P;
  const uint64_t n = pk->num_packets;
  if (n == 0) return GG_OK;
  if (!pk->src_dev || !pk->dst_dev || !pk->length_bits_dev || !pk->time_ps_dev ||
      !out->arrival_ps_dev || !out->zero_load_ps_dev || !out->contention_ps_dev)
    return gg_fail(GG_ERR_INVALID, "NULL packet or output pointer");
  if (n >= (1ull << 32)) return gg_fail(GG_ERR_RANGE, "batch larger than 2^32 packets");
  const uint32_t blocks = (uint32_t)((n + 255) / 256);
  if (P.net_model == GG_NET_MAGIC || P.net_model == GG_NET_EMESH_HOP_COUNTER) {
    gg_timer_begin(ctx, "noc_hop_counter", s);
    hipLaunchKernelGGL(k_hop_counter, dim3(blocks), dim3(256), 0, s, P, pk->src_dev, pk->dst_dev,
                       pk->length_bits_dev, pk->time_ps_dev, n, out->arrival_ps_dev, out->zero_load_ps_dev,
                       out->contention_ps_dev, S->ctr);
    GG_HIP(hipGetLastError());
    gg_timer_end(ctx, "noc_hop_counter", s);
    return GG_OK;
  }
  if (P.net_model != GG_NET_EMESH_HOP_BY_HOP) return gg_fail(GG_ERR_UNSUPPORTED, "network model %u", P.net_model);
  if (P.w * P.h != P.tiles) return gg_fail(GG_ERR_UNSUPPORTED, "emesh_hop_by_hop needs a full W x H mesh (hop_by_hop.cc:55-59)");
  if (gg_status st = gg_noc_hbh(ctx, pk->src_dev, pk->dst_dev, pk->length_bits_dev, pk->time_ps_dev, nullptr, nullptr,
                                n, nullptr, s))
    return st;
  GG_HIP(hipMemcpyAsync(out->arrival_ps_dev, S->t, 8 * n, hipMemcpyDeviceToDevice, s));
  GG_HIP(hipMemcpyAsync(out->zero_load_ps_dev, S->zl, 8 * n, hipMemcpyDeviceToDevice, s));
  GG_HIP(hipMemcpyAsync(out->contention_ps_dev, S->ct, 8 * n, hipMemcpyDeviceToDevice, s));
  return GG_OK;
}

gg_status gg_noc_tree(gg_ctx* ctx, const gg_packets* pk, const gg_packet_out* out, const gg_packet_out* bout,
                      uint64_t nb, hipStream_t s)
{
  gg_noc_state* S = ctx->noc;
  const NocParams& P = S->P;
  const uint64_t n = pk->num_packets;
  if (P.net_model != GG_NET_EMESH_HOP_BY_HOP)
    return gg_fail(GG_ERR_UNSUPPORTED, "broadcast tree: emesh_hop_by_hop only (network.cc:187-195 unrolls the others)");
  if (P.w * P.h != P.tiles) return gg_fail(GG_ERR_UNSUPPORTED, "emesh_hop_by_hop needs a full W x H mesh (hop_by_hop.cc:55-59)");
  if (n == 0) return GG_OK;
  if (!pk->src_dev || !pk->dst_dev || !pk->length_bits_dev || !pk->time_ps_dev ||
      !out->arrival_ps_dev || !out->zero_load_ps_dev || !out->contention_ps_dev ||
      (nb && (!bout || !bout->arrival_ps_dev || !bout->zero_load_ps_dev || !bout->contention_ps_dev)))
    return gg_fail(GG_ERR_INVALID, "NULL packet or output pointer");
  if (n >= (1ull << 32) || nb > n) return gg_fail(GG_ERR_RANGE, "batch larger than 2^32 packets or num_broadcasts > packets");
  const uint64_t hcap = n + nb * P.tiles;          // live copies of a broadcast <= tiles
  // the windowed walk needs lookahead (a hop takes >= 1 cycle), its LDS per-router
  // arrays (kTreeMaxT) and 32-bit event indices; everything else takes the serial walk
  const bool win = (uint64_t)P.router_delay + P.link_delay > 0 && P.tiles <= kTreeMaxT &&
                   hcap < (1ull << 32) && !(getenv("GG_NOC_TREE_SERIAL") && atoi(getenv("GG_NOC_TREE_SERIAL")));
  const uint32_t tp_gcap = P.tiles <= 2048 ? 1024u : 512u;
  const size_t tp_base = tp_lds_bytes(P.tiles, tp_gcap, 0);
  const uint32_t tp_ecap = tp_base < kTpLds ? (uint32_t)((kTpLds - tp_base) / (2 * sizeof(TEv))) : 0u;
  // the grid form where its LDS, its scratch and a co-resident grid fit
  // (GG_NOC_TREE_POOL=1: the one-workgroup form, A/B)
  const uint32_t tg_qb = (uint32_t)(sizeof(HQueue) + (size_t)P.max_size * sizeof(HNode));
  const uint32_t tg_G0 = std::min<uint32_t>((uint32_t)ctx->num_cus, P.tiles);
  const uint32_t tg_R = (P.tiles + tg_G0 - 1) / tg_G0, tg_G = (P.tiles + tg_R - 1) / tg_R;
  const uint32_t tg_gcap = 256;
  const size_t tg_base = tg_lds_bytes(tg_R, tg_qb, 0, tg_gcap);
  const uint32_t tg_ecap = tg_base < kTpLds ? (uint32_t)std::min<size_t>(2048, (kTpLds - tg_base) / (2 * sizeof(TEv))) : 0u;
  const uint64_t tg_bwg = (n - nb) + nb * tg_R + 64;
  const uint64_t tg_need = 4 * n * sizeof(TEv) + 4ull * (P.tiles + 1) + (uint64_t)tg_G * tg_bwg * (4 * sizeof(TEv) + sizeof(TGe)) +
                           8 * (uint64_t)tg_G + 128ull * (kTgBarShards + kTgBarFlags) + 256;
  bool gridf = win && tg_ecap >= 64 && tg_need <= (2ull << 30) &&
               !(getenv("GG_NOC_TREE_POOL") && atoi(getenv("GG_NOC_TREE_POOL")));
  const size_t tg_lds = tg_lds_bytes(tg_R, tg_qb, tg_ecap, tg_gcap);
  if (gridf) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_tree_grid, kTgThreads, tg_lds) != hipSuccess ||
        (uint64_t)per_cu * (uint64_t)ctx->num_cus < tg_G)
      gridf = false;
  }
  const bool pool = win && !gridf && tp_ecap >= 64;
  const bool lds = !gridf && !pool && hcap <= kTreeLdsEv;
  const uint64_t need = gridf || pool || lds ? 0 : hcap;
  if (need > S->tcap) {
    if (S->theap) hipFree(S->theap);
    GG_HIP(hipMalloc((void**)&S->theap, sizeof(TEv) * need));
    S->tcap = need;
  }
  if (n > S->bcap) {
    if (S->bidx) hipFree(S->bidx);
    GG_HIP(hipMalloc((void**)&S->bidx, 4 * n));
    S->bcap = n;
  }
  TgBufs GB{};
  if (gridf) {
    if (tg_need > S->tg_bytes) {
      if (S->tg) hipFree(S->tg);
      GG_HIP(hipMalloc((void**)&S->tg, tg_need));
      S->tg_bytes = tg_need;
    }
    uint8_t* b = S->tg;
    auto take = [&](uint64_t bytes) { uint8_t* r = b; b += (bytes + 15) & ~15ull; return r; };
    GB.pk = reinterpret_cast<TEv*>(take(n * sizeof(TEv)));
    GB.run = reinterpret_cast<TEv*>(take(n * sizeof(TEv)));
    GB.spill = reinterpret_cast<TEv*>(take(2ull * tg_G * tg_bwg * sizeof(TEv)));
    GB.inbox = reinterpret_cast<TEv*>(take(2ull * tg_G * tg_bwg * sizeof(TEv)));
    GB.gh = reinterpret_cast<TGe*>(take((uint64_t)tg_G * tg_bwg * sizeof(TGe)));
    GB.off = reinterpret_cast<uint32_t*>(take(4ull * (P.tiles + 1)));
    GB.icnt = reinterpret_cast<uint32_t*>(take(8ull * tg_G));
    GB.gmin = reinterpret_cast<unsigned long long*>(take(3 * 8));
    GB.flag = reinterpret_cast<uint32_t*>(take(4));
    GB.bar = reinterpret_cast<uint32_t*>(take(128ull * (kTgBarShards + kTgBarFlags)));
    GG_HIP(hipMemsetAsync(GB.icnt, 0, 8ull * tg_G, s));
    GG_HIP(hipMemsetAsync(GB.bar, 0, 128ull * (kTgBarShards + kTgBarFlags), s));
    GG_HIP(hipMemsetAsync(GB.gmin, 0xFF, 3 * 8, s));
  }
  TpBufs TB{};
  if (pool) {
    const uint64_t need_b = 2 * n * sizeof(TEv) + 2 * hcap * sizeof(TEv) + hcap * sizeof(TGe);
    if (need_b > S->tp_bytes) {
      if (S->tp) hipFree(S->tp);
      GG_HIP(hipMalloc((void**)&S->tp, need_b));
      S->tp_bytes = need_b;
    }
    TEv* e = reinterpret_cast<TEv*>(S->tp);
    TB.run = e; TB.heap = e + n; TB.hp[0] = e + 2 * n; TB.hp[1] = e + 2 * n + hcap;
    TB.gh = reinterpret_cast<TGe*>(e + 2 * n + 2 * hcap);
  }
  NocDev D{P, S->q, S->nd, S->ctr, ctx->err_dev};
  const gg_packet_out none{nullptr, nullptr, nullptr};
  TreeIO IO{pk->src_dev, pk->dst_dev, pk->length_bits_dev, pk->time_ps_dev, S->bidx, *out, nb ? *bout : none};
  gg_timer_begin(ctx, "noc_tree", s);
  if (gridf) {
    hipLaunchKernelGGL(k_tree_setup, dim3(1), dim3(1024), 4 * P.tiles, s, D, IO, n, nb, GB, hcap);
    GG_HIP(hipGetLastError());
    uint32_t R = tg_R, qb = tg_qb, ec = tg_ecap, gc = tg_gcap;
    uint64_t bwg = tg_bwg;
    unsigned long long* pr = S->prof;
    void* args[] = {(void*)&D, (void*)&IO, (void*)&GB, (void*)&R, (void*)&qb, (void*)&bwg, (void*)&ec, (void*)&gc, (void*)&pr};
    GG_HIP(hipLaunchCooperativeKernel((const void*)k_tree_grid, dim3(tg_G), dim3(kTgThreads), args, (unsigned)tg_lds, s));
  } else if (pool)
    hipLaunchKernelGGL(k_tree_pool, dim3(1), dim3(kTpThreads), tp_lds_bytes(P.tiles, tp_gcap, tp_ecap), s, D, IO, n, nb,
                       TB, hcap, tp_gcap, tp_ecap, S->prof);
  else if (lds)
    hipLaunchKernelGGL(k_tree_walk<true>, dim3(1), dim3(64), hcap * sizeof(TEv), s, D, IO, n, nb, nullptr, hcap);
  else
    hipLaunchKernelGGL(k_tree_walk<false>, dim3(1), dim3(64), 0, s, D, IO, n, nb, S->theap, hcap);
  GG_HIP(hipGetLastError());
  gg_timer_end(ctx, "noc_tree", s);
  if (S->prof && gridf) {
    unsigned long long h[16];
    GG_HIP(hipMemcpyAsync(h, S->prof + 16, sizeof(h), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    fprintf(stderr, "[gg_noc tree] k_tree_grid %u blocks x %u routers, ecap %u: windows %llu | block 0 cycles: setup+injection "
            "%llu barrier %llu inbox+due %llu router sort %llu port tasks %llu forward %llu | busiest block: work %llu, "
            "least barrier wait %llu | block 0 barrier: store wait %llu poll %llu (%llu polls)\n", tg_G, tg_R, tg_ecap, h[6], h[0],
            h[1], h[2], h[3], h[4], h[5], h[8], h[9], h[10], h[11], h[12]);
    GG_HIP(hipMemsetAsync(S->prof + 16, 0, sizeof(h), s));
    GG_HIP(hipMemsetAsync(S->prof + 25, 0xFF, 8, s));
  }
  if (S->prof && pool) {
    unsigned long long h[16];
    GG_HIP(hipMemcpyAsync(h, S->prof, sizeof(h), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    fprintf(stderr, "[gg_noc tree] k_tree_pool gcap %u ecap %u: windows %llu pending %llu | cycles: setup+injection %llu "
            "min %llu due %llu router sort %llu port tasks %llu forward %llu\n", tp_gcap, tp_ecap, h[6], h[7], h[0],
            h[1], h[2], h[3], h[4], h[5]);
    GG_HIP(hipMemsetAsync(S->prof, 0, sizeof(h), s));
  }
  return GG_OK;
}

// The hop-by-hop stage pipeline over up to `cap` packets; the packet count is
// `cap` or, when n_dev is given, *n_dev read on the device (the coherent path
// launches whole batches of steps without a host sync).  Arrival / zero-load /
// contention land in the NoC state's packet arrays (gg_noc_packet_times).
gg_status gg_noc_hbh(gg_ctx* ctx, const uint32_t* src, const uint32_t* dst, const uint32_t* len, const uint64_t* t0,
                     const uint64_t* khi, const uint64_t* klo, uint64_t cap, const uint32_t* n_dev, hipStream_t s)
{
  gg_noc_state* S = ctx->noc;
  const NocParams& P = S->P;
  if (P.net_model != GG_NET_EMESH_HOP_BY_HOP) return gg_fail(GG_ERR_UNSUPPORTED, "network model %u", P.net_model);
  if (P.w * P.h != P.tiles) return gg_fail(GG_ERR_UNSUPPORTED, "emesh_hop_by_hop needs a full W x H mesh (hop_by_hop.cc:55-59)");
  if (cap >= (1ull << 32)) return gg_fail(GG_ERR_RANGE, "batch larger than 2^32 packets");
  const uint32_t nb_max = std::max(P.tiles, 2 * std::max(P.w, P.h));
  if (gg_status st = noc_grow(S, cap, nb_max)) return st;
  NocDev D{P, S->q, S->nd, S->ctr, ctx->err_dev};
  PktState PS{S->t, S->zl, S->ct, S->cur, khi, klo};
  const uint32_t blocks = (uint32_t)((cap + 255) / 256);
  gg_timer_begin(ctx, "noc_hop_by_hop", s);
  hipLaunchKernelGGL(k_init_pkts, dim3(blocks), dim3(256), 0, s, src, t0, cap, n_dev, PS);
  for (int stage = 0; stage < 4; ++stage) {
    const uint32_t nb = (stage == 0 || stage == 3) ? P.tiles : (stage == 1 ? 2 * P.h : 2 * P.w);
    GG_HIP(hipMemsetAsync(S->counts, 0, 4 * (nb + 1), s));
    hipLaunchKernelGGL(k_keys, dim3(blocks), dim3(256), 0, s, P, stage, src, dst, cap, n_dev, S->keys,
                       S->counts, ctx->err_dev);
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, S->counts, nb, S->off, S->cursor);
    hipLaunchKernelGGL(k_bucket, dim3(blocks), dim3(256), 0, s, S->keys, cap, n_dev, S->off, S->cursor, S->ids);
    const uint32_t tb = (nb + 63) / 64;
    const size_t qb = qimg_bytes(P.max_size);
    // chains: the general walk (chain_staged, the fallback of the pipeline and the sweep) stages the
    // chain's queue images in LDS
    const size_t chain_lds = (stage == 1 ? P.w : P.h) * qb;
    const bool staged = chain_lds <= kStageLdsMax;
    if (stage == 0 || stage == 3) {
      const uint32_t pb = (P.tiles + kPortWaves - 1) / kPortWaves;
      if (stage == 0)
        hipLaunchKernelGGL(k_port_sweep<false>, dim3(pb), dim3(64 * kPortWaves), kPortLds, s, D, len, S->off, S->ids,
                           S->heap, PS);
      else
        hipLaunchKernelGGL(k_port_sweep<true>, dim3(pb), dim3(64 * kPortWaves), kPortLds, s, D, len, S->off, S->ids,
                           S->heap, PS);
    } else if (staged && std::max(P.w, P.h) <= kPipePos) {
      const uint64_t stride = 3ull * std::max(P.w, P.h);
      if (S->pscr_cap < cap * stride) {
        if (S->pscr) hipFree(S->pscr);
        S->pscr = nullptr; S->pscr_cap = 0;
        GG_HIP(hipMalloc((void**)&S->pscr, sizeof(SK) * cap * stride));
        S->pscr_cap = cap * stride;
      }
      hipLaunchKernelGGL(k_chain_pipe, dim3(nb), dim3(64 * kPipeWaves), kStageLdsMax, s, D, stage - 1, dst, len, S->off,
                         S->ids, S->heap, PS, S->pscr, stride, S->prof);
    } else if (staged) {
      hipLaunchKernelGGL(k_chain_sweep, dim3(nb), dim3(kSweepThreads), kStageLdsMax, s, D, stage - 1, dst, len, S->off,
                         S->ids, S->heap, PS, S->prof);
    } else {
      hipLaunchKernelGGL(k_chain, dim3(tb), dim3(64), 0, s, D, stage - 1, src, dst, len, S->off, S->ids, S->heap,
                         PS, nb);
    }
    GG_HIP(hipGetLastError());
  }
  gg_timer_end(ctx, "noc_hop_by_hop", s);
  if (S->prof) {
    unsigned long long h[16];
    GG_HIP(hipMemcpyAsync(h, S->prof, sizeof(h), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    for (int st = 0; st < 2; ++st)
      fprintf(stderr, "[gg_noc sweep %c] chains %llu requests %llu | cycles summed over chains: setup %llu sort %llu "
              "serve %llu hand-off %llu | slowest chain %llu\n", st ? 'Y' : 'X', h[8 * st + 5], h[8 * st + 4],
              h[8 * st + 0], h[8 * st + 1], h[8 * st + 2], h[8 * st + 3], h[8 * st + 6]);
    GG_HIP(hipMemsetAsync(S->prof, 0, sizeof(h), s));
  }
  return GG_OK;
}

const uint64_t* gg_noc_packet_times(gg_ctx* ctx) { return ctx->noc->t; }

gg_status gg_noc_counters(gg_ctx* ctx, uint64_t* out)
{
  gg_noc_state* S = ctx->noc;
  if (S->P.net_model == GG_NET_EMESH_HOP_BY_HOP && S->P.qm) {
    hipLaunchKernelGGL(k_analytical, dim3((S->P.tiles + 63) / 64), dim3(64), 0, ctx->last_stream, S->q, S->P.tiles, S->ctr);
    GG_HIP(hipGetLastError());
    GG_HIP(hipStreamSynchronize(ctx->last_stream));
  }
  GG_HIP(hipMemcpy(out, S->ctr, sizeof(uint64_t) * S->P.tiles * GG_NUM_NET_COUNTERS, hipMemcpyDeviceToHost));
  return GG_OK;
}

gg_status gg_htree_run(gg_ctx* ctx, uint64_t min_proc, const uint64_t* t, const uint64_t* p, uint64_t n, uint64_t* d)
{
  gg_noc_state* S = ctx->noc;
  hipStream_t s = ctx->last_stream;
  const uint64_t qi = (uint64_t)S->P.tiles * 6;   // the stand-alone queue
  hipLaunchKernelGGL(k_htree_reset, dim3(1), dim3(1), 0, s, S->q + qi, S->nd + qi * S->P.max_size,
                     1ull, S->P.max_size, S->P.qtype, S->P.qaux);
  uint64_t* buf = nullptr;
  GG_HIP(hipMalloc((void**)&buf, 24 * (n ? n : 1)));
  GG_HIP(hipMemcpyAsync(buf, t, 8 * n, hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(buf + n, p, 8 * n, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_htree_seq, dim3(1), dim3(64), 0, s, S->q + qi, S->nd + qi * S->P.max_size,
                     min_proc, S->P.analytical, buf, buf + n, n, buf + 2 * n, ctx->err_dev);
  GG_HIP(hipGetLastError());
  GG_HIP(hipMemcpyAsync(d, buf + 2 * n, 8 * n, hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  hipFree(buf);
  return GG_OK;
}

gg::NocParams gg_noc_params(gg_ctx* ctx) { return ctx->noc->P; }
void gg_noc_queues(gg_ctx* ctx, gg::HQueue** q, gg::HNode** nd) { *q = ctx->noc->q; *nd = ctx->noc->nd; }
uint64_t* gg_noc_ctr(gg_ctx* ctx) { return ctx->noc->ctr; }
