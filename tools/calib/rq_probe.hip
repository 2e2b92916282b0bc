// RegQueue (gg_dev.h) vs a candidate rewrite (RQ2 below): request-by-request
// equality (delays + written-back image) and ns per request on one wave, by
// stream shape.  Tools only, not part of the product.
#include "gg_dev.h"
#include <cstdio>
using namespace gg;

template <int PRED> __device__ __forceinline__ uint64_t cmpl(uint64_t a, uint64_t b) { return __builtin_amdgcn_uicmpl(a, b, PRED); }
constexpr int kULE = 37, kUGE = 35;
__device__ __forceinline__ uint64_t lowbits(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }

struct RQ2 : RegQueue {
  __device__ __forceinline__ uint64_t A2(uint32_t i) const { const uint32_t l = i & 63; const uint64_t u = rl64(a0, l), v = rl64(a1, l); return i < 64 ? u : v; }
  __device__ __forceinline__ uint64_t B2(uint32_t i) const { const uint32_t l = i & 63; const uint64_t u = rl64(b0, l), v = rl64(b1, l); return i < 64 ? u : v; }
  __device__ __forceinline__ uint64_t request2(uint64_t t, uint64_t p, uint32_t* err)
  {
    errp = err;
    if (sz >= cap) { shift_down(0); --sz; }
    uint64_t qd = 0;
    const uint64_t tp = t + p;
    const uint64_t v0 = lowbits(sz), v1 = sz > 64 ? lowbits(sz - 64) : 0ull;
    const uint64_t la = A2(sz - 1), lb = B2(sz - 1);
    if (la <= t && tp <= lb && lb - tp >= min_proc) {                // the last interval: no search, no delay
      ++n_fast;
      if (t - la >= min_proc) { set(sz - 1, la, t); set(sz, tp, lb); ++sz; }
      else set(sz - 1, tp, lb);
    } else if (sz >= 2 && t < la && t >= A2(sz - 2)) {
      // the tail (as RegQueue): interval sz-2 is the last one starting at or before t
      ++n_fast;
      const uint32_t i2 = sz - 2, i1 = sz - 1;
      const uint64_t a2 = A2(i2), b2 = B2(i2);
      if (tp <= b2) {
        if (t - a2 >= min_proc) {
          if (b2 - tp >= min_proc) { set(i1 + 1, la, lb); set(i1, tp, b2); ++sz; }
          set(i2, a2, t);
        } else if (b2 - tp >= min_proc) {
          set(i2, tp, b2);
        } else {
          set(i2, la, lb); --sz;
        }
      } else {
        qd = la - t;
        if (lb - (la + p) >= min_proc) set(i1, la + p, lb);
        else --sz;
      }
    } else if (analytical && A2(0) > tp) {
      ++anl; ++n_anl;
      qd = mg1_queue_delay(nreq, newest, sig_sq, sig);
    } else {
      ++n_gen;
      // fit: a <= t && t + p <= b (at most one: the last interval starting at or before t);
      // later: a > t && b - a >= p (the first)
      const uint64_t le0 = cmpl<kULE>(a0, t) & v0, le1 = cmpl<kULE>(a1, t) & v1;
      const uint64_t f0 = le0 & cmpl<kUGE>(b0, tp), f1 = le1 & cmpl<kUGE>(b1, tp);
      const uint64_t l0 = ~le0 & v0 & cmpl<kUGE>(b0 - a0, p), l1 = ~le1 & v1 & cmpl<kUGE>(b1 - a1, p);
      const bool fit = (f0 | f1) != 0;
      const uint64_t m0 = fit ? f0 : l0, m1 = fit ? f1 : l1;
      if ((m0 | m1) == 0) { errs |= GG_DERR_STATE; }
      else {
        const uint32_t ui = m0 ? (uint32_t)__builtin_ctzll(m0) : 64u + (uint32_t)__builtin_ctzll(m1);
        const uint64_t a = A2(ui), b = B2(ui);
        if (fit) {
          if (t - a >= min_proc) {
            if (b - tp >= min_proc) { shift_up(ui + 1); set(ui + 1, tp, b); ++sz; }
            set(ui, a, t);
          } else if (b - tp >= min_proc) {
            set(ui, tp, b);
          } else { shift_down(ui); --sz; }
        } else {
          qd = a - t;
          if (b - (a + p) >= min_proc) set(ui, a + p, b);
          else { shift_down(ui); --sz; }
        }
      }
    }
    sig_sq += p * p; sig += p;
    if (sig_sq >= kMg1Exact || p >= (1ull << 26)) errs |= GG_DERR_RANGE;
    ++nreq;
    const uint64_t x = t + qd + p;
    newest = x > newest ? x : newest;
    util += p;
    last_req = x > last_req ? x : last_req;
    ++total_req;
    return qd;
  }
};

__device__ __forceinline__ uint64_t next_t(int shape, uint64_t& base, uint32_t& x, uint64_t& p)
{
  x = x * 1664525u + 1013904223u;
  const uint32_t r = x >> 8;
  p = (r >> 20) & 1 ? 10 : 2;
  if (shape == 0) { base += 3 + (r & 7); return base; }
  if (shape == 1) { base += 3; return base + 5000 - (r % 1500); }
  base += 20; return base + 5000 - (r % 1000);
}
constexpr int kN = 20000;

template <int V>
__global__ void __launch_bounds__(64) k_time(int shape, uint64_t* out, uint32_t* err)
{
  __shared__ __attribute__((aligned(16))) uint8_t img[sizeof(HQueue) + 128 * sizeof(HNode)];
  const uint32_t ln = threadIdx.x;
  HQueue* q = reinterpret_cast<HQueue*>(img);
  HNode* nd = reinterpret_cast<HNode*>(img + sizeof(HQueue));
  if (ln == 0) hq_init(q, nd, 100, GG_QM_HISTORY_TREE, 0);
  __syncthreads();
  RQ2 rq;
  rq.load(q, nd, 1, true, ln);
  uint64_t acc = 0, base = 1000;
  uint32_t x = 12345;
  for (int i = 0; i < kN; ++i) {
    uint64_t p;
    const uint64_t tt = next_t(shape, base, x, p);
    acc += V == 0 ? rq.request(tt, p, err) : (V == 1 ? rq.request2(tt, p, err) : rq.request<false>(tt, p, err));
  }
  if (ln == 0) out[0] = acc;
}

__global__ void __launch_bounds__(64) k_check(int shape, uint64_t* out, uint32_t* err)
{
  __shared__ __attribute__((aligned(16))) uint8_t i1[sizeof(HQueue) + 128 * sizeof(HNode)];
  __shared__ __attribute__((aligned(16))) uint8_t i2[sizeof(HQueue) + 128 * sizeof(HNode)];
  const uint32_t ln = threadIdx.x;
  HQueue* q1 = reinterpret_cast<HQueue*>(i1); HNode* n1 = reinterpret_cast<HNode*>(i1 + sizeof(HQueue));
  HQueue* q2 = reinterpret_cast<HQueue*>(i2); HNode* n2 = reinterpret_cast<HNode*>(i2 + sizeof(HQueue));
  if (ln == 0) { hq_init(q1, n1, 100, GG_QM_HISTORY_TREE, 0); hq_init(q2, n2, 100, GG_QM_HISTORY_TREE, 0); }
  __syncthreads();
  RQ2 a, b;
  a.load(q1, n1, 1, true, ln); b.load(q2, n2, 1, true, ln);
  uint64_t base = 1000, bad = 0;
  int64_t first = -1;
  uint32_t x = 777;
  for (int i = 0; i < kN; ++i) {
    uint64_t p;
    const uint64_t tt = next_t(shape, base, x, p);
    if (a.request<false>(tt, p, err) != b.request2(tt, p, err)) { ++bad; if (first < 0) first = i; }
    if (i % 997 == 0 || i == kN - 1) {
      a.store(q1, n1); b.store(q2, n2);
      __syncthreads();
      uint32_t diff = 0;
      const uint32_t words = (uint32_t)(sizeof(HQueue) + q1->size * sizeof(HNode)) / 4;
      for (uint32_t w = ln; w < words; w += 64) diff |= reinterpret_cast<uint32_t*>(i1)[w] != reinterpret_cast<uint32_t*>(i2)[w];
      if (__ballot(diff)) { ++bad; if (first < 0) first = i; }
      __syncthreads();
      a.load(q1, n1, 1, true, ln); b.load(q2, n2, 1, true, ln);
    }
  }
  if (ln == 0) { out[0] = bad; out[1] = (uint64_t)first; }
}

int main()
{
  uint64_t* o; uint32_t* e;
  (void)hipMalloc(&o, 64); (void)hipMalloc(&e, 4); (void)hipMemset(e, 0, 4);
  const char* sn[] = {"in order", "spread 1500", "walker-like"};
  for (int sh = 0; sh < 3; ++sh) {
    uint64_t h[2];
    k_check<<<1, 64>>>(sh, o, e);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, o, 16, hipMemcpyDeviceToHost);
    float ms[3];
    for (int v = 0; v < 3; ++v) {
      hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      if (v == 0) k_time<0><<<1, 64>>>(sh, o, e); else if (v == 1) k_time<1><<<1, 64>>>(sh, o, e); else k_time<2><<<1, 64>>>(sh, o, e);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      if (v == 0) k_time<0><<<1, 64>>>(sh, o, e); else if (v == 1) k_time<1><<<1, 64>>>(sh, o, e); else k_time<2><<<1, 64>>>(sh, o, e);
      (void)hipEventRecord(e1);
      (void)hipDeviceSynchronize();
      (void)hipEventElapsedTime(&ms[v], e0, e1);
    }
    printf("{\"stream\": \"%s\", \"mismatches\": %llu, \"first\": %lld, \"request_ns\": %.1f, \"probe_rq_ns\": %.1f, \"request_notail_ns\": %.1f}\n", sn[sh],
           (unsigned long long)h[0], (long long)h[1], ms[0] * 1e6 / kN, ms[1] * 1e6 / kN, ms[2] * 1e6 / kN);
  }
  return 0;
}
