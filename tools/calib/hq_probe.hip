// Cycles per history-tree request on one wave (queue in LDS / registers), by
// stream shape: in order; contention (bursts closer than the service time,
// queued at the tail); lagging senders (30 % of requests 40..4000 cycles
// back).  Variants: delay_w (LDS image), RegQueue.
#include "gg_dev.h"
#include <cstdio>
using namespace gg;

__device__ __forceinline__ uint64_t next_t(int shape, uint64_t& base, uint32_t& x)
{
  x = x * 1664525u + 1013904223u;
  const uint32_t r = x >> 8;
  if (shape == 0) { base += 3 + (r & 7); return base; }
  if (shape == 1) { base += (r & 3); return base; }
  base += (r & 7);
  return (r % 10 < 3 && base > 5000) ? base - 40 - (r % 3960) : base;
}

__global__ void __launch_bounds__(64) k(int variant, int shape, int n, uint64_t* out, uint32_t* err)
{
  __shared__ __attribute__((aligned(16))) uint8_t img[sizeof(HQueue) + 128 * sizeof(HNode)];
  const uint32_t ln = threadIdx.x;
  HQueue* q = reinterpret_cast<HQueue*>(img);
  HNode* nd = reinterpret_cast<HNode*>(img + sizeof(HQueue));
  if (ln == 0) hq_init(q, nd, 100, GG_QM_HISTORY_TREE, 0);
  __syncthreads();
  HTree tr{q, nd, 1, true};
  RegQueue rq;
  rq.load(q, nd, 1, true, ln);
  uint64_t acc = 0, base = 1000, tsum = 0;
  uint32_t x = 12345;
  for (int i = 0; i < n; ++i) {
    const uint64_t tt = next_t(shape, base, x);
    const uint64_t p = 5 + (x & 3);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    if (variant == 0) acc += tr.delay_w(tt, p, err, ln);
    else acc += rq.request(tt, p, err);
    tsum += __builtin_amdgcn_s_memtime() - c0;
  }
  if (ln == 0) { out[0] = tsum; out[1] = acc; out[2] = rq.n_fast; out[3] = rq.n_anl; out[4] = rq.n_gen; }
}

int main()
{
  uint64_t* o; uint32_t* e;
  (void)hipMalloc(&o, 64); (void)hipMalloc(&e, 4);
  const char* vn[] = {"delay_w", "RegQueue"};
  const char* sn[] = {"in order", "contention", "lagging"};
  for (int sh = 0; sh < 3; ++sh)
    for (int v = 0; v < 2; ++v) {
      const int n = 20000;
      k<<<1, 64>>>(v, sh, n, o, e);
      (void)hipDeviceSynchronize();
      uint64_t h[5]; (void)hipMemcpy(h, o, 40, hipMemcpyDeviceToHost);
      printf("{\"stream\": \"%s\", \"variant\": \"%s\", \"cycles_per_req\": %.1f, \"fast\": %llu, \"mg1\": %llu, \"search\": %llu}\n",
             sn[sh], vn[v], (double)h[0] / n, (unsigned long long)h[2], (unsigned long long)h[3], (unsigned long long)h[4]);
    }
  return 0;
}
