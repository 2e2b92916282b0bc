// Dependent global-load latency inside a 1024-workgroup launch, reading
// records that the previous launch wrote (the walker -> step hand-off
// pattern): list word, then the 64-B record it names.  Tools only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct Rec { uint64_t w[8]; };

__global__ void __launch_bounds__(64) k_write(Rec* pool, uint32_t* list, uint32_t npool, uint32_t salt)
{
  const uint32_t b = blockIdx.x, ln = threadIdx.x;
  if (ln < 16) {
    uint32_t h = (b * 16 + ln) * 2654435761u ^ salt;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    const uint32_t r = h % npool;
    pool[r].w[0] = b; pool[r].w[1] = ln;
    list[b * 256 + ln] = r;
  }
}

__device__ __forceinline__ uint64_t now_after_loads()
{
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  return __builtin_amdgcn_s_memtime();
}

__global__ void __launch_bounds__(64) k_read(const Rec* pool, const uint32_t* list, unsigned long long* st)
{
  const uint32_t b = blockIdx.x, ln = threadIdx.x;
  const uint64_t t0 = now_after_loads();
  uint32_t r = ln < 16 ? list[b * 256 + ln] : 0;
  const uint64_t t1 = now_after_loads();
  uint64_t v = ln < 16 ? pool[r].w[0] : 0;
  const uint64_t t2 = now_after_loads();
  uint64_t v2 = ln < 16 ? pool[(r + 7919) % 1048576].w[0] : 0;     // an unrelated line (not written)
  const uint64_t t3 = now_after_loads();
  if (ln == 0) {
    atomicAdd(&st[0], (unsigned long long)(t1 - t0)); atomicAdd(&st[1], (unsigned long long)(t2 - t1));
    atomicAdd(&st[2], (unsigned long long)(t3 - t2));
    atomicMax(&st[3], (unsigned long long)(t1 - t0)); atomicMax(&st[4], (unsigned long long)(t2 - t1));
    atomicAdd(&st[5], (unsigned long long)(v + v2 + r) & 1);
  }
}

int main()
{
  const uint32_t npool = 1 << 20;
  Rec* pool; uint32_t* list; unsigned long long* st;
  (void)hipMalloc(&pool, sizeof(Rec) * npool); (void)hipMalloc(&list, 1024 * 256 * 4); (void)hipMalloc(&st, 64);
  (void)hipMemset(pool, 0, sizeof(Rec) * npool); (void)hipMemset(list, 0, 1024 * 256 * 4);
  for (int rep = 0; rep < 4; ++rep) {
    unsigned long long h[6];
    (void)hipMemset(st, 0, 64);
    k_write<<<1024, 64>>>(pool, list, npool, 77u * rep);
    k_read<<<1024, 64>>>(pool, list, st);                 // right after the writer
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, st, 48, hipMemcpyDeviceToHost);
    printf("{\"case\": \"after writer\", \"list_word_cyc\": %.0f, \"record_cyc\": %.0f, \"unwritten_line_cyc\": %.0f, \"max_list\": %llu, \"max_rec\": %llu}\n",
           h[0] / 1024.0, h[1] / 1024.0, h[2] / 1024.0, h[3], h[4]);
    (void)hipMemset(st, 0, 64);
    k_read<<<1024, 64>>>(pool, list, st);                 // again (warm)
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, st, 48, hipMemcpyDeviceToHost);
    printf("{\"case\": \"second read\", \"list_word_cyc\": %.0f, \"record_cyc\": %.0f, \"unwritten_line_cyc\": %.0f, \"max_list\": %llu, \"max_rec\": %llu}\n",
           h[0] / 1024.0, h[1] / 1024.0, h[2] / 1024.0, h[3], h[4]);
  }
  return 0;
}
