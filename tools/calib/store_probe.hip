// Probe: cost of a "uniform" 8-B store made by all 64 lanes (same address,
// same value) vs by lane 0 only, in a dependent store -> load chain (one
// wave per workgroup, 1024 workgroups), and WRITE_SIZE under rocprofv3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(64) void k_chain(uint64_t* p, int n, int mode)
{
  uint64_t* q = p + blockIdx.x * 64;
  uint64_t v = threadIdx.x == 100;
  for (int i = 0; i < n; i++) {
    uint64_t w = v + i;
    if (mode == 0) q[i & 7] = w;                            // every lane, same address
    else if (mode == 1) { if (threadIdx.x == 0) q[i & 7] = w; }
    else if (mode == 3) q[(i & 7) * 0 + 8 + (threadIdx.x & 7)] = w;   // 8 distinct words
    asm volatile("" ::: "memory");
    v = __builtin_nontemporal_load(q + 16 + ((v + i) & 7)) ;    // dependent load
  }
  if (v == 12345) q[40] = v;
}

int main()
{
  uint64_t* p;
  hipMalloc(&p, 1024 * 64 * 8);
  hipMemset(p, 0, 1024 * 64 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"all-lane store", "lane-0 store", "no store", "8 distinct words"};
  for (int mode : {0, 1, 2, 3, 0, 1, 2, 3}) {
    hipEventRecord(a);
    k_chain<<<1024, 64>>>(p, 4096, mode);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"mode\": \"%s\", \"us\": %.1f, \"ns_per_iter\": %.1f}\n", names[mode], ms * 1e3, ms * 1e6 / 4096);
  }
  return 0;
}
