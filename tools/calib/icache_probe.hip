// Cold instruction-fetch cost: one wave runs a long straight-line VALU/SALU
// sequence twice in one launch (first pass cold, second warm), after another
// kernel with a large body ran on the same CUs.  Cycles per pass, per 1k
// instructions.  Tools only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define OP1 "v_add_u32 %0, %0, 1\n s_add_u32 s0, s0, 1\n"
#define OP4 OP1 OP1 OP1 OP1
#define OP16 OP4 OP4 OP4 OP4
#define OP64 OP16 OP16 OP16 OP16
#define OP256 OP64 OP64 OP64 OP64
#define OP1K OP256 OP256 OP256 OP256

__device__ __forceinline__ uint64_t now()
{
  uint64_t t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}

__global__ void __launch_bounds__(64) k_body(uint32_t* out, int passes)
{
  uint32_t v = threadIdx.x;
  uint64_t t[4];
  t[0] = now();
  asm volatile(OP1K OP1K OP1K OP1K : "+v"(v) : : "s0");       // 4k VALU + 4k SALU = 8k instructions (~40 KB), cold
  t[1] = now();
  for (int p = 1; p < passes && p < 3; ++p) {                // the same code again (a second copy: the loop body)
    asm volatile(OP1K OP1K OP1K OP1K : "+v"(v) : : "s0");
    t[p + 1] = now();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = (uint32_t)(t[1] - t[0]); out[1] = (uint32_t)(t[2] - t[1]); out[2] = (uint32_t)(t[3] - t[2]);
  }
  if (v == 12345u) out[8] = v;
}

// a different large body, to evict the first from the instruction cache
__global__ void __launch_bounds__(64) k_evict(uint32_t* out)
{
  uint32_t v = threadIdx.x;
  asm volatile(OP1K OP1K OP1K OP1K OP1K OP1K OP1K OP1K : "+v"(v) : : "s0");
  if (v == 12345u) out[9] = v;
}

int main()
{
  uint32_t* o; uint32_t h[3];
  (void)hipMalloc(&o, 64);
  for (int rep = 0; rep < 3; ++rep) {
    k_evict<<<256, 64>>>(o);
    k_body<<<1, 64>>>(o, 3);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, o, 12, hipMemcpyDeviceToHost);
    printf("{\"rep\": %d, \"pass_cycles\": [%u, %u, %u], \"instructions_per_pass\": 8192}\n", rep, h[0], h[1], h[2]);
  }
  return 0;
}
