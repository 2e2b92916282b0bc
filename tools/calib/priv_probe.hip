// Dependent-load latency of a tile's private state across launches (the
// step kernel's pattern: block b reads and writes its own lines every launch)
// and the cost of a load issued behind outstanding stores (vmcnt counts both
// on gfx9).  Tools only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint32_t kLines = 64;          // private lines per block (128 B apart)
constexpr uint32_t kStride = 16;         // u64 per line

__device__ __forceinline__ uint64_t now_after_loads()
{
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  return __builtin_amdgcn_s_memtime();
}

// every block links its lines into a chain: line i holds the index of line i+1
__global__ void __launch_bounds__(64) k_write(uint64_t* st, uint32_t salt)
{
  const uint32_t b = blockIdx.x, ln = threadIdx.x;
  uint64_t* my = st + (size_t)b * kLines * kStride;
  if (ln < kLines) my[ln * kStride] = (ln * 7 + 3 + salt) % kLines;
}

// mode 0: chain of 8 dependent loads over the block's own lines (written by
// the previous launch, same block index); mode 1: over block b+1's lines;
// mode 2: own lines, each load issued behind 8 stores to other own lines
__global__ void __launch_bounds__(64) k_read(uint64_t* st, int mode, unsigned long long* out)
{
  const uint32_t b = blockIdx.x, ln = threadIdx.x;
  const uint32_t src = mode == 1 ? (b + 1) % gridDim.x : b;
  uint64_t* my = st + (size_t)src * kLines * kStride;
  uint64_t* mine = st + (size_t)b * kLines * kStride;
  uint64_t i = 0;
  uint64_t t[9];
  t[0] = now_after_loads();
  for (int k = 0; k < 8; ++k) {
    if (mode == 2) {
      // the stores go to word 8 of lines (not the chain words)
      for (int s = 0; s < 8; ++s) mine[((k * 8 + s) % kLines) * kStride + 8] = k;
    }
    i = __shfl((long long)(ln == 0 ? *(volatile uint64_t*)&my[(i % kLines) * kStride] : 0), 0);
    t[k + 1] = now_after_loads();
  }
  if (ln == 0) {
    for (int k = 0; k < 8; ++k) atomicAdd(&out[k], (unsigned long long)(t[k + 1] - t[k]));
    atomicAdd(&out[8], (unsigned long long)(i & 1));
  }
}

int main()
{
  const uint32_t nb = 1024;
  uint64_t* st; unsigned long long* out;
  (void)hipMalloc(&st, sizeof(uint64_t) * nb * kLines * kStride); (void)hipMalloc(&out, 16 * 8);
  (void)hipMemset(st, 0, sizeof(uint64_t) * nb * kLines * kStride);
  const char* names[] = {"own lines, previous launch wrote", "neighbour block's lines", "own lines behind 8 stores"};
  for (int rep = 0; rep < 3; ++rep)
    for (int mode = 0; mode < 3; ++mode) {
      unsigned long long h[9];
      k_write<<<nb, 64>>>(st, rep);
      (void)hipMemset(out, 0, 16 * 8);
      k_read<<<nb, 64>>>(st, mode, out);
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(h, out, 72, hipMemcpyDeviceToHost);
      printf("{\"case\": \"%s\", \"rep\": %d, \"cycles_per_load\": [", names[mode], rep);
      for (int k = 0; k < 8; ++k) printf("%s%.0f", k ? ", " : "", h[k] / (double)nb);
      printf("]}\n");
    }
  // warm: the same launch twice (the second read after a reader, not a writer)
  {
    unsigned long long h[9];
    k_write<<<nb, 64>>>(st, 9);
    k_read<<<nb, 64>>>(st, 0, out);
    (void)hipMemset(out, 0, 16 * 8);
    k_read<<<nb, 64>>>(st, 0, out);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, out, 72, hipMemcpyDeviceToHost);
    printf("{\"case\": \"own lines, previous launch read them\", \"cycles_per_load\": [");
    for (int k = 0; k < 8; ++k) printf("%s%.0f", k ? ", " : "", h[k] / (double)nb);
    printf("]}\n");
  }
  return 0;
}
