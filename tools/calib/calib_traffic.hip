// calib_traffic.hip — calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access widths of k_cache_stream (MI355X_MICROARCH.md §HBM:
// "other access widths are uncalibrated").  Each kernel moves a known byte
// count once (buffers far larger than the 256 MiB Infinity Cache):
//   read4 / read8 / read16 : coalesced streaming loads of 4 / 8 / 16 B per lane
//   scatter4               : 4-B stores, each wave's 64 lanes to 64 different
//                            128-B lines, every dword written exactly once
//                            (the result-store pattern of k_cache_stream)
//   write16                : coalesced 16-B stores (reference: exact per the guide)
// usage: calib_traffic <MiB>   (prints the byte count of each kernel)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

template <class T>
__global__ void k_read(const T* __restrict__ p, size_t n, uint32_t* sink)
{
  T acc{};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = __builtin_nontemporal_load(p + i);
    acc ^= v;
  }
  if (acc == (T)0x1234567) atomicAdd(sink, 1u);
}

__global__ void k_read16(const uint4* __restrict__ p, size_t n, uint32_t* sink)
{
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x1234567u) atomicAdd(sink, 1u);
}

// Each workgroup (256 lanes) owns consecutive 8-KiB chunks (64 lines of 128 B);
// per store instruction the 64 lanes of a wave write 64 different lines, and
// the chunk's lines fill up within the workgroup (one CU, one XCD's L2) — the
// result-store pattern of k_cache_stream, whose tile region is written by one
// workgroup.
__global__ void k_scatter4(uint32_t* __restrict__ p, size_t n)
{
  const uint32_t t = threadIdx.x;
  for (size_t c = blockIdx.x; c < n / 2048; c += gridDim.x) {
#pragma unroll
    for (uint32_t r = 0; r < 8; ++r)
      p[c * 2048 + (t % 64) * 32 + (t / 64) * 8 + r] = t + r;
  }
}

__global__ void k_write16(uint4* __restrict__ p, size_t n)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main(int argc, char** argv)
{
  const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 2048;
  const size_t bytes = mib << 20;
  void* buf = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc((void**)&sink, 4) != hipSuccess) return 1;
  hipMemset(buf, 1, bytes);
  hipDeviceSynchronize();
  const dim3 g(256 * 16), b(256);
  hipLaunchKernelGGL(k_read<uint32_t>, g, b, 0, 0, (const uint32_t*)buf, bytes / 4, sink);
  hipLaunchKernelGGL(k_read<uint64_t>, g, b, 0, 0, (const uint64_t*)buf, bytes / 8, sink);
  hipLaunchKernelGGL(k_read16, g, b, 0, 0, (const uint4*)buf, bytes / 16, sink);
  hipLaunchKernelGGL(k_scatter4, g, b, 0, 0, (uint32_t*)buf, bytes / 4);
  hipLaunchKernelGGL(k_write16, g, b, 0, 0, (uint4*)buf, bytes / 16);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"bytes_per_kernel\": %zu}\n", bytes);
  hipFree(buf);
  hipFree(sink);
  return 0;
}
