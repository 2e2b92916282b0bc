// Multi-line accesses of the coherent mode:
// Core::initiateMemoryAccess (common/tile/core/core.cc:139-266) splits an
// access [addr, addr + size) into line accesses, runs them back to back (each
// starts at the previous one's completion, sync delay 0 in one DVFS domain,
// core.cc:233) and reports latency = final - initial time and the number of
// lines that missed the L1-D (l1_cache_cntlr.cc:100-179 returns the hit flag).
//
// gg_split_accesses turns a tile-major access trace into line records (later
// lines carry GG_META_CONT: the coherent step issues them without a barrier
// check, the access being one instruction); gg_combine_accesses folds the
// per-line result words back into per-access {latency, misses}.  Both are
// plain data-parallel passes: one thread per access, a two-level exclusive
// scan of the line counts in between.
#include "gg_internal.h"

namespace {

constexpr uint32_t kScanBlock = 1024;

__device__ __forceinline__ uint64_t lines_of(uint64_t addr, uint32_t size, uint32_t line)
{
  if (size == 0) return 0;                                          // core.cc:145-155
  const uint64_t end = addr + size;
  const uint64_t ba = addr - addr % line, ea = end - end % line;
  return (ea - ba) / line + (end % line ? 1 : 0);                   // the zero-size tail line is skipped (:190-197)
}

// first index of the tile holding access i (tile_offsets ascending, [tiles + 1])
__device__ __forceinline__ uint64_t tile_start(const uint64_t* off, uint32_t tiles, uint64_t i)
{
  uint32_t lo = 0, hi = tiles;                                      // largest t with off[t] <= i
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (off[mid] <= i) lo = mid; else hi = mid;
  }
  return off[lo];
}

__global__ void __launch_bounds__(kScanBlock) k_split_count(const uint64_t* addr, const uint32_t* size, uint64_t n,
                                                            uint32_t line, uint64_t* cnt, uint64_t* bsum)
{
  __shared__ uint64_t part[kScanBlock / 64];
  const uint64_t i = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x;
  const uint64_t c = i < n ? lines_of(addr[i], size[i], line) : 0;
  if (i < n) cnt[i] = c;
  uint64_t v = c;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x / 64] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
    for (uint32_t w = 0; w < kScanBlock / 64; ++w) s += part[w];
    bsum[blockIdx.x] = s;
  }
}

// exclusive scan of the block sums (one workgroup; nb <= a few million)
__global__ void __launch_bounds__(kScanBlock) k_scan_blocks(uint64_t* bsum, uint64_t nb, uint64_t* total)
{
  __shared__ uint64_t carry;
  __shared__ uint64_t wsum[kScanBlock / 64];
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const uint32_t ln = threadIdx.x & 63, w = threadIdx.x / 64;
  for (uint64_t base = 0; base < nb; base += kScanBlock) {
    const uint64_t i = base + threadIdx.x;
    const uint64_t x = i < nb ? bsum[i] : 0;
    uint64_t v = x;                                                 // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(v, d);
      if (ln >= (uint32_t)d) v += y;
    }
    if (ln == 63) wsum[w] = v;
    __syncthreads();
    uint64_t before = carry;
    for (uint32_t k = 0; k < w; ++k) before += wsum[k];
    if (i < nb) bsum[i] = before + v - x;
    __syncthreads();
    if (threadIdx.x == kScanBlock - 1) carry = before + v;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// first[i] = exclusive scan of cnt; then (when the lines are wanted) write them
__global__ void __launch_bounds__(kScanBlock) k_split_write(const uint64_t* addr, const uint32_t* size,
                                                            const uint32_t* meta, uint64_t n, uint32_t line,
                                                            const uint64_t* cnt, const uint64_t* bsum,
                                                            const uint64_t* toff, uint32_t tiles, uint64_t* first,
                                                            uint64_t* laddr, uint32_t* lmeta, uint64_t cap,
                                                            uint32_t* err)
{
  __shared__ uint64_t wsum[kScanBlock / 64];
  const uint64_t i = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x;
  const uint32_t ln = threadIdx.x & 63, w = threadIdx.x / 64;
  const uint64_t x = i < n ? cnt[i] : 0;
  uint64_t v = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(v, d);
    if (ln >= (uint32_t)d) v += y;
  }
  if (ln == 63) wsum[w] = v;
  __syncthreads();
  uint64_t before = bsum[blockIdx.x];
  for (uint32_t k = 0; k < w; ++k) before += wsum[k];
  const uint64_t f = before + v - x;
  if (i >= n) return;
  if (meta[i] == GG_META_BARRIER) { atomicOr(err, GG_DERR_BARRIER); return; }   // not an access: insert after the split
  first[i] = f;
  if (i == n - 1) first[n] = f + x;
  if (!laddr || x == 0) return;
  // the gap cycles of the zero-size accesses right before this one (same tile)
  uint64_t gap = (meta[i] & 0x7FFFFFFFu) >> 1;
  const uint64_t t0 = tile_start(toff, tiles, i);
  for (uint64_t j = i; j > t0 && size[j - 1] == 0; --j) gap += (meta[j - 1] & 0x7FFFFFFFu) >> 1;
  if (gap >= (1ull << 30)) { atomicOr(err, GG_DERR_RANGE); return; }   // (a BARRIER before it is flagged by its own thread)
  const uint64_t ba = addr[i] - addr[i] % line;
  const uint32_t wr = meta[i] & GG_META_WRITE;
  for (uint64_t k = 0; k < x && f + k < cap; ++k) {
    laddr[f + k] = ba + k * line;
    lmeta[f + k] = k == 0 ? (wr | ((uint32_t)gap << 1)) : (wr | GG_META_CONT);
  }
}

__global__ void k_combine(const uint64_t* lout, const uint64_t* first, uint64_t n, uint64_t* lat, uint32_t* miss)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t l = 0;
  uint32_t m = 0;
  for (uint64_t k = first[i]; k < first[i + 1]; ++k) {
    const uint64_t wv = lout[k];
    l += wv >> 2;
    m += (uint32_t)((wv & 3u) != GG_LVL_L1);
  }
  if (lat) lat[i] = l;
  if (miss) miss[i] = m;
}

}  // namespace

extern "C" {

gg_status gg_split_accesses(const uint64_t* addr_dev, const uint32_t* size_dev, const uint32_t* meta_dev,
                            const uint64_t* tile_offsets, uint32_t tiles, uint32_t line_size, uint64_t* first_dev,
                            uint64_t* line_addr_dev, uint32_t* line_meta_dev, uint64_t cap, uint64_t* num_lines,
                            uint64_t* line_tile_offsets, void* stream)
{
  if (!tile_offsets || !num_lines || !first_dev || line_size == 0 || (line_size & (line_size - 1)) ||
      (tiles && tile_offsets[0] != 0) || (!!line_addr_dev != !!line_meta_dev))
    return gg_fail(GG_ERR_INVALID, "gg_split_accesses: bad arguments");
  for (uint32_t t = 0; t < tiles; ++t)
    if (tile_offsets[t + 1] < tile_offsets[t]) return gg_fail(GG_ERR_INVALID, "gg_split_accesses: tile offsets decrease");
  const uint64_t n = tiles ? tile_offsets[tiles] : 0;
  if (n && (!addr_dev || !size_dev || !meta_dev)) return gg_fail(GG_ERR_INVALID, "gg_split_accesses: NULL trace");
  hipStream_t s = (hipStream_t)stream;
  *num_lines = 0;
  if (n == 0) {
    GG_HIP(hipMemsetAsync(first_dev, 0, sizeof(uint64_t), s));
    if (line_tile_offsets) for (uint32_t t = 0; t <= tiles; ++t) line_tile_offsets[t] = 0;
    GG_HIP(hipStreamSynchronize(s));
    return GG_OK;
  }
  const uint64_t nb = (n + kScanBlock - 1) / kScanBlock;
  uint64_t *cnt = nullptr, *bsum = nullptr, *toff = nullptr, *total = nullptr;
  uint32_t* err = nullptr;
  gg_status st = GG_OK;
  auto run = [&]() -> gg_status {
    GG_HIP(hipMalloc((void**)&cnt, sizeof(uint64_t) * n));
    GG_HIP(hipMalloc((void**)&bsum, sizeof(uint64_t) * nb));
    GG_HIP(hipMalloc((void**)&toff, sizeof(uint64_t) * (tiles + 1)));
    GG_HIP(hipMalloc((void**)&total, sizeof(uint64_t)));
    GG_HIP(hipMalloc((void**)&err, sizeof(uint32_t)));
    GG_HIP(hipMemcpyAsync(toff, tile_offsets, sizeof(uint64_t) * (tiles + 1), hipMemcpyHostToDevice, s));
    GG_HIP(hipMemsetAsync(err, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_split_count, dim3((uint32_t)nb), dim3(kScanBlock), 0, s, addr_dev, size_dev, n, line_size, cnt, bsum);
    GG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kScanBlock), 0, s, bsum, nb, total);
    GG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_split_write, dim3((uint32_t)nb), dim3(kScanBlock), 0, s, addr_dev, size_dev, meta_dev, n,
                       line_size, cnt, bsum, toff, tiles, first_dev, line_addr_dev, line_meta_dev, cap, err);
    GG_HIP(hipGetLastError());
    uint32_t e = 0;
    GG_HIP(hipMemcpyAsync(num_lines, total, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    GG_HIP(hipMemcpyAsync(&e, err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (line_tile_offsets)
      for (uint32_t t = 0; t <= tiles; ++t)
        GG_HIP(hipMemcpyAsync(&line_tile_offsets[t], first_dev + tile_offsets[t], sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    if (e & GG_DERR_BARRIER)
      return gg_fail(GG_ERR_UNSUPPORTED, "gg_split_accesses: a BARRIER record in the access trace (insert barriers "
                     "into the line records after the split)");
    if (e) return gg_fail(GG_ERR_INVALID, "gg_split_accesses: carried gap above 2^30 cycles");
    if (line_addr_dev && *num_lines > cap)
      return gg_fail(GG_ERR_INVALID, "gg_split_accesses: %llu lines, capacity %llu", (unsigned long long)*num_lines,
                     (unsigned long long)cap);
    return GG_OK;
  };
  st = run();
  for (void* p : {(void*)cnt, (void*)bsum, (void*)toff, (void*)total, (void*)err}) if (p) hipFree(p);
  return st;
}

gg_status gg_combine_accesses(const uint64_t* line_out_dev, const uint64_t* first_dev, uint64_t n,
                              uint64_t* latency_ps_dev, uint32_t* misses_dev, void* stream)
{
  if (n && (!line_out_dev || !first_dev)) return gg_fail(GG_ERR_INVALID, "gg_combine_accesses: NULL arguments");
  if (!n) return GG_OK;
  hipLaunchKernelGGL(k_combine, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, line_out_dev,
                     first_dev, n, latency_ps_dev, misses_dev);
  GG_HIP(hipGetLastError());
  return GG_OK;
}

}  // extern "C"
