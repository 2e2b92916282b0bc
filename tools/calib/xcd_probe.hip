// Probe: does a block's working set stay in its XCD's L2 across kernel
// launches?  1024 blocks each chase a pointer list through a private 16 KB
// chunk.  Launch pairs: same block->chunk map twice; a rotated map (chunk of
// block b+1, another XCD under round-robin dealing); an XCC_ID-affine map
// (chunk claimed from the XCD's own counter).  Also reports whether the
// block -> XCC_ID assignment repeats across launches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <random>

constexpr int NB = 1024, W = 2048, STEPS = 512;

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u; }

__global__ void k_chase(const uint32_t* next, uint32_t* ctr, uint32_t* xcc_of_block, int mode, uint64_t* sink)
{
  if (threadIdx.x != 0) return;
  const uint32_t x = xcc_id();
  xcc_of_block[blockIdx.x] = x;
  uint32_t c;
  if (mode == 0) c = blockIdx.x;
  else if (mode == 1) c = (blockIdx.x + 1) % NB;
  else c = x * (NB / 8) + (atomicAdd(&ctr[x], 1u) % (NB / 8));
  const uint32_t* p = next + (size_t)c * W;
  uint32_t i = 0;
  for (int s = 0; s < STEPS; ++s) i = __builtin_nontemporal_load(p + i) & 0 ? 0 : p[i];
  sink[blockIdx.x] = i;
}

int main()
{
  std::vector<uint32_t> h((size_t)NB * W);
  std::mt19937 rng(1);
  for (int c = 0; c < NB; ++c) {
    std::vector<uint32_t> perm(W);
    for (int i = 0; i < W; ++i) perm[i] = i;
    std::shuffle(perm.begin() + 1, perm.end(), rng);
    for (int i = 0; i < W; ++i) h[(size_t)c * W + perm[i]] = perm[(i + 1) % W];
  }
  uint32_t *next, *ctr, *xb; uint64_t* sink;
  (void)hipMalloc(&next, h.size() * 4); (void)hipMalloc(&ctr, 64); (void)hipMalloc(&xb, NB * 4); (void)hipMalloc(&sink, NB * 8);
  (void)hipMemcpy(next, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  std::vector<uint32_t> x0(NB), x1(NB);
  auto run = [&](int mode, std::vector<uint32_t>* xs) {
    (void)hipMemset(ctr, 0, 64);
    (void)hipEventRecord(a);
    k_chase<<<NB, 64>>>(next, ctr, xb, mode, sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    if (xs) (void)hipMemcpy(xs->data(), xb, NB * 4, hipMemcpyDeviceToHost);
    return ms * 1e3f;
  };
  for (int rep = 0; rep < 3; ++rep) {
    run(0, &x0);
    const float same = run(0, &x1);
    int moved = 0; for (int i = 0; i < NB; ++i) moved += x0[i] != x1[i];
    run(0, nullptr);
    const float rot = run(1, nullptr);
    run(2, nullptr);
    const float aff = run(2, nullptr);
    printf("{\"same_map_us\": %.1f, \"rotated_map_us\": %.1f, \"xcc_affine_us\": %.1f, \"blocks_changing_xcc\": %d}\n", same, rot, aff, moved);
  }
  return 0;
}
