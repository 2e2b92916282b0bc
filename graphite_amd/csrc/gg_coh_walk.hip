// gg_coh_walk.hip — the hop-by-hop walker kernels k_c_walk<PIPE, RQ> (one
// workgroup per X / Y run) and their host launcher.  Device
// code: gg_coh_dev.h.
#include "gg_coh_dev.h"

namespace ggc {

template <bool PIPE, bool RQ>
__global__ void __launch_bounds__(PIPE ? 64 * kMaxWalkWaves : 64) k_c_walk(const CP* __restrict__ Pp, const CS* __restrict__ Sp, uint32_t L, int stage,
                                                                         unsigned long long* kt, uint32_t kt_slot)
{
  kwarm(Pp, Sp);
  const CP& P = *Pp;                 // the launch state read on use (see k_c_step)
  const CS& S = *Sp;
  if (kt && threadIdx.x == 0) kt[(size_t)kt_slot * S.kt_stride + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  if (DG(S.trs) && L < S.tr_n && threadIdx.x == 0)
    DG(S.trw)[(((size_t)L * 2 + stage) * S.tr_wb + blockIdx.x) * 8] = __builtin_amdgcn_s_memrealtime();
  walk_body<PIPE, RQ>(P, S, L, stage, blockIdx.x);
  if (kt) {
    __syncthreads();
    if (threadIdx.x == 0) kt[(size_t)kt_slot * S.kt_stride + 2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

void launch_walk(bool pipe, bool rq, uint32_t blocks, uint32_t threads, size_t lds, hipStream_t s, const StepArgs& a,
                 uint32_t L, int stage)
{
  if (pipe && rq) hipLaunchKernelGGL((k_c_walk<true, true>), dim3(blocks), dim3(threads), lds, s, a.P, a.S, L, stage, a.kt, a.kt_slot);
  else if (pipe) hipLaunchKernelGGL((k_c_walk<true, false>), dim3(blocks), dim3(threads), lds, s, a.P, a.S, L, stage, a.kt, a.kt_slot);
  else if (rq) hipLaunchKernelGGL((k_c_walk<false, true>), dim3(blocks), dim3(64), lds, s, a.P, a.S, L, stage, a.kt, a.kt_slot);
  else hipLaunchKernelGGL((k_c_walk<false, false>), dim3(blocks), dim3(64), lds, s, a.P, a.S, L, stage, a.kt, a.kt_slot);
}
hipError_t walk_set_lds(size_t lds)
{
  for (const void* f : {(const void*)k_c_walk<true, true>, (const void*)k_c_walk<true, false>,
                        (const void*)k_c_walk<false, true>, (const void*)k_c_walk<false, false>})
    if (hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) return e;
  return hipSuccess;
}

}  // namespace ggc
