// gg_coh_walk.hip — the hop-by-hop walker kernels k_c_walk<PIPE, RQ> (one
// workgroup per X / Y run) and their host launcher.  Device
// code: gg_coh_dev.h.
#include "gg_coh_dev.h"

namespace ggc {

template <bool PIPE, bool RQ>
__global__ void __launch_bounds__(PIPE ? 64 * kMaxWalkWaves : 64) k_c_walk(CP P, CS S, uint32_t L, int stage)
{
  diag_off(S);
  kt_begin(S);
  if (DG(S.trs) && L < S.tr_n && threadIdx.x == 0)
    DG(S.trw)[(((size_t)L * 2 + stage) * S.tr_wb + blockIdx.x) * 8] = __builtin_amdgcn_s_memrealtime();
  walk_body<PIPE, RQ>(P, S, L, stage, blockIdx.x);
  kt_end(S);
}

void launch_walk(bool pipe, bool rq, uint32_t blocks, uint32_t threads, size_t lds, hipStream_t s, const CP& P, const CS& S,
                 uint32_t L, int stage)
{
  if (pipe && rq) hipLaunchKernelGGL((k_c_walk<true, true>), dim3(blocks), dim3(threads), lds, s, P, S, L, stage);
  else if (pipe) hipLaunchKernelGGL((k_c_walk<true, false>), dim3(blocks), dim3(threads), lds, s, P, S, L, stage);
  else if (rq) hipLaunchKernelGGL((k_c_walk<false, true>), dim3(blocks), dim3(64), lds, s, P, S, L, stage);
  else hipLaunchKernelGGL((k_c_walk<false, false>), dim3(blocks), dim3(64), lds, s, P, S, L, stage);
}
hipError_t walk_set_lds(size_t lds)
{
  for (const void* f : {(const void*)k_c_walk<true, true>, (const void*)k_c_walk<true, false>,
                        (const void*)k_c_walk<false, true>, (const void*)k_c_walk<false, false>})
    if (hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) return e;
  return hipSuccess;
}

}  // namespace ggc
