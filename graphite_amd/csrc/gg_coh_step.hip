// gg_coh_step.hip — the coherent step kernel k_c_step (one wave per owned
// tile) and its host launcher.  Device code: gg_coh_dev.h.
#include "gg_coh_dev.h"

namespace ggc {

__global__ void __launch_bounds__(64) k_c_step(CP P, CS S, uint32_t L, uint32_t devloop, uint64_t barrier_arg)
{
  diag_off(S);
  kt_begin(S);
  const uint64_t r0 = S.trs ? __builtin_amdgcn_s_memrealtime() : 0;
  TraceWin W{~0ull, 0, 0};
  step_body<false, false>(P, S, L, devloop, barrier_arg, W);
  if (S.trs && L < S.tr_n && threadIdx.x == 0) {
    unsigned long long* r = S.trs + ((size_t)L * P.L + blockIdx.x) * kTrStep;
    r[0] = r0; r[1] = __builtin_amdgcn_s_memrealtime();
  }
  kt_end(S);
}


void launch_step(const CP& P, const CS& S, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier)
{
  hipLaunchKernelGGL(k_c_step, dim3(P.L), dim3(64), lds, s, P, S, L, devloop, barrier);
}
hipError_t step_set_lds(size_t step_lds, size_t persist_lc_lds, size_t persist_lds)
{
  hipError_t e = hipFuncSetAttribute((const void*)k_c_step, hipFuncAttributeMaxDynamicSharedMemorySize, (int)step_lds);
  if (e == hipSuccess) e = persist_set_lds(persist_lc_lds, persist_lds);
  return e;
}

}  // namespace ggc
