// gg_coh_step.hip — k_c_step<false> (gg_coh_step.inc: every queue form and
// the miss-type hooks) and the step launcher, which takes k_c_step<true>
// (gg_coh_step_fast.hip) when the configuration allows it (P.fast), and
// k_c_step<false, 1> (gg_coh_step_mosi.hip) for the MOSI protocol and
// k_c_step<false, 2> (gg_coh_step_shl2.hip) for the shared-L2 MSI protocol.
#include "gg_coh_dev.h"

namespace ggc {

#include "gg_coh_step.inc"

void launch_step(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier)
{
  if (P.mosi) launch_step_mosi(P, a, lds, s, L, devloop, barrier);
  else if (P.shl2) launch_step_shl2(P, a, lds, s, L, devloop, barrier);
  else if (P.fast) launch_step_fast(P, a, lds, s, L, devloop, barrier);
  else hipLaunchKernelGGL(k_c_step<false>, dim3(P.L), dim3(64), lds, s, a.P, a.S, L, devloop, barrier, a.kt, a.kt_slot);
}
hipError_t step_set_lds(size_t step_lds, size_t persist_lc_lds, size_t persist_lds)
{
  hipError_t e = hipFuncSetAttribute((const void*)k_c_step<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)step_lds);
  if (e == hipSuccess) e = step_fast_set_lds(step_lds);
  if (e == hipSuccess) e = step_mosi_set_lds(step_lds);
  if (e == hipSuccess) e = step_shl2_set_lds(step_lds);
  if (e == hipSuccess) e = persist_set_lds(persist_lc_lds, persist_lds);
  return e;
}

}  // namespace ggc
