// gg_coh_step_shl2.hip — k_c_step<false, 2> and <false, 3> (gg_coh_step.inc):
// the step kernels of the shared-L2 protocols (pr_l1_sh_l2_msi, Tile's PR =
// 2; pr_l1_sh_l2_mesi, PR = 3), and their launcher.  Like MOSI it runs on the per-step launches only (no
// persistent instance).
#include "gg_coh_dev.h"
namespace ggc {
#include "gg_coh_step.inc"
void launch_step_shl2(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier)
{
  if (P.mesi) hipLaunchKernelGGL((k_c_step<false, 3>), dim3(P.L), dim3(64), lds, s, a.P, a.S, L, devloop, barrier, a.kt, a.kt_slot);
  else hipLaunchKernelGGL((k_c_step<false, 2>), dim3(P.L), dim3(64), lds, s, a.P, a.S, L, devloop, barrier, a.kt, a.kt_slot);
}
hipError_t step_shl2_set_lds(size_t lds)
{
  hipError_t e = hipFuncSetAttribute((const void*)k_c_step<false, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_c_step<false, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return e;
}
}  // namespace ggc
