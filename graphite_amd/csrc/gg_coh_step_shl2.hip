// gg_coh_step_shl2.hip — k_c_step<false, 2> (gg_coh_step.inc): the step
// kernel of the shared-L2 MSI protocol (pr_l1_sh_l2_msi, Tile's PR = 2), and
// its launcher.  Like MOSI it runs on the per-step launches only (no
// persistent instance).
#include "gg_coh_dev.h"
namespace ggc {
#include "gg_coh_step.inc"
void launch_step_shl2(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier)
{
  hipLaunchKernelGGL((k_c_step<false, 2>), dim3(P.L), dim3(64), lds, s, a.P, a.S, L, devloop, barrier, a.kt, a.kt_slot);
}
hipError_t step_shl2_set_lds(size_t lds)
{
  return hipFuncSetAttribute((const void*)k_c_step<false, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}
}  // namespace ggc
