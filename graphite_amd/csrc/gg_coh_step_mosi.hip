// gg_coh_step_mosi.hip — k_c_step<false, 1> (gg_coh_step.inc): the step
// kernel of the MOSI protocol (pr_l1_pr_l2_dram_directory_mosi, Tile's PR = 1),
// and its launcher.  MOSI runs on the per-step launches only (no persistent
// instance).
#include "gg_coh_dev.h"
namespace ggc {
#include "gg_coh_step.inc"
void launch_step_mosi(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier)
{
  hipLaunchKernelGGL((k_c_step<false, 1>), dim3(P.L), dim3(64), lds, s, a.P, a.S, L, devloop, barrier, a.kt, a.kt_slot);
}
hipError_t step_mosi_set_lds(size_t lds)
{
  return hipFuncSetAttribute((const void*)k_c_step<false, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}
}  // namespace ggc
