// gg_coh_step_fast.hip — k_c_step<true> (gg_coh_step.inc): the step kernel
// of configurations whose queues are all register history trees and whose
// caches track no miss types (the headline's), and its launcher.
#include "gg_coh_dev.h"

namespace ggc {

#include "gg_coh_step.inc"

void launch_step_fast(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier)
{
  hipLaunchKernelGGL(k_c_step<true>, dim3(P.L), dim3(64), lds, s, a.P, a.S, L, devloop, barrier, a.kt, a.kt_slot);
}
hipError_t step_fast_set_lds(size_t lds)
{
  return hipFuncSetAttribute((const void*)k_c_step<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

}  // namespace ggc
