// gg_coh_persist_lc.hip — k_c_persist<true> (gg_coh_persist.inc) with the cache state in LDS and
// its host launchers.  Device code: gg_coh_dev.h.
#include "gg_coh_dev.h"

namespace ggc {

#include "gg_coh_persist.inc"

void launch_persist_lc(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L0, uint32_t L1)
{
  hipLaunchKernelGGL(k_c_persist<true>, dim3(P.L), dim3(64), lds, s, a.P, a.S, L0, L1);
}
hipError_t persist_lc_set_lds(size_t lds)
{
  return hipFuncSetAttribute((const void*)k_c_persist<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}
hipError_t persist_lc_occ(size_t lds, int* per_cu)
{
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, (const void*)k_c_persist<true>, 64, lds);
}

}  // namespace ggc
