// gg_coh_persist.hip — k_c_persist<false> (gg_coh_persist.inc) and
// its host launchers.  Device code: gg_coh_dev.h.
#include "gg_coh_dev.h"

namespace ggc {

#include "gg_coh_persist.inc"

void launch_persist_plain(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L0, uint32_t L1)
{
  hipLaunchKernelGGL(k_c_persist<false>, dim3(P.L), dim3(64), lds, s, a.P, a.S, L0, L1);
}
hipError_t persist_plain_set_lds(size_t lds)
{
  return hipFuncSetAttribute((const void*)k_c_persist<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}
hipError_t persist_plain_occ(size_t lds, int* per_cu)
{
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, (const void*)k_c_persist<false>, 64, lds);
}

void launch_persist(bool lc, const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L0, uint32_t L1)
{
  if (lc) launch_persist_lc(P, a, lds, s, L0, L1); else launch_persist_plain(P, a, lds, s, L0, L1);
}
hipError_t persist_occupancy(bool lc, size_t lds, int* per_cu)
{
  return lc ? persist_lc_occ(lds, per_cu) : persist_plain_occ(lds, per_cu);
}
hipError_t persist_set_lds(size_t persist_lc_lds, size_t persist_lds)
{
  hipError_t e = hipSuccess;
  if (persist_lc_lds) e = persist_lc_set_lds(persist_lc_lds);
  if (e == hipSuccess) e = persist_plain_set_lds(persist_lds);
  return e;
}

}  // namespace ggc
