// bdl_step_sghmc.hip — SGHMC step kernel instances (methods/sghmc.py:482-510).
#include "bdl_kernels.hpp"

namespace bdl {

StepKernel pick_step_sghmc(int method, int noise, int collect, int unroll) {
  if (method == BDL_SGHMC) return pick_noise<BDL_SGHMC>(noise, collect, unroll);
  if (method == BDL_SGHMC_GRAD && collect == BDL_COLLECT_NONE)
    return pick_noise<BDL_SGHMC_GRAD>(noise, BDL_COLLECT_NONE, unroll);
  return nullptr;
}

}  // namespace bdl
