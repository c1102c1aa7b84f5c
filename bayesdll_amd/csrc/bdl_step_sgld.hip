// bdl_step_sgld.hip — SGLD / cSGLD step kernel instances (methods/sgld.py:469-484).
#include "bdl_kernels.hpp"

namespace bdl {

StepKernel pick_step_sgld(int method, int noise, int collect, int unroll) {
  if (method == BDL_SGLD) return pick_noise<BDL_SGLD>(noise, collect, unroll);
  if (method == BDL_SGLD_GRAD && collect == BDL_COLLECT_NONE)
    return pick_noise<BDL_SGLD_GRAD>(noise, BDL_COLLECT_NONE, unroll);
  return nullptr;
}

}  // namespace bdl
