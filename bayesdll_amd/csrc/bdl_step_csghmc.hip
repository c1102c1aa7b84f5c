// bdl_step_csghmc.hip — cSGHMC step kernel instances (methods/csghmc.py:747-778).
#include "bdl_kernels.hpp"

namespace bdl {

StepKernel pick_step_csghmc(int noise, int collect, int unroll) {
  return pick_noise<BDL_CSGHMC>(noise, collect, unroll);
}

// the same sweeps with the arithmetic removed (bdl_sgmcmc_step_bare)
StepKernel pick_step_csghmc_bare(int collect, int unroll) {
  return pick_collect<kMethodBare, BDL_NOISE_NONE>(collect, unroll);
}

}  // namespace bdl
