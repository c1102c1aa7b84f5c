// bdl_adam.hip — Adam-preconditioned SGHMC kernel instances (methods/adam_sghmc.py:500-553).
#include "bdl_kernels.hpp"

namespace bdl {

template <int NOISE, int COLLECT>
StepKernel pick_adam_unroll(int unroll) {
  // unroll variants only where production runs (noise on); the test-only
  // NONE mode keeps the default depth
  if constexpr (NOISE == BDL_NOISE_NONE) {
    (void)unroll;
    return bdl_adam_kernel<NOISE, COLLECT, false, 2>;
  } else if constexpr (NOISE == BDL_NOISE_BUFFER && COLLECT != BDL_COLLECT_NONE) {
    // the buffer-noise collect at depth 4 holds eleven streams in two
    // register sets and spilled VGPRs to scratch (164-188 B/lane): depth <= 2
    return unroll == 1 ? bdl_adam_kernel<NOISE, COLLECT, false, 1>
                       : bdl_adam_kernel<NOISE, COLLECT, false, 2>;
  } else {
    switch (unroll) {
      case 1:
        return bdl_adam_kernel<NOISE, COLLECT, false, 1>;
      case 4:
        return bdl_adam_kernel<NOISE, COLLECT, false, 4>;
      default:
        return bdl_adam_kernel<NOISE, COLLECT, false, 2>;
    }
  }
}

template <int NOISE>
StepKernel pick_adam_collect(int collect, bool grad_only, int unroll) {
  if (grad_only)
    return collect == BDL_COLLECT_NONE ? bdl_adam_kernel<NOISE, BDL_COLLECT_NONE, true, 2> : nullptr;
  switch (collect) {
    case BDL_COLLECT_NONE:
      return pick_adam_unroll<NOISE, BDL_COLLECT_NONE>(unroll);
    case BDL_COLLECT_MEAN_INIT:
      return pick_adam_unroll<NOISE, BDL_COLLECT_MEAN_INIT>(unroll);
    case BDL_COLLECT_MEAN:
      return pick_adam_unroll<NOISE, BDL_COLLECT_MEAN>(unroll);
  }
  return nullptr;  // the Adam runners collect running means only
}

StepKernel pick_adam(int noise, int collect, bool grad_only, int unroll) {
  switch (noise) {
    case BDL_NOISE_NONE:
      return pick_adam_collect<BDL_NOISE_NONE>(collect, grad_only, unroll);
    case BDL_NOISE_BUFFER:
      return pick_adam_collect<BDL_NOISE_BUFFER>(collect, grad_only, unroll);
    case BDL_NOISE_PHILOX:
      return pick_adam_collect<BDL_NOISE_PHILOX>(collect, grad_only, unroll);
  }
  return nullptr;
}


}  // namespace bdl
