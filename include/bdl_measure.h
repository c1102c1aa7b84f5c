/* bdl_measure.h — measurement entry point of the fused SG-MCMC library.
 *
 * Not part of the reference's interface (the reference has no kernels to
 * measure): bench.py times it on a sweep's own buffers to report the HBM
 * ceiling of that sweep's exact access pattern next to the sweep itself
 * (`mix_ceiling` / `of_ceiling` in the bench line).
 * Errors: negative bdl_status (bdl_sgmcmc.h) and bdl_last_error(). */
#ifndef BDL_MEASURE_H
#define BDL_MEASURE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The bare access mix of a sweep — nreads 16-B streams read and nwrites
 * written per float4 group over n fp32 elements, no arithmetic beyond a sum,
 * in the step kernels' loop shape and launch geometry (blocks_per_cu
 * workgroups of 256 per CU, unroll 1 / 2 / 4 groups per lane in flight).
 * Timed on a kernel's own buffers (writes may alias reads, as a step's
 * in-place vectors do) it is the HBM ceiling of that exact access pattern on
 * that exact memory.  Supported (nreads, nwrites): (2,1) posterior draw,
 * (3,2) explore / moments, (4,2) SGLD, (3,4) Welford init, (5,4) Welford
 * collect, (7,5) Adam-SGHMC + SGD.  The written vectors receive reads[0]
 * (+ 0 * the others): their contents are destroyed. */
int bdl_stream_mix(const float* const* reads, int32_t nreads, float* const* writes,
                   int32_t nwrites, int64_t n, int32_t blocks_per_cu, int32_t unroll,
                   void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* BDL_MEASURE_H */
