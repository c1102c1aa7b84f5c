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

#include "bdl_sgmcmc.h"

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

/* The cSGHMC step launch of `args` (bdl_sgmcmc_step, include/bdl_sgmcmc.h;
 * method BDL_CSGHMC, any collect kind) at the current launch configuration,
 * with the update arithmetic and the noise draw removed: the production
 * kernel's own loop, run table, loads and stores.  theta, mom and (steady
 * kinds) mom1 / mom2 are written back as loaded; the init kinds write
 * mom1 = theta and mom2 = 0 (Welford) or theta^2 (running mean), as the
 * step does.  Its time is the ceiling of that kernel's access schedule.
 * BDL_ERR_ARG for another method. */
int bdl_sgmcmc_step_bare(const bdl_step_args* args, void* hip_stream);

/* Issue schedules of the mix (bdl_stream_mix_schedule): the ceiling of an
 * access pattern is the fastest of them, since the memory system does not
 * serve every order of the same bytes equally fast. */
typedef enum bdl_mix_schedule {
  BDL_MIX_BARE = 0,      /* each iteration: all its loads, then all its stores (bdl_stream_mix) */
  BDL_MIX_PIPELINED = 1, /* the next iteration's loads issued before this one's stores          */
  BDL_MIX_PACED = 2      /* BARE with one Philox4x32-10 + Box-Muller draw per float4 group
                            between loads and stores (a noise-bearing sweep's arithmetic,
                            weighted 0 in the written value)                                 */
} bdl_mix_schedule;

/* bdl_stream_mix in one of the schedules above; same streams, sizes,
 * geometry and written values.  BDL_ERR_ARG for an unknown schedule. */
int bdl_stream_mix_schedule(const float* const* reads, int32_t nreads, float* const* writes,
                            int32_t nwrites, int64_t n, int32_t blocks_per_cu, int32_t unroll,
                            int32_t schedule, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* BDL_MEASURE_H */
