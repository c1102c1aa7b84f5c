// bdl_api.hip — fused SG-MCMC parameter update for MI355X (gfx950, CDNA4).
//
// One bandwidth-bound sweep over flat fp32 vectors (parameters_to_vector order)
// replaces the reference's per-tensor update loops plus torch.optim.SGD.step()
// plus the thinned posterior-moment accumulation:
//   cSGHMC  methods/csghmc.py:747-778  (+ Welford collect :327-345)
//   SGHMC   methods/sghmc.py:482-510   (+ SGD momentum 0, :229; moments :242-249)
//   SGLD    methods/sgld.py:469-484    (+ SGD momentum mu, :226; moments :239-246)
//   cSGLD   methods/csgld.py:665-680   (+ SGD, :253; per-cycle moments :280-293;
//           clip_grad_norm_ :250-251 through bdl_sgld_step_clipped)
//   Adam-SGHMC  methods/adam_sghmc.py:500-553, methods/adam_csghmc.py:812-860
//
// Design:
//   * elementwise, HBM-bound: no MFMA, no LDS on the data stream; 16-B
//     (dwordx4) non-temporal loads/stores per lane, 1/2/4 independent float4
//     groups in flight per lane, grid-stride sweep; workgroups per CU and
//     depth autotuned per method (kernels.autotune).
//   * per-element attributes (lr group, prior on/off, skip) come from a tiny
//     sorted run table staged in LDS; the block-uniform run cursor advances
//     monotonically, and an iteration wholly inside one run takes the
//     branch-free fast path.
//   * noise: either read from a buffer (torch-RNG parity mode) or generated in
//     registers by counter-based Philox4x32-10 keyed by (seed, chain, step,
//     element/4) + Box-Muller on v_log/v_sin/v_cos — no extra HBM traffic.
//   * every floating-point op is rounded separately in the reference's order
//     (compiled with -ffp-contract=off); SGD's add(alpha=-lr) is an explicit
//     fmaf, as torch's CPU kernel computes it; tensor / Python-scalar
//     divisions follow torch CPU (x / s) or torch on the device (x * fl32(1/s),
//     reciprocal from the host's float64) per BDL_FLAG_RECIP_DIV.
//
// Files: bdl_kernels.hpp (device code shared by the kernel families),
// bdl_step_{csghmc,sghmc,sgld}.hip and bdl_adam.hip (kernel instances per
// method, compiled in parallel), this file (host entry points of the C-ABI,
// validation, launch geometry, the clip-norm / moments / sample kernels).
#include <algorithm>
#include "bdl_kernels.hpp"
#include "bdl_measure.h"

#include <mutex>
#include <vector>

namespace bdl {
namespace {

thread_local std::string g_last_error;

int fail(int code, const char* msg) {
  g_last_error = msg;
  return code;
}

int fail(int code, const std::string& msg) { return fail(code, msg.c_str()); }

// Tunables (bdl_set_launch_config).  blocks_per_cu * #CUs workgroups, each
// lane keeps `unroll` float4 groups in flight per iteration.  Defaults (2
// workgroups/CU, depth 1, grid-stride) from the gfx950 sweep (tools/sweep.py,
// profiles/round1/kernel_v1/sweep_*.log); the Python side autotunes per method.
int g_blocks_per_cu = 2;
int g_unroll = 1;
int g_grid_stride = 1;  // 0: one contiguous span per block; 1: grid-stride sweep

int device_cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    cached[dev] = cus;
  }
  return cached[dev];
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ---------------------------------------------------------------------------
// Gradient-norm reduction for clip_grad_norm_ (csgld.py:250-251).  The SGLD
// sampler gradient G = g + prior + noise is recomputed per element (Philox
// noise is a pure function of its counter, so G is never stored) and
// sum(G^2) reduced: per-lane fp64 accumulation (the fp64 FMA is free next to
// the HBM stream; an fp32 accumulator over ~4 K elements per lane could drift
// past the 1e-5 tolerance), a 64-lane wavefront butterfly (__shfl_xor), the
// block's 4 wave sums through LDS, one fp64 partial per workgroup.  A
// single-workgroup finalize sums the partials in a fixed order
// (deterministic) and writes (total_norm, coef).
// ---------------------------------------------------------------------------
constexpr int kMaxNormPartials = 2048;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int NOISE, bool RECIP, bool PRIOR>
__device__ __forceinline__ double sqnorm_fast(const KArgs& a, const StepConst& c, int64_t gb,
                                              float ns, double acc, const float* gp) {
  constexpr int U = 2;
  f4v th[U], g[U], t0[U], ep[U];
  const f4v z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
    t0[u] = ep[u] = z;
    th[u] = vload(a.theta + e);
    g[u] = vload(gp + e);
    if constexpr (PRIOR) t0[u] = vload(a.prior_mean + e);
    if constexpr (NOISE == BDL_NOISE_BUFFER) ep[u] = vload(a.noise + e);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    if constexpr (NOISE == BDL_NOISE_PHILOX) ep[u] = step_noise4(a, gi);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xt = th[u][j], xg = g[u][j], xv = 0.f;
      update_core<BDL_SGLD_GRAD, NOISE, RECIP, PRIOR, false>(a, c, 0.f, ns, xt, xg, xv, t0[u][j],
                                                             ep[u][j]);
      acc = fma((double)xg, (double)xg, acc);
    }
  }
  return acc;
}

template <int NOISE, bool RECIP>
__device__ __forceinline__ void sqnorm_body(const KArgs& a, double* __restrict__ partials) {
  __shared__ double s_wave[kBlock / 64];
  constexpr int64_t kIter = (int64_t)kBlock * 2;
  StepConst c;
  c.sgd_mom = c.sgd_mom_read = c.has_m2 = c.grad_ready = c.clip = false;
  c.inv_s2 = a.inv_s2;
  c.inv_nd = a.inv_nd;
  c.inv_ca = c.inv_cb = c.clip_coef = 1.0f;
  const int64_t ngroups = (a.n + 3) >> 2, nfull = a.n >> 2;
  stage_runs(a);
  double acc = 0.0;
  int r = find_run_lds(a.nruns, (int64_t)blockIdx.x * kIter * 4);
  for (int64_t gb = (int64_t)blockIdx.x * kIter; gb < ngroups; gb += (int64_t)gridDim.x * kIter) {
    while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
    const int64_t gend = min(gb + kIter, ngroups);
    const uint32_t attr = run_attr(r);
    if (gend == gb + kIter && gend <= nfull && run_end(r) >= gend * 4 && !(attr & kNoFastPath)) {
      const float ns = (attr & BDL_ATTR_HEAD) ? a.ns1 : a.ns0;
      if (attr & BDL_ATTR_PRIOR)
        acc = sqnorm_fast<NOISE, RECIP, true>(a, c, gb, ns, acc, run_grad(a, r));
      else
        acc = sqnorm_fast<NOISE, RECIP, false>(a, c, gb, ns, acc, run_grad(a, r));
    } else {
      int rr = r;  // run of the chunk's first element; a lane's elements only move forward
      for (int u = 0; u < 2; ++u) {
        const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
        if (gi >= gend) continue;
        const int64_t e = gi * 4;
        const f4v z = {0.f, 0.f, 0.f, 0.f};
        const bool gt = a.gbase != nullptr;
        const f4v th = ld4(a.theta, e, a.n), g = gt ? z : ld4(a.grad, e, a.n);
        const f4v t0 = ld4(a.prior_mean, e, a.n);
        f4v ep = z;
        if (NOISE == BDL_NOISE_BUFFER) ep = ld4(a.noise, e, a.n);
        if (NOISE == BDL_NOISE_PHILOX) ep = step_noise4(a, gi);
        for (int j = 0; j < 4; ++j) {
          if (e + j >= a.n) break;
          while (rr < a.nruns - 1 && run_end(rr) <= e + j) ++rr;
          const uint32_t at = run_attr(rr);
          if (at & BDL_ATTR_SKIP) continue;  // .grad is None: not in the norm
          float xt = th[j], xg = gt ? sload(run_grad(a, rr) + e + j) : g[j], xv = 0.f;
          const float ns = (at & BDL_ATTR_HEAD) ? a.ns1 : a.ns0;
          if (at & BDL_ATTR_PRIOR)
            update_core<BDL_SGLD_GRAD, NOISE, RECIP, true, false>(a, c, 0.f, ns, xt, xg, xv, t0[j], ep[j]);
          else
            update_core<BDL_SGLD_GRAD, NOISE, RECIP, false, false>(a, c, 0.f, ns, xt, xg, xv, t0[j], ep[j]);
          acc = fma((double)xg, (double)xg, acc);
        }
      }
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) t += s_wave[w];
    partials[blockIdx.x] = t;
  }
}

template <int NOISE>
__global__ __launch_bounds__(kBlock) void bdl_sqnorm_kernel(const KArgs a, double* partials) {
  if (a.flags & BDL_FLAG_RECIP_DIV)
    sqnorm_body<NOISE, true>(a, partials);
  else
    sqnorm_body<NOISE, false>(a, partials);
}

__global__ __launch_bounds__(kBlock) void bdl_clip_finalize_kernel(const double* __restrict__ partials,
                                                                   int nparts, float max_norm,
                                                                   float* __restrict__ out) {
  __shared__ double s_d[kBlock / 64];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += kBlock) acc += partials[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) s_d[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kBlock / 64; ++w) t += s_d[w];
    const float norm = (float)sqrt(t);
    // clip_grad_norm_: clip_coef = max_norm / (total_norm + 1e-6) (Tensor.__rtruediv__
    // = reciprocal() * other), clamped at 1.0
    float coef = (1.0f / (norm + 1e-6f)) * max_norm;
    coef = fminf(coef, 1.0f);
    out[0] = norm;
    out[1] = coef;
  }
}

// ---------------------------------------------------------------------------
// Stand-alone moments, posterior sample, raw Philox stream.
// ---------------------------------------------------------------------------
struct MArgs {
  const float* __restrict__ theta;
  float* __restrict__ mom1;
  float* __restrict__ mom2;
  int64_t n;
  int32_t collect;
  int32_t recip;
  float ca, cb, inv_ca, inv_cb;
};

// Per-element moment update (the reference's op order; see collect_core for
// the fused-step twin).  COLLECT / RECIP / M2 are compile-time.
template <int COLLECT, bool RECIP>
__device__ __forceinline__ void moments_elem(const MArgs& a, float x, float& p, float& q) {
  if constexpr (COLLECT == BDL_COLLECT_WELFORD_INIT) {
    p = x;
    q = 0.f;
  } else if constexpr (COLLECT == BDL_COLLECT_WELFORD) {
    const float d = x - p;
    p = p + (RECIP ? d * a.inv_ca : d / a.ca);
    const float d2 = x - p;
    q = q + d * d2;
  } else if constexpr (COLLECT == BDL_COLLECT_MEAN_INIT) {
    p = x;
    q = x * x;
  } else {  // MEAN
    const float u = x + a.ca * p;
    p = RECIP ? u * a.inv_cb : u / a.cb;
    const float w = x * x + a.ca * q;
    q = RECIP ? w * a.inv_cb : w / a.cb;
  }
}

template <int COLLECT, bool RECIP>
__device__ __forceinline__ void moments4(const MArgs& a, const f4v t, f4v& m1, f4v& m2) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float p = m1[j], q = m2[j];
    moments_elem<COLLECT, RECIP>(a, t[j], p, q);
    m1[j] = p;
    m2[j] = q;
  }
}

// Grid-stride sweep, U float4 groups per lane in flight: an unguarded loop over
// the block iterations wholly inside the vector (all loads issued before any
// arithmetic), then at most one guarded iteration per block for the tail —
// the loop shape of bdl_sample_kernel.
template <int COLLECT, bool RECIP, bool M2, int U>
__global__ __launch_bounds__(kBlock) void bdl_moments_kernel(const MArgs a) {
  constexpr bool kRead = COLLECT == BDL_COLLECT_WELFORD || COLLECT == BDL_COLLECT_MEAN;
  constexpr int64_t kIter = (int64_t)kBlock * U;
  const int64_t ngroups = (a.n + 3) >> 2, nfull = a.n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kIter;
  const f4v z = {0.f, 0.f, 0.f, 0.f};
  int64_t gb = (int64_t)blockIdx.x * kIter;
  for (; gb + kIter <= nfull; gb += stride) {
    f4v t[U], m1[U], m2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
      m1[u] = m2[u] = z;
      t[u] = vload(a.theta + e);
      if constexpr (kRead) {
        m1[u] = vload(a.mom1 + e);
        if constexpr (M2) m2[u] = vload(a.mom2 + e);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
      moments4<COLLECT, RECIP>(a, t[u], m1[u], m2[u]);
      vstore(a.mom1 + e, m1[u]);
      if constexpr (M2) vstore(a.mom2 + e, m2[u]);
    }
  }
  if (gb < ngroups) {
    for (int u = 0; u < U; ++u) {
      const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
      if (gi >= ngroups) break;
      const int64_t e = gi * 4;
      f4v m1 = z, m2 = z;
      const f4v t = ld4(a.theta, e, a.n);
      if constexpr (kRead) {
        m1 = ld4(a.mom1, e, a.n);
        if constexpr (M2) m2 = ld4(a.mom2, e, a.n);
      }
      moments4<COLLECT, RECIP>(a, t, m1, m2);
      st4(a.mom1, e, a.n, m1);
      if constexpr (M2) st4(a.mom2, e, a.n, m2);
    }
  }
}

typedef void (*MomentsKernel)(const MArgs);

template <int COLLECT>
MomentsKernel pick_moments_c(bool recip, bool m2) {
  constexpr int U = 4;
  if (recip) return m2 ? bdl_moments_kernel<COLLECT, true, true, U> : bdl_moments_kernel<COLLECT, true, false, U>;
  return m2 ? bdl_moments_kernel<COLLECT, false, true, U> : bdl_moments_kernel<COLLECT, false, false, U>;
}

MomentsKernel pick_moments(int collect, bool recip, bool m2) {
  switch (collect) {
    case BDL_COLLECT_WELFORD_INIT: return pick_moments_c<BDL_COLLECT_WELFORD_INIT>(recip, m2);
    case BDL_COLLECT_WELFORD: return pick_moments_c<BDL_COLLECT_WELFORD>(recip, m2);
    case BDL_COLLECT_MEAN_INIT: return pick_moments_c<BDL_COLLECT_MEAN_INIT>(recip, m2);
    default: return pick_moments_c<BDL_COLLECT_MEAN>(recip, m2);
  }
}

struct SArgs {
  float* __restrict__ out;
  const float* __restrict__ mom1;
  const float* __restrict__ mom2;
  const float* __restrict__ noise;
  int64_t n;
  int32_t var_mode, noise_mode;
  float ratio, var_floor, inv_ratio;
  uint64_t seed, chain, step;
  uint32_t cgroups;  // stacked chains: float4 groups per chain (0 = one chain)
};

// theta_s = m1 + sqrt(clamp(var, floor)) * eps.  VAR: where the variance
// comes from (M2 = false: no second moment, var = floor — a single-sample
// cycle, csghmc.py:456-458); RECIP: Welford M2 * fl(1/(n-1)) as torch on the
// device; NOISE: buffer or in-register Philox.  Same sweep shape as the
// moments kernel.
// Philox draw for group gi (stacked chains as in step_noise4).
__device__ __forceinline__ f4v sample_noise4(const SArgs& a, int64_t gi) {
  uint64_t g = (uint64_t)gi, c = a.chain;
  if (a.cgroups) {
    const uint32_t k = (uint32_t)g / a.cgroups;
    g -= (uint64_t)k * a.cgroups;
    c += k;
  }
  return philox_normal4(g, a.seed, c, a.step);
}

template <int VAR, bool M2, bool RECIP>
__device__ __forceinline__ float sample_var(const SArgs& a, float mj, float qj) {
  float var;
  if constexpr (!M2)
    var = a.var_floor;
  else if constexpr (VAR == BDL_VAR_RAW_MOMENTS)
    var = a.ratio * (qj - mj * mj);  // sgld.py:342
  else if constexpr (VAR == BDL_VAR_WELFORD)
    var = RECIP ? qj * a.inv_ratio : qj / a.ratio;  // csghmc.py:455
  else
    var = qj;
  if (!(var != var)) var = fmaxf(var, a.var_floor);  // clamp_(min=1e-12); NaN stays NaN
  return var;
}

// FLOORED: the host saw var_floor >= 2^-96, so every variance is NaN or at
// least 2^-96 and sqrt_floored gives sqrtf's bits with ~6 VALU ops fewer.
template <int VAR, bool M2, bool RECIP, bool FLOORED>
__device__ __forceinline__ f4v sample4(const SArgs& a, const f4v m, const f4v q, const f4v ep) {
  f4v o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float var = sample_var<VAR, M2, RECIP>(a, m[j], q[j]);
    o[j] = m[j] + (FLOORED ? sqrt_floored(var) : sqrtf(var)) * ep[j];
  }
  return o;
}

// Unguarded loop over the full block iterations (all loads first, then the
// generator and the math, then the stores), then at most one guarded
// iteration per block for the vector's tail.  Split this way the fast loop
// carries no per-group range branch: 0.586-0.598 ms vs 0.608 ms for the
// per-group-guarded loop at ViT-L/32 size (tools/sample_probe.hip,
// profiles/round2/aux/sample_probe.jsonl).
template <int VAR, bool M2, bool RECIP, int NOISE, bool FLOORED, int U>
__global__ __launch_bounds__(kBlock) void bdl_sample_kernel(const SArgs a) {
  constexpr int64_t kIter = (int64_t)kBlock * U;
  const int64_t ngroups = (a.n + 3) >> 2, nfull = a.n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kIter;
  const f4v z = {0.f, 0.f, 0.f, 0.f};
  int64_t gb = (int64_t)blockIdx.x * kIter;
  for (; gb + kIter <= nfull; gb += stride) {
    f4v m[U], q[U], ep[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
      m[u] = vload(a.mom1 + e);
      q[u] = z;
      if constexpr (M2) q[u] = vload(a.mom2 + e);
      if constexpr (NOISE == BDL_NOISE_BUFFER) ep[u] = vload(a.noise + e);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
      if constexpr (NOISE == BDL_NOISE_PHILOX) ep[u] = sample_noise4(a, gi);
      vstore(a.out + gi * 4, sample4<VAR, M2, RECIP, FLOORED>(a, m[u], q[u], ep[u]));
    }
  }
  if (gb < ngroups) {
    for (int u = 0; u < U; ++u) {
      const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
      if (gi >= ngroups) break;
      const int64_t e = gi * 4;
      const f4v m = ld4(a.mom1, e, a.n);
      const f4v q = M2 ? ld4(a.mom2, e, a.n) : z;
      const f4v ep = NOISE == BDL_NOISE_BUFFER ? ld4(a.noise, e, a.n) : sample_noise4(a, gi);
      st4(a.out, e, a.n, sample4<VAR, M2, RECIP, FLOORED>(a, m, q, ep));
    }
  }
}

typedef void (*SampleKernel)(const SArgs);

// Posterior-sample geometry, independent of the step kernels' tuning:
// workgroups per CU (bdl_sample_args.blocks_per_cu, default 2) and float4
// groups per lane in flight (bdl_sample_args.unroll: 4, the default, or 1).
// The host tunes both once per vector size (kernels.posterior_sample): the
// bare access mix of the draw's buffers ranked 3 x 4 first at ViT-L/32 size
// and 4 x 1 at ResNet-101 size on one box (bench.py mix_ceiling), round 2's
// probes 2 x 4 on two others.
#ifndef BDL_SAMPLE_BPC
#define BDL_SAMPLE_BPC 2
#endif

template <int NOISE, bool FL, int U>
SampleKernel pick_sample_n(int var_mode, bool m2, bool recip) {
  if (!m2) return bdl_sample_kernel<BDL_VAR_GIVEN, false, false, NOISE, FL, U>;
  switch (var_mode) {
    case BDL_VAR_RAW_MOMENTS: return bdl_sample_kernel<BDL_VAR_RAW_MOMENTS, true, false, NOISE, FL, U>;
    case BDL_VAR_WELFORD:
      return recip ? bdl_sample_kernel<BDL_VAR_WELFORD, true, true, NOISE, FL, U>
                   : bdl_sample_kernel<BDL_VAR_WELFORD, true, false, NOISE, FL, U>;
    default: return bdl_sample_kernel<BDL_VAR_GIVEN, true, false, NOISE, FL, U>;
  }
}

template <int U>
SampleKernel pick_sample_u(int var_mode, bool m2, bool recip, int noise_mode, bool floored) {
  if (noise_mode == BDL_NOISE_BUFFER)
    return floored ? pick_sample_n<BDL_NOISE_BUFFER, true, U>(var_mode, m2, recip)
                   : pick_sample_n<BDL_NOISE_BUFFER, false, U>(var_mode, m2, recip);
  return floored ? pick_sample_n<BDL_NOISE_PHILOX, true, U>(var_mode, m2, recip)
                 : pick_sample_n<BDL_NOISE_PHILOX, false, U>(var_mode, m2, recip);
}

// floored: var_floor >= 2^-96 (the Runners' 1e-12 clamp), see sqrt_floored
SampleKernel pick_sample(int var_mode, bool m2, bool recip, int noise_mode, bool floored,
                         int unroll) {
  return unroll == 1 ? pick_sample_u<1>(var_mode, m2, recip, noise_mode, floored)
                     : pick_sample_u<4>(var_mode, m2, recip, noise_mode, floored);
}

__global__ __launch_bounds__(kBlock) void bdl_philox_kernel(float* __restrict__ out, int64_t n,
                                                            uint64_t seed, uint64_t chain,
                                                            uint64_t step) {
  const int64_t ngroups = (n + 3) >> 2;
  for (int64_t gi = (int64_t)blockIdx.x * kBlock + threadIdx.x; gi < ngroups;
       gi += (int64_t)gridDim.x * kBlock) {
    st4(out, gi * 4, n, philox_normal4((uint64_t)gi, seed, chain, step));
  }
}

StepKernel pick_step(int method, int noise, int collect, int unroll) {
  switch (method) {
    case BDL_CSGHMC:
      return pick_step_csghmc(noise, collect, unroll);
    case BDL_SGHMC:
    case BDL_SGHMC_GRAD:
      return pick_step_sghmc(method, noise, collect, unroll);
    case BDL_SGLD:
    case BDL_SGLD_GRAD:
      return pick_step_sgld(method, noise, collect, unroll);
  }
  return nullptr;
}

int grid_for(int64_t ngroups, int per_block_groups) {
  const int64_t want = (ngroups + per_block_groups - 1) / per_block_groups;
  const int64_t cap = (int64_t)device_cu_count() * g_blocks_per_cu;
  return (int)std::max<int64_t>(1, std::min(want, cap));
}

int grid_sample(int64_t ngroups, int blocks_per_cu, int unroll) {
  const int64_t per_block = (int64_t)kBlock * unroll;
  const int64_t want = (ngroups + per_block - 1) / per_block;
  const int64_t cap = (int64_t)device_cu_count() * (blocks_per_cu > 0 ? blocks_per_cu : BDL_SAMPLE_BPC);
  return (int)std::max<int64_t>(1, std::min(want, cap));
}

// Validate a step descriptor, pick the kernel instance and launch it; `clip`
// (device pointer to (norm, coef)) scales the SGLD sampler gradient when set.
// Dynamic LDS of a step launch: the run table, plus the per-run gradient
// bases in grad_base mode.  Both fit the 64 KiB a launch gets by default.
size_t run_lds_bytes(const bdl_step_args* s) {
  return (size_t)s->nruns * (sizeof(bdl_run) + (s->grad_base ? sizeof(int64_t) : 0));
}

// Shared checks of the run table and the gradient source ("what" prefixes errors).
int check_runs_and_grad(const bdl_step_args* s, const char* what) {
  if (!s->runs || s->nruns < 1)
    return fail(BDL_ERR_NULL, std::string(what) + ": runs are required");
  if (run_lds_bytes(s) > (size_t)kMaxRuns * sizeof(bdl_run))
    return fail(BDL_ERR_RUNS, std::string(what) + ": run table exceeds 64 KiB of LDS (4096 runs, "
                "2730 with grad_base; merge parameter groups)");
  if (!s->grad && !s->grad_base)
    return fail(BDL_ERR_NULL, std::string(what) + ": grad or grad_base is required");
  if (s->grad && !aligned16(s->grad))
    return fail(BDL_ERR_ALIGN, std::string(what) + ": grad not 16-B aligned");
  if (s->grad_base && (reinterpret_cast<uintptr_t>(s->grad_base) & 7u))
    return fail(BDL_ERR_ALIGN, std::string(what) + ": grad_base not 8-B aligned");
  if (s->chain_groups &&
      (s->chain_groups > 0xFFFFFFFFull ||
       (uint64_t)((s->n + 3) / 4) + s->philox_offset > 0xFFFFFFFFull))
    return fail(BDL_ERR_ARG, std::string(what) + ": stacked chains need every float4 group "
                "index below 2^32 (chain_groups, n / 4 + philox_offset)");
  return BDL_OK;
}

// Graph-node binding (bdl_graph_find_step_node / bdl_graph_redirect): the
// step kernels launched into a capture (to recognise their nodes), and the
// instantiated graph + node the thread's next bdl_sgmcmc_step rewrites
// instead of launching.  While a redirect is set, every other launching entry
// point refuses (no_redirect): their launches would go to the stream, mixed
// with node rewrites.
std::mutex g_captured_mu;
std::vector<const void*> g_captured_funcs;  // step kernels launched into a capture
thread_local hipGraphExec_t g_redirect_exec = nullptr;
thread_local hipGraphNode_t g_redirect_node = nullptr;

int no_redirect(const char* what) {
  if (!g_redirect_exec) return BDL_OK;
  return fail(BDL_ERR_ARG, std::string(what) + ": a graph redirect is active (bdl_graph_redirect); "
              "only bdl_sgmcmc_step rewrites a node");
}

int launch_step(const bdl_step_args* s, const float* clip, hipStream_t stream, bool bare = false) {
  if (!s) return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: null args");
  if (s->n < 0) return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: n < 0");
  if (s->method < BDL_CSGHMC || s->method > BDL_SGLD_GRAD)
    return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: unknown method");
  if (s->noise_mode < BDL_NOISE_NONE || s->noise_mode > BDL_NOISE_PHILOX)
    return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: unknown noise mode");
  if (s->collect < BDL_COLLECT_NONE || s->collect > BDL_COLLECT_MEAN)
    return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: unknown collect mode");
  if (s->n == 0) return BDL_OK;
  const bool grad_only = s->method == BDL_SGHMC_GRAD || s->method == BDL_SGLD_GRAD;
  const bool needs_mom = s->method == BDL_CSGHMC || s->method == BDL_SGHMC ||
                         s->method == BDL_SGHMC_GRAD ||
                         (s->method == BDL_SGLD && (s->flags & BDL_FLAG_MOMENTUM));
  const bool needs_prior = s->method != BDL_CSGHMC;
  if (!s->theta) return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: theta is required");
  if (const int rc = check_runs_and_grad(s, "bdl_sgmcmc_step")) return rc;
  if (needs_mom && !s->mom) return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: mom is required");
  if (needs_prior && !s->prior_mean)
    return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: prior_mean is required for sghmc/sgld");
  if (s->noise_mode == BDL_NOISE_BUFFER && !s->noise)
    return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: noise buffer is required");
  if (s->collect != BDL_COLLECT_NONE && !s->mom1)
    return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: mom1 is required to collect");
  if (grad_only && s->collect != BDL_COLLECT_NONE)
    return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: grad-only methods cannot collect");
  const void* ptrs[] = {s->theta, s->mom, s->prior_mean, s->noise, s->mom1, s->mom2};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(BDL_ERR_ALIGN, "bdl_sgmcmc_step: vector not 16-B aligned");

  const int unroll = g_unroll;
  StepKernel k = bare ? (s->method == BDL_CSGHMC ? pick_step_csghmc_bare(s->collect, unroll)
                                                 : nullptr)
                      : pick_step(s->method, s->noise_mode, s->collect, unroll);
  if (!k) return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: unsupported method/noise/collect combination");

  const int64_t ngroups = (s->n + 3) / 4;
  const int64_t per_iter = (int64_t)kBlock * unroll;
  const int64_t cap = (int64_t)device_cu_count() * g_blocks_per_cu;
  int64_t iters = (ngroups + per_iter - 1) / per_iter;
  int64_t grid = std::max<int64_t>(1, std::min(iters, cap));
  int64_t iters_per_block = (iters + grid - 1) / grid;
  grid = (iters + iters_per_block - 1) / iters_per_block;

  KArgs a;
  a.theta = s->theta;
  a.grad = s->grad;
  a.mom = s->mom;
  a.prior_mean = s->prior_mean;
  a.noise = s->noise;
  a.mom1 = s->mom1;
  a.mom2 = s->mom2;
  a.runs = s->runs;
  a.gbase = s->grad_base;
  a.nruns = s->nruns;
  a.flags = s->flags;
  a.n = s->n;
  a.groups_per_block = g_grid_stride ? 0 : iters_per_block * per_iter;
  a.lr0 = s->lr[0];
  a.lr1 = s->lr[1];
  a.ns0 = s->noise_scale[0];
  a.ns1 = s->noise_scale[1];
  a.one_minus_alpha = s->one_minus_alpha;
  a.prior_sig = s->prior_sig;
  a.sigma2 = s->sigma2;
  a.n_data = s->n_data;
  a.mu = s->mu;
  a.ca = s->collect_a;
  a.cb = s->collect_b;
  a.seed = s->seed;
  a.chain = s->chain;
  a.step = s->step;
  a.clip = clip;
  a.nonfinite = s->nonfinite;
  a.goff = s->philox_offset;
  a.cgroups = (uint32_t)s->chain_groups;
  a.inv_s2 = recip_or(s->inv_sigma2, s->sigma2);
  a.inv_nd = recip_or(s->inv_n_data, s->n_data);
  a.inv_ca = recip_or(s->inv_collect_a, s->collect_a);
  a.inv_cb = recip_or(s->inv_collect_b, s->collect_b);

  if (g_redirect_exec) {
    // the node must be a kernel node running this very kernel (checked on
    // the graph it was instantiated from): anything else is an error here,
    // never a launch of this kernel with another node's geometry
    hipGraphNodeType nt = hipGraphNodeTypeEmpty;
    hipKernelNodeParams cur{};
    if (hipGraphNodeGetType(g_redirect_node, &nt) != hipSuccess || nt != hipGraphNodeTypeKernel ||
        hipGraphKernelNodeGetParams(g_redirect_node, &cur) != hipSuccess ||
        cur.func != (void*)k) {
      (void)hipGetLastError();
      return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: the redirect node is not this step's kernel");
    }
    void* kp[] = {&a};
    hipKernelNodeParams p{};
    p.func = (void*)k;
    p.gridDim = dim3((unsigned)grid);
    p.blockDim = dim3(kBlock);
    p.sharedMemBytes = (unsigned)run_lds_bytes(s);
    p.kernelParams = kp;
    const hipError_t err = hipGraphExecKernelNodeSetParams(g_redirect_exec, g_redirect_node, &p);
    if (err != hipSuccess) {
      (void)hipGetLastError();
      g_last_error = std::string("bdl_sgmcmc_step: graph node update failed: ") +
                     hipGetErrorString(err);
      return BDL_ERR_LAUNCH;
    }
    return BDL_OK;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kBlock), run_lds_bytes(s), stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_sgmcmc_step: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (stream && hipStreamIsCapturing(stream, &cs) == hipSuccess &&
      cs == hipStreamCaptureStatusActive) {
    std::lock_guard<std::mutex> lk(g_captured_mu);
    if (std::find(g_captured_funcs.begin(), g_captured_funcs.end(), (const void*)k) ==
        g_captured_funcs.end())
      g_captured_funcs.push_back((const void*)k);
  }
  (void)hipGetLastError();
  return BDL_OK;
}


// ---------------------------------------------------------------------------
// Bare access mix of a sweep (measurement only, bdl_stream_mix /
// bdl_stream_mix_schedule): NR 16-B streams read and NW written per float4
// group with no arithmetic beyond a sum, in the step kernels' loop shape
// (unguarded full iterations, one guarded tail iteration) — the HBM ceiling
// of a kernel's exact access pattern on its exact buffers.  Written values:
// r0 + 0 * r1 + ... (finite, usually r0).  Three issue schedules, since the
// memory system does not serve every order of the same bytes equally fast
// and a ceiling is the fastest of them:
//   BARE       every load of an iteration, then every store;
//   PIPELINED  the next iteration's loads issued before this one's stores
//              (two register sets, as the Adam sweep);
//   PACED      BARE with one Philox4x32-10 + Box-Muller draw per group
//              between the loads and the stores (the noise-bearing sweeps'
//              arithmetic, multiplied by 0 into the written value): the
//              spacing of a real sweep's stores without its update.
// ---------------------------------------------------------------------------
constexpr int kMixMaxR = 8, kMixMaxW = 6;
struct MixArgs {
  const float* r[kMixMaxR];
  float* w[kMixMaxW];
  int64_t n;
};

template <int NR, int U>
__device__ __forceinline__ void mix_load(const MixArgs& a, int64_t gb, f4v (&x)[U][NR]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
#pragma unroll
    for (int r = 0; r < NR; ++r) x[u][r] = vload(a.r[r] + e);
  }
}

template <int NR, int NW, int U, bool PACED>
__device__ __forceinline__ void mix_store(const MixArgs& a, int64_t gb, f4v (&x)[U][NR]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    f4v acc = x[u][0];
#pragma unroll
    for (int r = 1; r < NR; ++r) acc = acc + x[u][r] * 0.0f;
    if constexpr (PACED) acc = acc + philox_normal4((uint64_t)gi, 0x5eedull, 0, 1) * 0.0f;
#pragma unroll
    for (int w = 0; w < NW; ++w) vstore(a.w[w] + e, acc);
  }
}

template <int NR, int NW, int U, int S>
__global__ __launch_bounds__(kBlock) void bdl_mix_kernel(const MixArgs a) {
  constexpr int64_t kIter = (int64_t)kBlock * U;
  const int64_t ngroups = (a.n + 3) >> 2, nfull = a.n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kIter;
  int64_t gb = (int64_t)blockIdx.x * kIter;
  if constexpr (S == BDL_MIX_PIPELINED) {
    f4v x[U][NR], y[U][NR];
    if (gb + kIter <= nfull) mix_load<NR, U>(a, gb, x);
    for (; gb + kIter <= nfull; gb += stride) {
      const bool more = gb + stride + kIter <= nfull;
      if (more) mix_load<NR, U>(a, gb + stride, y);
      mix_store<NR, NW, U, false>(a, gb, x);
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < NR; ++r) x[u][r] = y[u][r];
      }
    }
  } else {
    for (; gb + kIter <= nfull; gb += stride) {
      f4v x[U][NR];
      mix_load<NR, U>(a, gb, x);
      mix_store<NR, NW, U, S == BDL_MIX_PACED>(a, gb, x);
    }
  }
  if (gb < ngroups) {
    for (int u = 0; u < U; ++u) {
      const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
      if (gi >= ngroups) break;
      const int64_t e = gi * 4;
      f4v acc = ld4(a.r[0], e, a.n);
      for (int r = 1; r < NR; ++r) acc = acc + ld4(a.r[r], e, a.n) * 0.0f;
      for (int w = 0; w < NW; ++w) st4(a.w[w], e, a.n, acc);
    }
  }
}

typedef void (*MixKernel)(const MixArgs);

template <int NR, int NW, int S>
MixKernel pick_mix_u(int unroll) {
  switch (unroll) {
    case 1: return bdl_mix_kernel<NR, NW, 1, S>;
    case 4: return bdl_mix_kernel<NR, NW, 4, S>;
    default: return bdl_mix_kernel<NR, NW, 2, S>;
  }
}

template <int NR, int NW>
MixKernel pick_mix_s(int schedule, int unroll) {
  switch (schedule) {
    case BDL_MIX_BARE: return pick_mix_u<NR, NW, BDL_MIX_BARE>(unroll);
    case BDL_MIX_PIPELINED: return pick_mix_u<NR, NW, BDL_MIX_PIPELINED>(unroll);
    case BDL_MIX_PACED: return pick_mix_u<NR, NW, BDL_MIX_PACED>(unroll);
  }
  return nullptr;
}

// the mixes of the path's sweeps: draw (2, 1), explore / moments (3, 2),
// SGLD (4, 2), Welford init (3, 4), Welford collect (5, 4), Adam + SGD (7, 5)
MixKernel pick_mix(int nr, int nw, int schedule, int unroll) {
  if (nr == 2 && nw == 1) return pick_mix_s<2, 1>(schedule, unroll);
  if (nr == 3 && nw == 2) return pick_mix_s<3, 2>(schedule, unroll);
  if (nr == 4 && nw == 2) return pick_mix_s<4, 2>(schedule, unroll);
  if (nr == 3 && nw == 4) return pick_mix_s<3, 4>(schedule, unroll);
  if (nr == 5 && nw == 4) return pick_mix_s<5, 4>(schedule, unroll);
  if (nr == 7 && nw == 5) return pick_mix_s<7, 5>(schedule, unroll);
  return nullptr;
}

}  // namespace

// errors of the other host translation units (bdl_arena.hip)
void set_last_error(const std::string& msg) { g_last_error = msg; }

}  // namespace bdl

using namespace bdl;

extern "C" {

int bdl_version(void) { return BDL_ABI_VERSION; }

int bdl_graph_find_step_node(void* graph, const void* theta, int64_t n, void** node) {
  if (!graph || !node) return fail(BDL_ERR_NULL, "bdl_graph_find_step_node: null argument");
  *node = nullptr;
  std::vector<const void*> funcs;
  {
    std::lock_guard<std::mutex> lk(g_captured_mu);
    funcs = g_captured_funcs;
  }
  size_t count = 0;
  if (hipGraphGetNodes((hipGraph_t)graph, nullptr, &count) != hipSuccess) {
    (void)hipGetLastError();
    return fail(BDL_ERR_ARG, "bdl_graph_find_step_node: hipGraphGetNodes failed");
  }
  std::vector<hipGraphNode_t> nodes(count);
  if (count && hipGraphGetNodes((hipGraph_t)graph, nodes.data(), &count) != hipSuccess) {
    (void)hipGetLastError();
    return fail(BDL_ERR_ARG, "bdl_graph_find_step_node: hipGraphGetNodes failed");
  }
  int found = 0;
  for (hipGraphNode_t nd : nodes) {
    hipGraphNodeType t = hipGraphNodeTypeEmpty;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams p{};
    if (hipGraphKernelNodeGetParams(nd, &p) != hipSuccess) continue;
    // only nodes running one of our step kernels carry a KArgs to look at
    if (std::find(funcs.begin(), funcs.end(), (const void*)p.func) == funcs.end()) continue;
    if (!p.kernelParams || !p.kernelParams[0]) continue;
    const KArgs* ka = (const KArgs*)p.kernelParams[0];
    if ((const void*)ka->theta == theta && ka->n == n) {
      *node = (void*)nd;
      ++found;
    }
  }
  (void)hipGetLastError();
  if (found != 1) {
    *node = nullptr;
    return fail(BDL_ERR_ARG, "bdl_graph_find_step_node: " + std::to_string(found) +
                                 " step nodes over this range");
  }
  return BDL_OK;
}

int bdl_graph_node_step_args(void* node, int64_t* out, int32_t nout) {
  if (!node || !out) return fail(BDL_ERR_NULL, "bdl_graph_node_step_args: null argument");
  if (nout < 10) return fail(BDL_ERR_ARG, "bdl_graph_node_step_args: out needs 10 entries");
  hipGraphNodeType t = hipGraphNodeTypeEmpty;
  hipKernelNodeParams p{};
  if (hipGraphNodeGetType((hipGraphNode_t)node, &t) != hipSuccess || t != hipGraphNodeTypeKernel ||
      hipGraphKernelNodeGetParams((hipGraphNode_t)node, &p) != hipSuccess || !p.kernelParams ||
      !p.kernelParams[0]) {
    (void)hipGetLastError();
    return fail(BDL_ERR_ARG, "bdl_graph_node_step_args: not a kernel node with arguments");
  }
  {
    std::lock_guard<std::mutex> lk(g_captured_mu);
    if (std::find(g_captured_funcs.begin(), g_captured_funcs.end(), (const void*)p.func) ==
        g_captured_funcs.end())
      return fail(BDL_ERR_ARG, "bdl_graph_node_step_args: the node runs no captured step kernel");
  }
  const KArgs* ka = (const KArgs*)p.kernelParams[0];
  const int64_t v[10] = {(int64_t)(uintptr_t)ka->theta, (int64_t)(uintptr_t)ka->grad,
                         (int64_t)(uintptr_t)ka->mom,   (int64_t)(uintptr_t)ka->runs,
                         (int64_t)(uintptr_t)ka->gbase, (int64_t)ka->nruns,
                         ka->n,                          (int64_t)ka->flags,
                         (int64_t)(uintptr_t)ka->mom1,  (int64_t)(uintptr_t)ka->mom2};
  for (int i = 0; i < 10; ++i) out[i] = v[i];
  return BDL_OK;
}

int bdl_graph_redirect(void* graph_exec, void* node) {
  if (graph_exec && !node) return fail(BDL_ERR_NULL, "bdl_graph_redirect: null node");
  g_redirect_exec = (hipGraphExec_t)graph_exec;
  g_redirect_node = graph_exec ? (hipGraphNode_t)node : nullptr;
  return BDL_OK;
}

const char* bdl_last_error(void) { return g_last_error.c_str(); }

int bdl_set_launch_config(int32_t blocks_per_cu, int32_t unroll, int32_t grid_stride) {
  const int prev = (g_grid_stride << 24) | (g_blocks_per_cu << 8) | g_unroll;
  g_blocks_per_cu = blocks_per_cu > 0 ? blocks_per_cu : 2;
  g_unroll = (unroll == 1 || unroll == 2 || unroll == 4) ? unroll : 1;
  g_grid_stride = grid_stride > 0 ? 1 : 0;
  return prev;
}

int bdl_build_runs(const bdl_segment* segs, int32_t nseg, int64_t n, bdl_run* out, int32_t max_runs) {
  if (!out || (nseg > 0 && !segs)) return fail(BDL_ERR_NULL, "bdl_build_runs: null pointer");
  if (n < 0 || nseg < 0 || max_runs < 1) return fail(BDL_ERR_ARG, "bdl_build_runs: bad sizes");
  int nr = 0;
  int64_t pos = 0;
  auto push = [&](int64_t end, uint32_t attr) -> bool {
    if (end <= pos) return true;
    if (nr > 0 && out[nr - 1].attr == attr) {
      out[nr - 1].end = end;
    } else {
      if (nr >= max_runs) return false;
      out[nr].end = end;
      out[nr].attr = attr;
      out[nr].pad = 0;
      ++nr;
    }
    pos = end;
    return true;
  };
  for (int i = 0; i < nseg; ++i) {
    const bdl_segment& s = segs[i];
    if (s.offset < pos || s.numel < 0 || s.offset + s.numel > n)
      return fail(BDL_ERR_RUNS, "bdl_build_runs: segments overlap, are unsorted or exceed n");
    if (!push(s.offset, BDL_ATTR_SKIP)) return fail(BDL_ERR_ARG, "bdl_build_runs: too many runs");
    if (!push(s.offset + s.numel, s.attr & 0xFu))
      return fail(BDL_ERR_ARG, "bdl_build_runs: too many runs");
  }
  if (!push(n, BDL_ATTR_SKIP)) return fail(BDL_ERR_ARG, "bdl_build_runs: too many runs");
  if (nr == 0) {  // n == 0: one empty run keeps the table well-formed
    out[0].end = 0;
    out[0].attr = BDL_ATTR_SKIP;
    out[0].pad = 0;
    nr = 1;
  }
  return nr;
}

int bdl_sgmcmc_step(const bdl_step_args* s, void* stream) {
  return launch_step(s, nullptr, (hipStream_t)stream);
}

int bdl_sgmcmc_step_bare(const bdl_step_args* s, void* stream) {
  if (const int rc = no_redirect("bdl_sgmcmc_step_bare")) return rc;
  if (s && s->method != BDL_CSGHMC)
    return fail(BDL_ERR_ARG, "bdl_sgmcmc_step_bare: the bare sweep exists for cSGHMC only");
  return launch_step(s, nullptr, (hipStream_t)stream, true);
}

int64_t bdl_clip_workspace_bytes(int64_t n) {
  (void)n;
  // (total_norm, coef) + pad to 16 B, then one fp64 partial per workgroup
  return (int64_t)16 + (int64_t)kMaxNormPartials * (int64_t)sizeof(double);
}

int bdl_sgld_step_clipped(const bdl_step_args* s, float max_norm, void* workspace, void* stream) {
  if (const int rc = no_redirect("bdl_sgld_step_clipped")) return rc;
  if (!s) return fail(BDL_ERR_NULL, "bdl_sgld_step_clipped: null args");
  if (!workspace) return fail(BDL_ERR_NULL, "bdl_sgld_step_clipped: null workspace");
  if (!aligned16(workspace)) return fail(BDL_ERR_ALIGN, "bdl_sgld_step_clipped: workspace not 16-B aligned");
  if (s->method != BDL_SGLD)
    return fail(BDL_ERR_ARG, "bdl_sgld_step_clipped: only the SGLD sampler clips its gradient");
  if (s->flags & BDL_FLAG_GRAD_READY)
    return fail(BDL_ERR_ARG, "bdl_sgld_step_clipped: GRAD_READY is incompatible with clipping");
  if (!(max_norm > 0.0f)) return fail(BDL_ERR_ARG, "bdl_sgld_step_clipped: max_norm must be > 0");
  if (s->n < 0) return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: n < 0");
  if (s->n == 0) return BDL_OK;
  if (s->noise_mode < BDL_NOISE_NONE || s->noise_mode > BDL_NOISE_PHILOX)
    return fail(BDL_ERR_ARG, "bdl_sgld_step_clipped: unknown noise mode");
  if (!s->theta || !s->prior_mean)
    return fail(BDL_ERR_NULL, "bdl_sgld_step_clipped: theta and prior_mean are required");
  if (const int rc = check_runs_and_grad(s, "bdl_sgld_step_clipped")) return rc;
  if (s->noise_mode == BDL_NOISE_BUFFER && !s->noise)
    return fail(BDL_ERR_NULL, "bdl_sgld_step_clipped: noise buffer is required");
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  double* partials = reinterpret_cast<double*>(reinterpret_cast<char*>(workspace) + 16);

  KArgs a{};
  a.theta = s->theta;
  a.grad = s->grad;
  a.prior_mean = s->prior_mean;
  a.noise = s->noise;
  a.runs = s->runs;
  a.gbase = s->grad_base;
  a.nruns = s->nruns;
  a.flags = s->flags;
  a.n = s->n;
  a.goff = s->philox_offset;
  a.cgroups = (uint32_t)s->chain_groups;
  a.ns0 = s->noise_scale[0];
  a.ns1 = s->noise_scale[1];
  a.sigma2 = s->sigma2;
  a.n_data = s->n_data;
  a.seed = s->seed;
  a.chain = s->chain;
  a.step = s->step;
  a.inv_s2 = recip_or(s->inv_sigma2, s->sigma2);
  a.inv_nd = recip_or(s->inv_n_data, s->n_data);
  const int64_t ngroups = (s->n + 3) / 4;
  const int64_t iters = (ngroups + 2 * kBlock - 1) / (2 * kBlock);
  const int64_t cap = std::min<int64_t>((int64_t)device_cu_count() * g_blocks_per_cu, kMaxNormPartials);
  const int grid = (int)std::max<int64_t>(1, std::min(iters, cap));
  const size_t shmem = run_lds_bytes(s);
  switch (s->noise_mode) {
    case BDL_NOISE_NONE:
      hipLaunchKernelGGL(bdl_sqnorm_kernel<BDL_NOISE_NONE>, dim3(grid), dim3(kBlock), shmem, st, a, partials);
      break;
    case BDL_NOISE_BUFFER:
      hipLaunchKernelGGL(bdl_sqnorm_kernel<BDL_NOISE_BUFFER>, dim3(grid), dim3(kBlock), shmem, st, a, partials);
      break;
    default:
      hipLaunchKernelGGL(bdl_sqnorm_kernel<BDL_NOISE_PHILOX>, dim3(grid), dim3(kBlock), shmem, st, a, partials);
      break;
  }
  hipLaunchKernelGGL(bdl_clip_finalize_kernel, dim3(1), dim3(kBlock), 0, st, partials, grid, max_norm, ws);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_sgld_step_clipped: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return launch_step(s, ws, st);
}

int bdl_adam_step(const bdl_step_args* s, const bdl_adam_args* ad, void* stream) {
  if (const int rc = no_redirect("bdl_adam_step")) return rc;
  if (!s || !ad) return fail(BDL_ERR_NULL, "bdl_adam_step: null args");
  if (s->method != BDL_ADAM_SGHMC && s->method != BDL_ADAM_SGHMC_GRAD)
    return fail(BDL_ERR_ARG, "bdl_adam_step: method must be BDL_ADAM_SGHMC or BDL_ADAM_SGHMC_GRAD");
  if (s->noise_mode < BDL_NOISE_NONE || s->noise_mode > BDL_NOISE_PHILOX)
    return fail(BDL_ERR_ARG, "bdl_adam_step: unknown noise mode");
  if (s->collect < BDL_COLLECT_NONE || s->collect > BDL_COLLECT_MEAN)
    return fail(BDL_ERR_ARG, "bdl_adam_step: unknown collect mode");
  if (s->n < 0) return fail(BDL_ERR_ARG, "bdl_adam_step: n < 0");
  if (s->n == 0) return BDL_OK;
  const bool grad_only = s->method == BDL_ADAM_SGHMC_GRAD;
  if (!s->theta || !s->mom || !s->prior_mean || !ad->adam_m || !ad->adam_v)
    return fail(BDL_ERR_NULL, "bdl_adam_step: theta, mom, prior_mean, adam_m and adam_v are required");
  if (const int rc = check_runs_and_grad(s, "bdl_adam_step")) return rc;
  if (!grad_only && (s->flags & BDL_FLAG_MOMENTUM) && !ad->sgd_buf)
    return fail(BDL_ERR_NULL, "bdl_adam_step: sgd_buf is required with BDL_FLAG_MOMENTUM");
  if (s->noise_mode == BDL_NOISE_BUFFER && !s->noise)
    return fail(BDL_ERR_NULL, "bdl_adam_step: noise buffer is required");
  if (s->collect != BDL_COLLECT_NONE && !s->mom1)
    return fail(BDL_ERR_NULL, "bdl_adam_step: mom1 is required to collect");
  if (s->flags & BDL_FLAG_GRAD_READY)
    return fail(BDL_ERR_ARG, "bdl_adam_step: GRAD_READY is not an Adam flag (use bdl_sgmcmc_step)");
  const void* ptrs[] = {s->theta, s->mom, s->prior_mean, s->noise, s->mom1, s->mom2,
                        ad->adam_m, ad->adam_v, ad->sgd_buf};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(BDL_ERR_ALIGN, "bdl_adam_step: vector not 16-B aligned");
  const int unroll = grad_only ? 2 : g_unroll;
  StepKernel k = pick_adam(s->noise_mode, s->collect, grad_only, unroll);
  if (!k) return fail(BDL_ERR_ARG, "bdl_adam_step: unsupported noise/collect combination");

  KArgs a{};
  a.theta = s->theta;
  a.grad = s->grad;
  a.mom = s->mom;
  a.prior_mean = s->prior_mean;
  a.noise = s->noise;
  a.mom1 = s->mom1;
  a.mom2 = s->mom2;
  a.runs = s->runs;
  a.gbase = s->grad_base;
  a.nruns = s->nruns;
  a.flags = (s->flags & ~kFlagGradIsMom) | (ad->grad_is_mom ? kFlagGradIsMom : 0);
  a.n = s->n;
  a.lr0 = s->lr[0];
  a.lr1 = s->lr[1];
  a.one_minus_alpha = s->one_minus_alpha;
  a.sigma2 = s->sigma2;
  a.n_data = s->n_data;
  a.mu = s->mu;
  a.ca = s->collect_a;
  a.cb = s->collect_b;
  a.seed = s->seed;
  a.chain = s->chain;
  a.step = s->step;
  a.nonfinite = s->nonfinite;
  a.goff = s->philox_offset;
  a.cgroups = (uint32_t)s->chain_groups;
  a.adam_m = ad->adam_m;
  a.adam_v = ad->adam_v;
  a.sgd_buf = ad->sgd_buf;
  a.b1 = ad->beta1;
  a.omb1 = ad->one_minus_beta1;
  a.b2 = ad->beta2;
  a.omb2 = ad->one_minus_beta2;
  a.bc1 = ad->bias_corr1;
  a.bc2 = ad->bias_corr2;
  a.aeps = ad->eps;
  a.two_alpha = ad->two_alpha;
  a.nd = ad->nd;
  a.temp = ad->temperature;
  a.inv_s2 = recip_or(s->inv_sigma2, s->sigma2);
  a.inv_nd = recip_or(s->inv_n_data, s->n_data);
  a.inv_ca = recip_or(s->inv_collect_a, s->collect_a);
  a.inv_cb = recip_or(s->inv_collect_b, s->collect_b);
  a.inv_temp = recip_or(ad->inv_temperature, ad->temperature);
  a.inv_bc1 = recip_or(ad->inv_bias_corr1, ad->bias_corr1);
  a.inv_bc2 = recip_or(ad->inv_bias_corr2, ad->bias_corr2);
  const int64_t ngroups = (s->n + 3) / 4;
  const int64_t per_iter = (int64_t)kBlock * unroll;
  const int64_t iters = (ngroups + per_iter - 1) / per_iter;
  const int64_t cap = (int64_t)device_cu_count() * g_blocks_per_cu;
  const int grid = (int)std::max<int64_t>(1, std::min(iters, cap));
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), run_lds_bytes(s), (hipStream_t)stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_adam_step: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

int bdl_moments_update(const bdl_moments_args* m, void* stream) {
  if (const int rc = no_redirect("bdl_moments_update")) return rc;
  if (!m) return fail(BDL_ERR_NULL, "bdl_moments_update: null args");
  if (m->n < 0 || m->collect < BDL_COLLECT_WELFORD_INIT || m->collect > BDL_COLLECT_MEAN)
    return fail(BDL_ERR_ARG, "bdl_moments_update: bad n or collect mode");
  if (m->n == 0) return BDL_OK;
  if (!m->theta || !m->mom1) return fail(BDL_ERR_NULL, "bdl_moments_update: theta/mom1 required");
  const void* ptrs[] = {m->theta, m->mom1, m->mom2};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(BDL_ERR_ALIGN, "bdl_moments_update: vector not 16-B aligned");
  MArgs a{m->theta, m->mom1, m->mom2, m->n, m->collect, (m->flags & BDL_FLAG_RECIP_DIV) ? 1 : 0,
          m->collect_a, m->collect_b, recip_or(m->inv_collect_a, m->collect_a),
          recip_or(m->inv_collect_b, m->collect_b)};
  hipLaunchKernelGGL(pick_moments(m->collect, a.recip != 0, m->mom2 != nullptr),
                     dim3(grid_for((m->n + 3) / 4, kBlock * 4)), dim3(kBlock), 0,
                     (hipStream_t)stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_moments_update: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

int bdl_posterior_sample(const bdl_sample_args* s, void* stream) {
  if (const int rc = no_redirect("bdl_posterior_sample")) return rc;
  if (!s) return fail(BDL_ERR_NULL, "bdl_posterior_sample: null args");
  if (s->n < 0 || s->var_mode < BDL_VAR_GIVEN || s->var_mode > BDL_VAR_WELFORD ||
      (s->noise_mode != BDL_NOISE_BUFFER && s->noise_mode != BDL_NOISE_PHILOX))
    return fail(BDL_ERR_ARG, "bdl_posterior_sample: bad arguments");
  if (s->n == 0) return BDL_OK;
  if (!s->out || !s->mom1 || (s->noise_mode == BDL_NOISE_BUFFER && !s->noise))
    return fail(BDL_ERR_NULL, "bdl_posterior_sample: out, mom1 (and noise) required");
  const void* ptrs[] = {s->out, s->mom1, s->mom2, s->noise};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(BDL_ERR_ALIGN, "bdl_posterior_sample: vector not 16-B aligned");
  if (s->chain_groups &&
      (s->chain_groups > 0xFFFFFFFFull || (uint64_t)((s->n + 3) / 4) > 0xFFFFFFFFull))
    return fail(BDL_ERR_ARG, "bdl_posterior_sample: stacked chains need every float4 group "
                "index below 2^32");
  if (s->blocks_per_cu < 0 || s->blocks_per_cu > 8)
    return fail(BDL_ERR_ARG, "bdl_posterior_sample: blocks_per_cu in [0, 8]");
  if (s->unroll != 0 && s->unroll != 1 && s->unroll != 4)
    return fail(BDL_ERR_ARG, "bdl_posterior_sample: unroll 0 (default 4), 1 or 4");
  const int su = s->unroll == 1 ? 1 : 4;
  SArgs a{s->out, s->mom1, s->mom2, s->noise, s->n, s->var_mode, s->noise_mode,
          s->ratio, s->var_floor, s->inv_ratio, s->seed, s->chain, s->step,
          (uint32_t)s->chain_groups};
  const bool floored = s->var_floor >= 0x1p-96f;  // false for NaN
  hipLaunchKernelGGL(pick_sample(s->var_mode, s->mom2 != nullptr, s->inv_ratio != 0.0f,
                                 s->noise_mode, floored, su),
                     dim3(grid_sample((s->n + 3) / 4, s->blocks_per_cu, su)), dim3(kBlock), 0,
                     (hipStream_t)stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_posterior_sample: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

int bdl_stream_mix_schedule(const float* const* reads, int32_t nreads, float* const* writes,
                            int32_t nwrites, int64_t n, int32_t blocks_per_cu, int32_t unroll,
                            int32_t schedule, void* stream) {
  if (const int rc = no_redirect("bdl_stream_mix")) return rc;
  if (!reads || !writes) return fail(BDL_ERR_NULL, "bdl_stream_mix: null stream list");
  if (n < 0 || blocks_per_cu < 1 || blocks_per_cu > 16)
    return fail(BDL_ERR_ARG, "bdl_stream_mix: n >= 0 and blocks_per_cu in [1, 16]");
  if (schedule < BDL_MIX_BARE || schedule > BDL_MIX_PACED)
    return fail(BDL_ERR_ARG, "bdl_stream_mix: schedule is BDL_MIX_BARE, _PIPELINED or _PACED");
  MixKernel k = (nreads <= kMixMaxR && nwrites <= kMixMaxW)
                    ? pick_mix(nreads, nwrites, schedule, unroll)
                    : nullptr;
  if (!k)
    return fail(BDL_ERR_ARG, "bdl_stream_mix: supported (reads, writes): (2,1) (3,2) (4,2) "
                "(3,4) (5,4) (7,5)");
  MixArgs a{};
  for (int i = 0; i < nreads; ++i) {
    if (!reads[i] || !aligned16(reads[i]))
      return fail(BDL_ERR_ALIGN, "bdl_stream_mix: read stream null or not 16-B aligned");
    a.r[i] = reads[i];
  }
  for (int i = 0; i < nwrites; ++i) {
    if (!writes[i] || !aligned16(writes[i]))
      return fail(BDL_ERR_ALIGN, "bdl_stream_mix: write stream null or not 16-B aligned");
    a.w[i] = writes[i];
  }
  a.n = n;
  if (n == 0) return BDL_OK;
  const int u = unroll == 1 || unroll == 4 ? unroll : 2;
  const int64_t ngroups = (n + 3) / 4, per = (int64_t)kBlock * u;
  const int64_t want = (ngroups + per - 1) / per;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)device_cu_count() * blocks_per_cu));
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_stream_mix: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

int bdl_stream_mix(const float* const* reads, int32_t nreads, float* const* writes,
                   int32_t nwrites, int64_t n, int32_t blocks_per_cu, int32_t unroll,
                   void* stream) {
  return bdl_stream_mix_schedule(reads, nreads, writes, nwrites, n, blocks_per_cu, unroll,
                                 BDL_MIX_BARE, stream);
}

int bdl_philox_normal(float* out, int64_t n, uint64_t seed, uint64_t chain, uint64_t step,
                      void* stream) {
  if (const int rc = no_redirect("bdl_philox_normal")) return rc;
  if (n < 0) return fail(BDL_ERR_ARG, "bdl_philox_normal: n < 0");
  if (n == 0) return BDL_OK;
  if (!out) return fail(BDL_ERR_NULL, "bdl_philox_normal: null out");
  if (!aligned16(out)) return fail(BDL_ERR_ALIGN, "bdl_philox_normal: out not 16-B aligned");
  hipLaunchKernelGGL(bdl_philox_kernel, dim3(grid_for((n + 3) / 4, kBlock * 4)), dim3(kBlock), 0,
                     (hipStream_t)stream, out, n, seed, chain, step);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_philox_normal: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}


}  // extern "C"
