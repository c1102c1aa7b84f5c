// bdl_sgmcmc.hip — fused SG-MCMC parameter update for MI355X (gfx950, CDNA4).
//
// One bandwidth-bound sweep over flat fp32 vectors (parameters_to_vector order)
// replaces the reference's per-tensor update loops plus torch.optim.SGD.step()
// plus the thinned posterior-moment accumulation:
//   cSGHMC  methods/csghmc.py:747-778  (+ Welford collect :327-345)
//   SGHMC   methods/sghmc.py:482-510   (+ SGD momentum 0, :229; moments :242-249)
//   SGLD    methods/sgld.py:469-484    (+ SGD momentum mu, :226; moments :239-246)
//   cSGLD   methods/csgld.py:665-680   (+ SGD, :253; per-cycle moments :280-293)
//
// Design:
//   * elementwise, HBM-bound: no LDS on the data stream, no MFMA; 16-B (dwordx4)
//     loads/stores per lane, several independent float4 groups in flight per
//     lane, each workgroup sweeps one contiguous span of the vector.
//   * per-element attributes (lr group, prior on/off, skip) come from a tiny
//     sorted run table; a block finds its first run with a block-uniform
//     (scalar) binary search and each lane advances a cursor monotonically.
//   * noise: either read from a buffer (torch-RNG parity mode) or generated in
//     registers by counter-based Philox4x32-10 keyed by (seed, chain, step,
//     element/4) + Box-Muller on v_log/v_sin/v_cos — no extra HBM traffic.
//   * every floating-point op is rounded separately in the reference's order
//     (compiled with -ffp-contract=off); SGD's add(alpha=-lr) is an explicit
//     fmaf, as torch's CPU kernel computes it.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "bdl_sgmcmc.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* msg) {
  g_last_error = msg;
  return code;
}

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// Tunables (bdl_set_launch_config).  blocks_per_cu * 256 CUs workgroups, each
// lane keeps kUnroll float4 groups in flight per iteration.
// Defaults from the gfx950 sweep (tools/sweep.py, profiles/round1/kernel_v1/sweep_*.log):
// grid-stride with 2 workgroups/CU and 1 float4 group in flight per lane,
// non-temporal 16-B loads and stores, measured best on every kernel kind.
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
// Counter-based RNG: Philox4x32-10 (Salmon et al., SC'11) + Box-Muller.
// counter = (group index lo32, chain lo32, step lo32, step hi32), key = seed.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// uniform in (0, 1): 24 random bits, centred in their bucket -> never 0 or 1.
__device__ __forceinline__ float u01(uint32_t x) {
  return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// Four N(0,1) draws for flat elements 4*group .. 4*group+3.
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v philox_normal4(uint64_t group, uint64_t seed, uint64_t chain,
                                               uint64_t step) {
  const uint4 ctr = make_uint4((uint32_t)group, (uint32_t)chain, (uint32_t)step,
                               (uint32_t)(step >> 32));
  const uint4 r = philox4x32_10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
  // v_log_f32 is log2; v_sin_f32 / v_cos_f32 take the angle in revolutions,
  // so sin(2*pi*u) is one instruction with no range reduction.
  const float kM2Ln2 = -1.38629436111989061883f;  // -2 ln 2
  const float ra = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(r.x)));
  const float rb = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(r.z)));
  const float ta = u01(r.y), tb = u01(r.w);
  f4v z;
  z.x = ra * __builtin_amdgcn_cosf(ta);
  z.y = ra * __builtin_amdgcn_sinf(ta);
  z.z = rb * __builtin_amdgcn_cosf(tb);
  z.w = rb * __builtin_amdgcn_sinf(tb);
  return z;
}

// ---------------------------------------------------------------------------
// Vector helpers: a 16-B "group" covers flat elements [4g, 4g+4).  Only the
// very last group of a vector can be partial; it takes the guarded path.
// ---------------------------------------------------------------------------
// 16-B vector access.  Streaming (non-temporal) policy per direction:
// -DBDL_NT_LOAD / -DBDL_NT_STORE (or -DBDL_NT for both; the default build).
// Every vector is touched once per step and is far larger than the 256 MiB
// Infinity Cache, so nothing is lost by not keeping lines resident.
#ifdef BDL_NT
#define BDL_NT_LOAD 1
#define BDL_NT_STORE 1
#endif
__device__ __forceinline__ f4v vload(const float* p) {
#ifdef BDL_NT_LOAD
  return __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
#else
  return *reinterpret_cast<const f4v*>(p);
#endif
}

__device__ __forceinline__ void vstore(float* p, f4v v) {
#ifdef BDL_NT_STORE
  __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
#else
  *reinterpret_cast<f4v*>(p) = v;
#endif
}

__device__ __forceinline__ f4v ld4(const float* __restrict__ p, int64_t e, int64_t n) {
  if (e + 4 <= n) return vload(p + e);
  f4v v = {0.f, 0.f, 0.f, 0.f};
  if (e + 0 < n) v.x = p[e + 0];
  if (e + 1 < n) v.y = p[e + 1];
  if (e + 2 < n) v.z = p[e + 2];
  return v;
}

__device__ __forceinline__ void st4(float* __restrict__ p, int64_t e, int64_t n, f4v v) {
  if (e + 4 <= n) {
    vstore(p + e, v);
    return;
  }
  if (e + 0 < n) p[e + 0] = v.x;
  if (e + 1 < n) p[e + 1] = v.y;
  if (e + 2 < n) p[e + 2] = v.z;
}

struct KArgs {
  float* __restrict__ theta;
  float* __restrict__ grad;
  float* __restrict__ mom;
  const float* __restrict__ prior_mean;
  const float* __restrict__ noise;
  float* __restrict__ mom1;
  float* __restrict__ mom2;
  const bdl_run* __restrict__ runs;
  int32_t nruns;
  int32_t flags;
  int64_t n;
  int64_t groups_per_block;
  float lr0, lr1, ns0, ns1;
  float one_minus_alpha, prior_sig, sigma2, n_data, mu, ca, cb;
  uint64_t seed, chain, step;
  const float* __restrict__ clip;  // (total_norm, coef) from the clip finalize, or null
  // Adam-preconditioned SGHMC only (bdl_adam_step)
  float* __restrict__ adam_m;
  float* __restrict__ adam_v;
  float* __restrict__ sgd_buf;
  float b1, omb1, b2, omb2, bc1, bc2, aeps, two_alpha, nd, temp;
  // scalar-divisor reciprocals for BDL_FLAG_RECIP_DIV (host-rounded fl32(1/s64))
  float inv_s2, inv_nd, inv_ca, inv_cb, inv_temp, inv_bc1, inv_bc2;
};

// fl32(1/s64) from the caller, or 1/fl32(s) when it left the field 0
inline float recip_or(float inv, float s) { return inv != 0.0f ? inv : 1.0f / s; }

constexpr int32_t kFlagGradIsMom = 0x1000;  // internal: bdl_adam_args.grad_is_mom

// Scalar division in the reference's rounding: torch CPU divides (x / s);
// torch on a HIP device multiplies by the fp32 reciprocal (x * fl(1/s)).
template <bool RECIP>
__device__ __forceinline__ float sdiv(float x, float s, float inv_s) {
  if constexpr (RECIP)
    return x * inv_s;
  else
    return x / s;
}

// ---------------------------------------------------------------------------
// Run table staged in LDS (dynamic, 16 B per run, sized per launch).  The fast
// path reads the block-uniform attribute of its iteration from LDS, so the
// wait for it is an lgkmcnt wait and never sits behind the data stream's
// in-order vmcnt.
// ---------------------------------------------------------------------------
constexpr int kMaxRuns = 4096;  // 64 KiB of LDS

extern __shared__ bdl_run s_runs[];

__device__ __forceinline__ int64_t run_end(int r) { return s_runs[r].end; }
__device__ __forceinline__ uint32_t run_attr(int r) { return s_runs[r].attr; }

// First run whose end is > idx.
__device__ __forceinline__ int find_run_lds(int nruns, int64_t idx) {
  int lo = 0, hi = nruns - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (run_end(mid) <= idx)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

struct StepConst {
  bool sgd_mom, sgd_mom_read, has_m2, grad_ready, clip;
  float inv_s2, inv_nd, inv_ca, inv_cb, clip_coef;
};

// ---------------------------------------------------------------------------
// Per-element update.  All arithmetic is separately rounded fp32 in exactly
// the reference's op order (the file is compiled with -ffp-contract=off).
// eta / ns are the element's lr and noise scale (its lr group), PRIOR whether
// the Gaussian-prior term applies, GR = grad already formed (SGD step only).
// ---------------------------------------------------------------------------
template <int METHOD, int NOISE, bool RECIP, bool PRIOR, bool GR>
__device__ __forceinline__ void update_core(const KArgs& a, const StepConst& c, float eta,
                                            float ns, float& th, float& g, float& v, float th0,
                                            float eps) {
  if constexpr (GR) {
    // the sampler gradient was formed (and possibly clipped) by a previous
    // *_GRAD launch: only torch.optim.SGD's step remains
    float stepv = g;
    if (METHOD == BDL_SGLD && c.sgd_mom) {
      v = (a.flags & BDL_FLAG_FIRST_STEP) ? g : (a.mu * v + g);
      stepv = v;
    }
    th = fmaf(-eta, stepv, th);
  } else if constexpr (METHOD == BDL_CSGHMC) {
    // csghmc.py:759-762 — both branches are grad + prior_sig * theta (Q1)
    const float t = a.prior_sig * th;
    const float gU = g + t;
    const float x = v * a.one_minus_alpha;  // :770 v*(1-a)
    const float y = eta * gU;               //      lr*grad_U
    float vn = x - y;
    if constexpr (NOISE != BDL_NOISE_NONE) vn = vn + ns * eps;  // + noise (:765-770)
    v = vn;                                 // :775
    th = th + vn;                           // :778 p.data.add_(v)
  } else if constexpr (METHOD == BDL_SGHMC || METHOD == BDL_SGHMC_GRAD) {
    float gU = g;  // sghmc.py:494-497
    if constexpr (PRIOR) {
      const float d = th - th0;
      const float e = sdiv<RECIP>(d, a.sigma2, c.inv_s2);
      gU = g + sdiv<RECIP>(e, a.n_data, c.inv_nd);
    }
    const float s = v * a.one_minus_alpha + eta * gU;  // :504 (two products rounded)
    const float vn = s + ns * eps;
    const float gp = g + vn;  // :510 p.grad = p.grad + v
    v = vn;
    if constexpr (METHOD == BDL_SGHMC)
      th = fmaf(-eta, gp, th);  // SGD(momentum=0): param.add_(grad, alpha=-lr)
    else
      g = gp;
  } else {  // BDL_SGLD / BDL_SGLD_GRAD  (sgld.py:471-484)
    const float nz = ns * eps;
    float gp;
    if constexpr (PRIOR) {
      const float d = th - th0;
      const float e = sdiv<RECIP>(d, a.sigma2, c.inv_s2);
      const float f = sdiv<RECIP>(e, a.n_data, c.inv_nd);
      gp = g + (f + nz);
    } else {
      gp = g + nz;
    }
    if constexpr (METHOD == BDL_SGLD) {
      if (c.clip) gp = gp * c.clip_coef;  // clip_grad_norm_: grads.mul_(clip_coef_clamped)
      float stepv = gp;
      if (c.sgd_mom) {  // torch SGD momentum buffer
        v = (a.flags & BDL_FLAG_FIRST_STEP) ? gp : (a.mu * v + gp);
        stepv = v;
      }
      th = fmaf(-eta, stepv, th);
    } else {
      g = gp;
    }
  }
}

// Posterior moments on the updated theta (parameters_to_vector after step).
template <int COLLECT, bool RECIP>
__device__ __forceinline__ void collect_core(const KArgs& a, const StepConst& c, float th,
                                             float& m1, float& m2) {
  if constexpr (COLLECT == BDL_COLLECT_WELFORD_INIT) {
    m1 = th;
    m2 = 0.0f;
  } else if constexpr (COLLECT == BDL_COLLECT_WELFORD) {
    const float d = th - m1;
    m1 = m1 + sdiv<RECIP>(d, a.ca, c.inv_ca);
    const float d2 = th - m1;
    m2 = m2 + d * d2;
  } else if constexpr (COLLECT == BDL_COLLECT_MEAN_INIT) {
    m1 = th;
    m2 = th * th;
  } else if constexpr (COLLECT == BDL_COLLECT_MEAN) {
    m1 = sdiv<RECIP>(th + a.ca * m1, a.cb, c.inv_cb);
    m2 = sdiv<RECIP>(th * th + a.ca * m2, a.cb, c.inv_cb);
  }
}

// Per-kernel constants of a method / collect combination.
template <int METHOD, int COLLECT>
struct StepTraits {
  static constexpr bool kReadPrior = (METHOD != BDL_CSGHMC);
  static constexpr bool kMom =
      (METHOD == BDL_CSGHMC || METHOD == BDL_SGHMC || METHOD == BDL_SGHMC_GRAD);
  static constexpr bool kWriteTheta =
      (METHOD == BDL_CSGHMC || METHOD == BDL_SGHMC || METHOD == BDL_SGLD);
  static constexpr bool kWriteGrad = (METHOD == BDL_SGHMC_GRAD || METHOD == BDL_SGLD_GRAD);
  static constexpr bool kCollect = (COLLECT != BDL_COLLECT_NONE);
  static constexpr bool kReadMoments =
      (COLLECT == BDL_COLLECT_WELFORD || COLLECT == BDL_COLLECT_MEAN);
};

// FAST PATH: a whole block-iteration (kBlock*UNROLL float4 groups) in range
// and inside one non-skip run.  eta / ns are scalars, PRIOR / GR compile-time:
// no branch inside, no bounds checks, every load issued before any arithmetic.
template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL, bool PRIOR, bool GR>
__device__ __forceinline__ void chunk_fast(const KArgs& a, const StepConst& c, int64_t gb,
                                           float eta, float ns) {
  using T = StepTraits<METHOD, COLLECT>;
  constexpr bool kPriorLoad = T::kReadPrior && PRIOR && !GR;
  f4v th[UNROLL], g[UNROLL], v[UNROLL], t0[UNROLL], ep[UNROLL], m1[UNROLL], m2[UNROLL];
  const f4v z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
    v[u] = t0[u] = ep[u] = m1[u] = m2[u] = z;
    th[u] = vload(a.theta + e);
    g[u] = vload(a.grad + e);
    if constexpr (T::kMom) v[u] = vload(a.mom + e);
    if constexpr (METHOD == BDL_SGLD) {
      if (c.sgd_mom_read) v[u] = vload(a.mom + e);
    }
    if constexpr (kPriorLoad) t0[u] = vload(a.prior_mean + e);
    if constexpr (NOISE == BDL_NOISE_BUFFER && !GR) ep[u] = vload(a.noise + e);
    if constexpr (T::kReadMoments) {
      m1[u] = vload(a.mom1 + e);
      if (c.has_m2) m2[u] = vload(a.mom2 + e);
    }
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    if constexpr (NOISE == BDL_NOISE_PHILOX && !GR)
      ep[u] = philox_normal4((uint64_t)gi, a.seed, a.chain, a.step);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xt = th[u][j], xg = g[u][j], xv = v[u][j], x1 = m1[u][j], x2 = m2[u][j];
      update_core<METHOD, NOISE, RECIP, PRIOR, GR>(a, c, eta, ns, xt, xg, xv, t0[u][j], ep[u][j]);
      collect_core<COLLECT, RECIP>(a, c, xt, x1, x2);
      th[u][j] = xt;
      g[u][j] = xg;
      v[u][j] = xv;
      m1[u][j] = x1;
      m2[u][j] = x2;
    }
    if constexpr (T::kWriteTheta) vstore(a.theta + e, th[u]);
    if constexpr (T::kWriteGrad) vstore(a.grad + e, g[u]);
    if constexpr (T::kMom) vstore(a.mom + e, v[u]);
    if constexpr (METHOD == BDL_SGLD) {
      if (c.sgd_mom) vstore(a.mom + e, v[u]);
    }
    if constexpr (T::kCollect) {
      vstore(a.mom1 + e, m1[u]);
      if (c.has_m2) vstore(a.mom2 + e, m2[u]);
    }
  }
}

template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL>
__device__ __forceinline__ void chunk_fast_dispatch(const KArgs& a, const StepConst& c,
                                                    int64_t gb, uint32_t attr) {
  const bool head = (attr & BDL_ATTR_HEAD) != 0;
  const float eta = head ? a.lr1 : a.lr0;
  const float ns = head ? a.ns1 : a.ns0;
  if constexpr (METHOD == BDL_CSGHMC) {
    chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, false, false>(a, c, gb, eta, ns);
  } else {
    if constexpr (METHOD == BDL_SGLD || METHOD == BDL_SGHMC) {
      if (c.grad_ready) {
        chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, false, true>(a, c, gb, eta, ns);
        return;
      }
    }
    if (attr & BDL_ATTR_PRIOR)
      chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, true, false>(a, c, gb, eta, ns);
    else
      chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, false, false>(a, c, gb, eta, ns);
  }
}

// Element-wise update for the slow path: attribute-dependent branches allowed.
template <int METHOD, int NOISE, int COLLECT, bool RECIP>
__device__ __forceinline__ void update_elem(const KArgs& a, const StepConst& c, uint32_t attr,
                                            float& th, float& g, float& v, float th0, float eps,
                                            float& m1, float& m2) {
  const bool head = (attr & BDL_ATTR_HEAD) != 0;
  const float eta = head ? a.lr1 : a.lr0;
  const float ns = head ? a.ns1 : a.ns0;
  if (!(attr & BDL_ATTR_SKIP)) {
    if ((METHOD == BDL_SGLD || METHOD == BDL_SGHMC) && c.grad_ready) {
      if constexpr (METHOD == BDL_SGLD || METHOD == BDL_SGHMC)
        update_core<METHOD, NOISE, RECIP, false, true>(a, c, eta, ns, th, g, v, th0, eps);
    } else if (attr & BDL_ATTR_PRIOR) {
      update_core<METHOD, NOISE, RECIP, true, false>(a, c, eta, ns, th, g, v, th0, eps);
    } else {
      update_core<METHOD, NOISE, RECIP, false, false>(a, c, eta, ns, th, g, v, th0, eps);
    }
  }
  collect_core<COLLECT, RECIP>(a, c, th, m1, m2);
}

// SLOW PATH: an iteration that reaches the end of the vector / span, crosses a
// run boundary or covers a skipped parameter.  Per-lane predicates, guarded
// partial groups, a per-element run search (in LDS).  Taken for
// O(#runs + #blocks) iterations per launch.
template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL>
__device__ __forceinline__ void chunk_slow(const KArgs& a, const StepConst& c, int64_t gb,
                                           int64_t gend) {
  using T = StepTraits<METHOD, COLLECT>;
  const int64_t n = a.n;
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    if (gi >= gend) continue;
    const int64_t e = gi * 4;
    const f4v z = {0.f, 0.f, 0.f, 0.f};
    f4v th = ld4(a.theta, e, n), g = ld4(a.grad, e, n), v = z, t0 = z, ep = z, m1 = z, m2 = z;
    if (T::kMom || (METHOD == BDL_SGLD && c.sgd_mom_read)) v = ld4(a.mom, e, n);
    if (T::kReadPrior) t0 = ld4(a.prior_mean, e, n);
    if (NOISE == BDL_NOISE_BUFFER) ep = ld4(a.noise, e, n);
    if (NOISE == BDL_NOISE_PHILOX) ep = philox_normal4((uint64_t)gi, a.seed, a.chain, a.step);
    if (T::kReadMoments) {
      m1 = ld4(a.mom1, e, n);
      if (c.has_m2) m2 = ld4(a.mom2, e, n);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (e + j >= n) break;
      const uint32_t at = run_attr(find_run_lds(a.nruns, e + j));
      float xt = th[j], xg = g[j], xv = v[j], x1 = m1[j], x2 = m2[j];
      update_elem<METHOD, NOISE, COLLECT, RECIP>(a, c, at, xt, xg, xv, t0[j], ep[j], x1, x2);
      th[j] = xt;
      g[j] = xg;
      v[j] = xv;
      m1[j] = x1;
      m2[j] = x2;
    }
    if (T::kWriteTheta) st4(a.theta, e, n, th);
    if (T::kWriteGrad) st4(a.grad, e, n, g);
    if (T::kMom || (METHOD == BDL_SGLD && c.sgd_mom)) st4(a.mom, e, n, v);
    if (T::kCollect) {
      st4(a.mom1, e, n, m1);
      if (c.has_m2) st4(a.mom2, e, n, m2);
    }
  }
}

template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL>
__device__ __forceinline__ void step_body(const KArgs& a) {
  StepConst c;
  c.sgd_mom = (METHOD == BDL_SGLD) && (a.flags & BDL_FLAG_MOMENTUM);
  c.sgd_mom_read = c.sgd_mom && !(a.flags & BDL_FLAG_FIRST_STEP);
  c.has_m2 = (COLLECT != BDL_COLLECT_NONE) && (a.mom2 != nullptr);
  c.grad_ready = (METHOD == BDL_SGLD || METHOD == BDL_SGHMC) && (a.flags & BDL_FLAG_GRAD_READY);
  c.clip = (METHOD == BDL_SGLD) && a.clip != nullptr;
  c.clip_coef = c.clip ? a.clip[1] : 1.0f;
  c.inv_s2 = a.inv_s2;
  c.inv_nd = a.inv_nd;
  c.inv_ca = a.inv_ca;
  c.inv_cb = a.inv_cb;

  const int64_t ngroups = (a.n + 3) >> 2;
  const int64_t nfull = a.n >> 2;  // groups entirely inside [0, n)
  // Two sweep orders: each block owns one contiguous span (groups_per_block >
  // 0), or all blocks advance through the vector together (grid-stride,
  // groups_per_block == 0).  Either way the block's iterations only move
  // forward, so its (block-uniform) run cursor advances monotonically.
  constexpr int64_t kIter = (int64_t)kBlock * UNROLL;
  int64_t g0, g1, gstep;
  if (a.groups_per_block > 0) {
    g0 = (int64_t)blockIdx.x * a.groups_per_block;
    g1 = min(g0 + a.groups_per_block, ngroups);
    gstep = kIter;
  } else {
    g0 = (int64_t)blockIdx.x * kIter;
    g1 = ngroups;
    gstep = (int64_t)gridDim.x * kIter;
  }

  // stage the run table in LDS
  for (int i = threadIdx.x; i < a.nruns; i += kBlock) s_runs[i] = a.runs[i];
  __syncthreads();
  if (g0 >= g1) return;

  int r = find_run_lds(a.nruns, g0 * 4);
  for (int64_t gb = g0; gb < g1; gb += gstep) {
    while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
    const int64_t gend = min(gb + kIter, g1);
    const uint32_t attr = run_attr(r);
    if (gend == gb + kIter && gend <= nfull && run_end(r) >= gend * 4 &&
        !(attr & BDL_ATTR_SKIP))
      chunk_fast_dispatch<METHOD, NOISE, COLLECT, RECIP, UNROLL>(a, c, gb, attr);
    else
      chunk_slow<METHOD, NOISE, COLLECT, RECIP, UNROLL>(a, c, gb, gend);
  }
}

template <int METHOD, int NOISE, int COLLECT, int UNROLL>
__global__ __launch_bounds__(kBlock) void bdl_step_kernel(const KArgs a) {
  if (a.flags & BDL_FLAG_RECIP_DIV)
    step_body<METHOD, NOISE, COLLECT, true, UNROLL>(a);
  else
    step_body<METHOD, NOISE, COLLECT, false, UNROLL>(a);
}

// ---------------------------------------------------------------------------
// Adam-preconditioned SGHMC (methods/adam_sghmc.py:500-553,
// methods/adam_csghmc.py:812-860) + torch.optim.SGD step + running moments.
// Same sweep as the SG-MCMC step (run table in LDS, branch-free fast path over
// whole iterations inside one run, guarded slow path elsewhere); the element
// update carries three more state vectors (v_mom in args.mom, Adam m and v) and
// optionally the SGD buffer: 40 B/element, 48 with the buffer.
// ---------------------------------------------------------------------------
struct AdamConst {
  bool sgd_mom, sgd_mom_read, has_m2, grad_is_mom;
  float inv_s2, inv_nd, inv_temp, inv_bc1, inv_bc2, inv_ca, inv_cb;
};

template <int NOISE, bool RECIP, bool PRIOR, bool GRADONLY>
__device__ __forceinline__ void adam_core(const KArgs& a, const AdamConst& c, float eta, float& th,
                                          float& g, float& vm, float& m, float& v, float& buf,
                                          float th0, float eps) {
  const float gs = sdiv<RECIP>(g, a.temp, c.inv_temp);  // p.grad / temperature
  float gU = gs;
  if constexpr (PRIOR) {
    const float d = th - th0;
    const float e = sdiv<RECIP>(d, a.sigma2, c.inv_s2);
    gU = gs + sdiv<RECIP>(e, a.n_data, c.inv_nd);
  }
  m = m * a.b1 + gU * a.omb1;            // beta1*m + (1-beta1)*grad_U
  v = v * a.b2 + (gU * gU) * a.omb2;     // beta2*v + (1-beta2)*(grad_U*grad_U)
  const float mh = sdiv<RECIP>(m, a.bc1, c.inv_bc1);
  const float vh = sdiv<RECIP>(v, a.bc2, c.inv_bc2);
  const float den = sqrtf(vh) + a.aeps;  // torch.sqrt(v_hat) + eps
  const float pg = mh / den;             // precond_grad (tensor / tensor: true division)
  const float pt = 1.0f / den;           // precond_term = 1.0 / (...) = reciprocal() * 1.0
  float nz = 0.0f;
  if constexpr (NOISE != BDL_NOISE_NONE) {
    const float q = sdiv<RECIP>(pt * a.two_alpha, a.n_data, c.inv_nd);
    nz = (sqrtf(q) * a.nd) * eps;        // nd*sqrt(2a*pt/N) * randn_like
  }
  vm = (vm * a.one_minus_alpha + pg * eta) + nz;
  const float gp = c.grad_is_mom ? vm : g + vm;  // p.grad = v_mom (.clone()) | p.grad + v_mom
  if constexpr (GRADONLY) {
    g = gp;
  } else {
    float stepv = gp;
    if (c.sgd_mom) {
      buf = (a.flags & BDL_FLAG_FIRST_STEP) ? gp : (a.mu * buf + gp);
      stepv = buf;
    }
    th = fmaf(-eta, stepv, th);  // SGD: param.add_(d_p, alpha=-lr)
  }
}

template <int NOISE, int COLLECT, bool RECIP, bool GRADONLY, bool PRIOR, int U>
__device__ __forceinline__ void adam_fast(const KArgs& a, const AdamConst& c, int64_t gb,
                                          float eta) {
  constexpr bool kReadMoments = (COLLECT == BDL_COLLECT_MEAN);
  const f4v z = {0.f, 0.f, 0.f, 0.f};
  f4v th[U], g[U], vm[U], m[U], v[U], buf[U], t0[U], ep[U], m1[U], m2[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
    buf[u] = t0[u] = ep[u] = m1[u] = m2[u] = z;
    th[u] = vload(a.theta + e);
    g[u] = vload(a.grad + e);
    vm[u] = vload(a.mom + e);
    m[u] = vload(a.adam_m + e);
    v[u] = vload(a.adam_v + e);
    if (!GRADONLY && c.sgd_mom_read) buf[u] = vload(a.sgd_buf + e);
    if constexpr (PRIOR) t0[u] = vload(a.prior_mean + e);
    if constexpr (NOISE == BDL_NOISE_BUFFER) ep[u] = vload(a.noise + e);
    if constexpr (kReadMoments) {
      m1[u] = vload(a.mom1 + e);
      if (c.has_m2) m2[u] = vload(a.mom2 + e);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    if constexpr (NOISE == BDL_NOISE_PHILOX) ep[u] = philox_normal4((uint64_t)gi, a.seed, a.chain, a.step);
    StepConst cc;  // collect_core only reads inv_ca / inv_cb
    cc.inv_ca = c.inv_ca;
    cc.inv_cb = c.inv_cb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xt = th[u][j], xg = g[u][j], xvm = vm[u][j], xm = m[u][j], xv = v[u][j],
            xb = buf[u][j], x1 = m1[u][j], x2 = m2[u][j];
      adam_core<NOISE, RECIP, PRIOR, GRADONLY>(a, c, eta, xt, xg, xvm, xm, xv, xb, t0[u][j],
                                               ep[u][j]);
      collect_core<COLLECT, RECIP>(a, cc, xt, x1, x2);
      th[u][j] = xt;
      g[u][j] = xg;
      vm[u][j] = xvm;
      m[u][j] = xm;
      v[u][j] = xv;
      buf[u][j] = xb;
      m1[u][j] = x1;
      m2[u][j] = x2;
    }
    if constexpr (GRADONLY)
      vstore(a.grad + e, g[u]);
    else
      vstore(a.theta + e, th[u]);
    vstore(a.mom + e, vm[u]);
    vstore(a.adam_m + e, m[u]);
    vstore(a.adam_v + e, v[u]);
    if (!GRADONLY && c.sgd_mom) vstore(a.sgd_buf + e, buf[u]);
    if constexpr (COLLECT != BDL_COLLECT_NONE) {
      vstore(a.mom1 + e, m1[u]);
      if (c.has_m2) vstore(a.mom2 + e, m2[u]);
    }
  }
}

template <int NOISE, int COLLECT, bool RECIP, bool GRADONLY, int U>
__device__ __forceinline__ void adam_slow(const KArgs& a, const AdamConst& c, int64_t gb,
                                          int64_t gend) {
  const int64_t n = a.n;
  const f4v z = {0.f, 0.f, 0.f, 0.f};
  StepConst cc;
  cc.inv_ca = c.inv_ca;
  cc.inv_cb = c.inv_cb;
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    if (gi >= gend) continue;
    const int64_t e = gi * 4;
    f4v th = ld4(a.theta, e, n), g = ld4(a.grad, e, n), vm = ld4(a.mom, e, n);
    f4v m = ld4(a.adam_m, e, n), v = ld4(a.adam_v, e, n), t0 = ld4(a.prior_mean, e, n);
    f4v buf = z, ep = z, m1 = z, m2 = z;
    if (!GRADONLY && c.sgd_mom_read) buf = ld4(a.sgd_buf, e, n);
    if (NOISE == BDL_NOISE_BUFFER) ep = ld4(a.noise, e, n);
    if (NOISE == BDL_NOISE_PHILOX) ep = philox_normal4((uint64_t)gi, a.seed, a.chain, a.step);
    if (COLLECT == BDL_COLLECT_MEAN) {
      m1 = ld4(a.mom1, e, n);
      if (c.has_m2) m2 = ld4(a.mom2, e, n);
    }
    for (int j = 0; j < 4; ++j) {
      if (e + j >= n) break;
      const uint32_t at = run_attr(find_run_lds(a.nruns, e + j));
      float xt = th[j], xg = g[j], xvm = vm[j], xm = m[j], xv = v[j], xb = buf[j];
      float x1 = m1[j], x2 = m2[j];
      if (!(at & BDL_ATTR_SKIP)) {
        const float eta = (at & BDL_ATTR_HEAD) ? a.lr1 : a.lr0;
        if (at & BDL_ATTR_PRIOR)
          adam_core<NOISE, RECIP, true, GRADONLY>(a, c, eta, xt, xg, xvm, xm, xv, xb, t0[j], ep[j]);
        else
          adam_core<NOISE, RECIP, false, GRADONLY>(a, c, eta, xt, xg, xvm, xm, xv, xb, t0[j], ep[j]);
      }
      collect_core<COLLECT, RECIP>(a, cc, xt, x1, x2);
      th[j] = xt;
      g[j] = xg;
      vm[j] = xvm;
      m[j] = xm;
      v[j] = xv;
      buf[j] = xb;
      m1[j] = x1;
      m2[j] = x2;
    }
    if (GRADONLY)
      st4(a.grad, e, n, g);
    else
      st4(a.theta, e, n, th);
    st4(a.mom, e, n, vm);
    st4(a.adam_m, e, n, m);
    st4(a.adam_v, e, n, v);
    if (!GRADONLY && c.sgd_mom) st4(a.sgd_buf, e, n, buf);
    if (COLLECT != BDL_COLLECT_NONE) {
      st4(a.mom1, e, n, m1);
      if (c.has_m2) st4(a.mom2, e, n, m2);
    }
  }
}

template <int NOISE, int COLLECT, bool RECIP, bool GRADONLY, int U>
__device__ __forceinline__ void adam_body(const KArgs& a) {
  AdamConst c;
  c.sgd_mom = !GRADONLY && (a.flags & BDL_FLAG_MOMENTUM);
  c.sgd_mom_read = c.sgd_mom && !(a.flags & BDL_FLAG_FIRST_STEP);
  c.has_m2 = (COLLECT != BDL_COLLECT_NONE) && (a.mom2 != nullptr);
  c.grad_is_mom = (a.flags & kFlagGradIsMom) != 0;
  c.inv_s2 = a.inv_s2;
  c.inv_nd = a.inv_nd;
  c.inv_temp = a.inv_temp;
  c.inv_bc1 = a.inv_bc1;
  c.inv_bc2 = a.inv_bc2;
  c.inv_ca = a.inv_ca;
  c.inv_cb = a.inv_cb;
  constexpr int64_t kIter = (int64_t)kBlock * U;
  const int64_t ngroups = (a.n + 3) >> 2, nfull = a.n >> 2;
  for (int i = threadIdx.x; i < a.nruns; i += kBlock) s_runs[i] = a.runs[i];
  __syncthreads();
  int r = find_run_lds(a.nruns, (int64_t)blockIdx.x * kIter * 4);
  for (int64_t gb = (int64_t)blockIdx.x * kIter; gb < ngroups; gb += (int64_t)gridDim.x * kIter) {
    while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
    const int64_t gend = min(gb + kIter, ngroups);
    const uint32_t attr = run_attr(r);
    if (gend == gb + kIter && gend <= nfull && run_end(r) >= gend * 4 && !(attr & BDL_ATTR_SKIP)) {
      const float eta = (attr & BDL_ATTR_HEAD) ? a.lr1 : a.lr0;
      if (attr & BDL_ATTR_PRIOR)
        adam_fast<NOISE, COLLECT, RECIP, GRADONLY, true, U>(a, c, gb, eta);
      else
        adam_fast<NOISE, COLLECT, RECIP, GRADONLY, false, U>(a, c, gb, eta);
    } else {
      adam_slow<NOISE, COLLECT, RECIP, GRADONLY, U>(a, c, gb, gend);
    }
  }
}

template <int NOISE, int COLLECT, bool GRADONLY, int U>
__global__ __launch_bounds__(kBlock) void bdl_adam_kernel(const KArgs a) {
  if (a.flags & BDL_FLAG_RECIP_DIV)
    adam_body<NOISE, COLLECT, true, GRADONLY, U>(a);
  else
    adam_body<NOISE, COLLECT, false, GRADONLY, U>(a);
}

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
                                              float ns, double acc) {
  constexpr int U = 2;
  f4v th[U], g[U], t0[U], ep[U];
  const f4v z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
    t0[u] = ep[u] = z;
    th[u] = vload(a.theta + e);
    g[u] = vload(a.grad + e);
    if constexpr (PRIOR) t0[u] = vload(a.prior_mean + e);
    if constexpr (NOISE == BDL_NOISE_BUFFER) ep[u] = vload(a.noise + e);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    if constexpr (NOISE == BDL_NOISE_PHILOX) ep[u] = philox_normal4((uint64_t)gi, a.seed, a.chain, a.step);
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
  for (int i = threadIdx.x; i < a.nruns; i += kBlock) s_runs[i] = a.runs[i];
  __syncthreads();
  double acc = 0.0;
  int r = find_run_lds(a.nruns, (int64_t)blockIdx.x * kIter * 4);
  for (int64_t gb = (int64_t)blockIdx.x * kIter; gb < ngroups; gb += (int64_t)gridDim.x * kIter) {
    while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
    const int64_t gend = min(gb + kIter, ngroups);
    const uint32_t attr = run_attr(r);
    if (gend == gb + kIter && gend <= nfull && run_end(r) >= gend * 4 && !(attr & BDL_ATTR_SKIP)) {
      const float ns = (attr & BDL_ATTR_HEAD) ? a.ns1 : a.ns0;
      if (attr & BDL_ATTR_PRIOR)
        acc = sqnorm_fast<NOISE, RECIP, true>(a, c, gb, ns, acc);
      else
        acc = sqnorm_fast<NOISE, RECIP, false>(a, c, gb, ns, acc);
    } else {
      for (int u = 0; u < 2; ++u) {
        const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
        if (gi >= gend) continue;
        const int64_t e = gi * 4;
        const f4v z = {0.f, 0.f, 0.f, 0.f};
        const f4v th = ld4(a.theta, e, a.n), g = ld4(a.grad, e, a.n);
        const f4v t0 = ld4(a.prior_mean, e, a.n);
        f4v ep = z;
        if (NOISE == BDL_NOISE_BUFFER) ep = ld4(a.noise, e, a.n);
        if (NOISE == BDL_NOISE_PHILOX) ep = philox_normal4((uint64_t)gi, a.seed, a.chain, a.step);
        for (int j = 0; j < 4; ++j) {
          if (e + j >= a.n) break;
          const uint32_t at = run_attr(find_run_lds(a.nruns, e + j));
          if (at & BDL_ATTR_SKIP) continue;  // .grad is None: not in the norm
          float xt = th[j], xg = g[j], xv = 0.f;
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

__global__ __launch_bounds__(kBlock) void bdl_moments_kernel(const MArgs a) {
  const int64_t ngroups = (a.n + 3) >> 2;
  const float inv_ca = a.inv_ca, inv_cb = a.inv_cb;
  for (int64_t gi = (int64_t)blockIdx.x * kBlock + threadIdx.x; gi < ngroups;
       gi += (int64_t)gridDim.x * kBlock) {
    const int64_t e = gi * 4;
    const f4v t = ld4(a.theta, e, a.n);
    f4v m1 = {0.f, 0.f, 0.f, 0.f}, m2 = m1;
    if (a.collect == BDL_COLLECT_WELFORD || a.collect == BDL_COLLECT_MEAN) {
      m1 = ld4(a.mom1, e, a.n);
      if (a.mom2) m2 = ld4(a.mom2, e, a.n);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = t[j];
      float p = m1[j], q = m2[j];
      switch (a.collect) {
        case BDL_COLLECT_WELFORD_INIT:
          p = x;
          q = 0.f;
          break;
        case BDL_COLLECT_WELFORD: {
          const float d = x - p;
          p = p + (a.recip ? d * inv_ca : d / a.ca);
          const float d2 = x - p;
          q = q + d * d2;
          break;
        }
        case BDL_COLLECT_MEAN_INIT:
          p = x;
          q = x * x;
          break;
        default: {  // MEAN
          const float u = x + a.ca * p;
          p = a.recip ? u * inv_cb : u / a.cb;
          const float w = x * x + a.ca * q;
          q = a.recip ? w * inv_cb : w / a.cb;
        }
      }
      m1[j] = p;
      m2[j] = q;
    }
    st4(a.mom1, e, a.n, m1);
    if (a.mom2) st4(a.mom2, e, a.n, m2);
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
};

__global__ __launch_bounds__(kBlock) void bdl_sample_kernel(const SArgs a) {
  const int64_t ngroups = (a.n + 3) >> 2;
  for (int64_t gi = (int64_t)blockIdx.x * kBlock + threadIdx.x; gi < ngroups;
       gi += (int64_t)gridDim.x * kBlock) {
    const int64_t e = gi * 4;
    const f4v m = ld4(a.mom1, e, a.n);
    f4v q = {0.f, 0.f, 0.f, 0.f};
    if (a.mom2) q = ld4(a.mom2, e, a.n);
    const f4v eps = (a.noise_mode == BDL_NOISE_BUFFER)
                        ? ld4(a.noise, e, a.n)
                        : philox_normal4((uint64_t)gi, a.seed, a.chain, a.step);
    f4v o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float mj = m[j];
      const float qj = q[j];
      float var;
      if (!a.mom2)
        var = a.var_floor;  // single-sample cycle: ones*1e-12 (csghmc.py:456-458)
      else if (a.var_mode == BDL_VAR_RAW_MOMENTS)
        var = a.ratio * (qj - mj * mj);  // sgld.py:342
      else if (a.var_mode == BDL_VAR_WELFORD)
        var = a.inv_ratio != 0.0f ? qj * a.inv_ratio : qj / a.ratio;  // csghmc.py:455
      else
        var = qj;
      if (!(var != var)) var = fmaxf(var, a.var_floor);  // clamp_(min=1e-12); NaN stays NaN
      o[j] = mj + sqrtf(var) * eps[j];  // p_m + p_v.sqrt()*eps
    }
    st4(a.out, e, a.n, o);
  }
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

// ---------------------------------------------------------------------------
// Dispatch
// ---------------------------------------------------------------------------
using StepKernel = void (*)(const KArgs);

template <int METHOD, int NOISE, int COLLECT>
StepKernel pick_unroll(int unroll) {
  // Every unroll depth for cSGHMC and for the noise-bearing SGHMC / SGLD
  // production kernels; the *_GRAD and test-only noise-free variants use the
  // default depth to keep build time down.
  constexpr bool kAllDepths =
      METHOD == BDL_CSGHMC ||
      ((METHOD == BDL_SGLD || METHOD == BDL_SGHMC) && NOISE != BDL_NOISE_NONE);
  if constexpr (!kAllDepths) {
    (void)unroll;
    return bdl_step_kernel<METHOD, NOISE, COLLECT, 2>;
  } else {
    switch (unroll) {
      case 1:
        return bdl_step_kernel<METHOD, NOISE, COLLECT, 1>;
      case 4:
        return bdl_step_kernel<METHOD, NOISE, COLLECT, 4>;
      default:
        return bdl_step_kernel<METHOD, NOISE, COLLECT, 2>;
    }
  }
}

template <int METHOD, int NOISE>
StepKernel pick_collect(int collect, int unroll) {
  switch (collect) {
    case BDL_COLLECT_NONE:
      return pick_unroll<METHOD, NOISE, BDL_COLLECT_NONE>(unroll);
    case BDL_COLLECT_WELFORD_INIT:
      return pick_unroll<METHOD, NOISE, BDL_COLLECT_WELFORD_INIT>(unroll);
    case BDL_COLLECT_WELFORD:
      return pick_unroll<METHOD, NOISE, BDL_COLLECT_WELFORD>(unroll);
    case BDL_COLLECT_MEAN_INIT:
      return pick_unroll<METHOD, NOISE, BDL_COLLECT_MEAN_INIT>(unroll);
    case BDL_COLLECT_MEAN:
      return pick_unroll<METHOD, NOISE, BDL_COLLECT_MEAN>(unroll);
  }
  return nullptr;
}

template <int METHOD>
StepKernel pick_noise(int noise, int collect, int unroll) {
  switch (noise) {
    case BDL_NOISE_NONE:
      return pick_collect<METHOD, BDL_NOISE_NONE>(collect, unroll);
    case BDL_NOISE_BUFFER:
      return pick_collect<METHOD, BDL_NOISE_BUFFER>(collect, unroll);
    case BDL_NOISE_PHILOX:
      return pick_collect<METHOD, BDL_NOISE_PHILOX>(collect, unroll);
  }
  return nullptr;
}

StepKernel pick_step(int method, int noise, int collect, int unroll) {
  switch (method) {
    case BDL_CSGHMC:
      return pick_noise<BDL_CSGHMC>(noise, collect, unroll);
    case BDL_SGHMC:
      return pick_noise<BDL_SGHMC>(noise, collect, unroll);
    case BDL_SGLD:
      return pick_noise<BDL_SGLD>(noise, collect, unroll);
    case BDL_SGHMC_GRAD:
      return collect == BDL_COLLECT_NONE ? pick_noise<BDL_SGHMC_GRAD>(noise, BDL_COLLECT_NONE, unroll)
                                         : nullptr;
    case BDL_SGLD_GRAD:
      return collect == BDL_COLLECT_NONE ? pick_noise<BDL_SGLD_GRAD>(noise, BDL_COLLECT_NONE, unroll)
                                         : nullptr;
  }
  return nullptr;
}

template <int NOISE, int COLLECT>
StepKernel pick_adam_unroll(int unroll) {
  // unroll variants only where production runs (noise on); the test-only
  // NONE mode keeps the default depth
  if constexpr (NOISE == BDL_NOISE_NONE) {
    (void)unroll;
    return bdl_adam_kernel<NOISE, COLLECT, false, 2>;
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

int grid_for(int64_t ngroups, int per_block_groups) {
  const int64_t want = (ngroups + per_block_groups - 1) / per_block_groups;
  const int64_t cap = (int64_t)device_cu_count() * g_blocks_per_cu;
  return (int)std::max<int64_t>(1, std::min(want, cap));
}

// Validate a step descriptor, pick the kernel instance and launch it; `clip`
// (device pointer to (norm, coef)) scales the SGLD sampler gradient when set.
int launch_step(const bdl_step_args* s, const float* clip, hipStream_t stream) {
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
  if (!s->theta || !s->grad || !s->runs || s->nruns < 1)
    return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: theta, grad and runs are required");
  if (s->nruns > kMaxRuns)
    return fail(BDL_ERR_RUNS, "bdl_sgmcmc_step: more than 4096 runs (merge parameter groups)");
  if (needs_mom && !s->mom) return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: mom is required");
  if (needs_prior && !s->prior_mean)
    return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: prior_mean is required for sghmc/sgld");
  if (s->noise_mode == BDL_NOISE_BUFFER && !s->noise)
    return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: noise buffer is required");
  if (s->collect != BDL_COLLECT_NONE && !s->mom1)
    return fail(BDL_ERR_NULL, "bdl_sgmcmc_step: mom1 is required to collect");
  if (grad_only && s->collect != BDL_COLLECT_NONE)
    return fail(BDL_ERR_ARG, "bdl_sgmcmc_step: grad-only methods cannot collect");
  const void* ptrs[] = {s->theta, s->grad, s->mom, s->prior_mean, s->noise, s->mom1, s->mom2};
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return fail(BDL_ERR_ALIGN, "bdl_sgmcmc_step: vector not 16-B aligned");

  const int unroll = g_unroll;
  StepKernel k = pick_step(s->method, s->noise_mode, s->collect, unroll);
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
  a.inv_s2 = recip_or(s->inv_sigma2, s->sigma2);
  a.inv_nd = recip_or(s->inv_n_data, s->n_data);
  a.inv_ca = recip_or(s->inv_collect_a, s->collect_a);
  a.inv_cb = recip_or(s->inv_collect_b, s->collect_b);

  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kBlock), (size_t)s->nruns * sizeof(bdl_run),
                     stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_sgmcmc_step: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

}  // namespace

extern "C" {

int bdl_version(void) { return BDL_ABI_VERSION; }

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
    if (!push(s.offset + s.numel, s.attr & 7u))
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

int64_t bdl_clip_workspace_bytes(int64_t n) {
  (void)n;
  // (total_norm, coef) + pad to 16 B, then one fp64 partial per workgroup
  return (int64_t)16 + (int64_t)kMaxNormPartials * (int64_t)sizeof(double);
}

int bdl_sgld_step_clipped(const bdl_step_args* s, float max_norm, void* workspace, void* stream) {
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
  if (!s->theta || !s->grad || !s->runs || !s->prior_mean || s->nruns < 1)
    return fail(BDL_ERR_NULL, "bdl_sgld_step_clipped: theta, grad, prior_mean and runs are required");
  if (s->nruns > kMaxRuns)
    return fail(BDL_ERR_RUNS, "bdl_sgld_step_clipped: more than 4096 runs (merge parameter groups)");
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
  a.nruns = s->nruns;
  a.flags = s->flags;
  a.n = s->n;
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
  const size_t shmem = (size_t)s->nruns * sizeof(bdl_run);
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
  if (!s->theta || !s->grad || !s->mom || !s->prior_mean || !ad->adam_m || !ad->adam_v ||
      !s->runs || s->nruns < 1)
    return fail(BDL_ERR_NULL, "bdl_adam_step: theta, grad, mom, prior_mean, adam_m, adam_v and runs are required");
  if (s->nruns > kMaxRuns)
    return fail(BDL_ERR_RUNS, "bdl_adam_step: more than 4096 runs (merge parameter groups)");
  if (!grad_only && (s->flags & BDL_FLAG_MOMENTUM) && !ad->sgd_buf)
    return fail(BDL_ERR_NULL, "bdl_adam_step: sgd_buf is required with BDL_FLAG_MOMENTUM");
  if (s->noise_mode == BDL_NOISE_BUFFER && !s->noise)
    return fail(BDL_ERR_NULL, "bdl_adam_step: noise buffer is required");
  if (s->collect != BDL_COLLECT_NONE && !s->mom1)
    return fail(BDL_ERR_NULL, "bdl_adam_step: mom1 is required to collect");
  if (s->flags & BDL_FLAG_GRAD_READY)
    return fail(BDL_ERR_ARG, "bdl_adam_step: GRAD_READY is not an Adam flag (use bdl_sgmcmc_step)");
  const void* ptrs[] = {s->theta, s->grad, s->mom, s->prior_mean, s->noise, s->mom1, s->mom2,
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
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), (size_t)s->nruns * sizeof(bdl_run),
                     (hipStream_t)stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_adam_step: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

int bdl_moments_update(const bdl_moments_args* m, void* stream) {
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
  hipLaunchKernelGGL(bdl_moments_kernel, dim3(grid_for((m->n + 3) / 4, kBlock * 4)), dim3(kBlock), 0,
                     (hipStream_t)stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_moments_update: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

int bdl_posterior_sample(const bdl_sample_args* s, void* stream) {
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
  SArgs a{s->out, s->mom1, s->mom2, s->noise, s->n, s->var_mode, s->noise_mode,
          s->ratio, s->var_floor, s->inv_ratio, s->seed, s->chain, s->step};
  hipLaunchKernelGGL(bdl_sample_kernel, dim3(grid_for((s->n + 3) / 4, kBlock * 4)), dim3(kBlock), 0,
                     (hipStream_t)stream, a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    g_last_error = std::string("bdl_posterior_sample: launch failed: ") + hipGetErrorString(err);
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

int bdl_philox_normal(float* out, int64_t n, uint64_t seed, uint64_t chain, uint64_t step,
                      void* stream) {
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
