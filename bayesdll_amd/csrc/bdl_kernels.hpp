// bdl_kernels.hpp — device side of the fused SG-MCMC library (shared by the
// per-method translation units; see bdl_api.hip for the overview).
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "bdl_sgmcmc.h"

namespace bdl {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// ---------------------------------------------------------------------------
// Counter-based RNG: Philox4x32-10 (Salmon et al., SC'11) + Box-Muller.
// counter = (group index lo32, chain lo32, step lo32, step hi32), key = seed.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
  // The key schedule is wave-uniform: left to itself the compiler hoists all
  // twenty round keys (and the uniform counter words' xors) out of the sweep
  // loop into SGPRs, which then spill into VGPR lanes (v_writelane /
  // v_readlane + hazard s_nops in the hot loop).  BDL_PHILOX_KEYS_PER_CALL: an
  // empty asm that "modifies" the keys keeps them per call (one s_add per
  // round key).  Which schedule is faster depends on the kernel and its
  // occupancy (1-4 % either way, same-process A/Bs: DESIGN.md §4), so the
  // choice is made per translation unit in the Makefile, as is the xor form.
#ifdef BDL_PHILOX_KEYS_PER_CALL
  asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#ifdef BDL_PHILOX_TWO_XORS
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
#else
    // gfx950's three-input bit op (truth table 0x96 = a ^ b ^ c): one VALU op
    // per output word instead of two xors.
    c = make_uint4(__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
                   __builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0);
#endif
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// uniform in (0, 1]: 24 random bits, centred in their bucket; the value is
// fl32((x>>8) + 0.5) * 2^-24 (the top bucket rounds to 1.0).  Written as one
// fma: scaling by a power of two commutes with the rounding, so
// fma(a, 2^-24, 2^-25) == (a + 0.5f) * 2^-24 bit for bit for every 24-bit a
// (checked over all 2^24 inputs, tools/sample_probe.hip) — one VALU op fewer
// per draw.
__device__ __forceinline__ float u01(uint32_t x) {
  return __builtin_fmaf((float)(x >> 8), 1.0f / 16777216.0f, 1.0f / 33554432.0f);
}

// Correctly rounded fp32 sqrt for x >= 2^-96, +inf and NaN (bit-identical to
// sqrtf there; checked over every such float, tools/sample_probe.hip):
// v_sqrt_f32 (within 1 ulp) and the two-sided fma residual correction of the
// compiler's own sequence, without its denormal-range scaling and its
// zero / inf class fix-up, which that domain never needs.
__device__ __forceinline__ float sqrt_floored(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float dn = __int_as_float(__float_as_int(s) - 1);
  const float up = __int_as_float(__float_as_int(s) + 1);
  const float rdn = __builtin_fmaf(-dn, s, x);
  const float rup = __builtin_fmaf(-up, s, x);
  const float r = rdn <= 0.f ? dn : s;
  return rup > 0.f ? up : r;
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
// Every data-stream access is non-temporal: each vector is touched once per
// step and is far larger than the 256 MiB Infinity Cache.  Stores and the
// guarded path's scalar accesses are cast to the global address space; the
// 16-B loads are left generic (a gradient base read from the LDS run table
// then loads with flat_load): cast to global they ran 1-1.7 % slower in the
// explore, Welford and SGLD sweeps, same process, builds alternating
// (profiles/round5/ab_loads/: flat explore 1.0657 vs 1.0482 ms, per-tensor
// gradients 1.052 vs 1.0415, collect 2.014 vs 1.997, ResNet-101 SGLD at 2 x 1
// 0.1757 vs 0.1742).
typedef __attribute__((address_space(1))) f4v gf4v;
typedef __attribute__((address_space(1))) float gfloat;

__device__ __forceinline__ f4v vload(const float* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
}

// A 16-B load through the global address space: never a flat_load, so it is
// not counted in lgkmcnt.  For loads that are in flight while the same wave
// waits on scalar (kernarg) loads — the pipelined Adam sweep's next-iteration
// gradient — where a flat_load would hold every such wait until its data came
// back from HBM.
__device__ __forceinline__ f4v gvload(const float* p) {
  return __builtin_nontemporal_load((const gf4v*)p);
}

__device__ __forceinline__ void vstore(float* p, f4v v) {
  __builtin_nontemporal_store(v, (gf4v*)p);
}

__device__ __forceinline__ float sload(const float* p) { return *(const gfloat*)p; }
__device__ __forceinline__ void sstore(float* p, float v) { *(gfloat*)p = v; }

__device__ __forceinline__ f4v ld4(const float* __restrict__ p, int64_t e, int64_t n) {
  if (e + 4 <= n) return vload(p + e);
  f4v v = {0.f, 0.f, 0.f, 0.f};
  if (e + 0 < n) v.x = sload(p + e + 0);
  if (e + 1 < n) v.y = sload(p + e + 1);
  if (e + 2 < n) v.z = sload(p + e + 2);
  return v;
}

__device__ __forceinline__ void st4(float* __restrict__ p, int64_t e, int64_t n, f4v v) {
  if (e + 4 <= n) {
    vstore(p + e, v);
    return;
  }
  if (e + 0 < n) sstore(p + e + 0, v.x);
  if (e + 1 < n) sstore(p + e + 1, v.y);
  if (e + 2 < n) sstore(p + e + 2, v.z);
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
  const int64_t* __restrict__ gbase;  // per-run gradient bases (grad_base mode) or null
  int32_t nruns;
  int32_t flags;
  int64_t n;
  int64_t groups_per_block;
  float lr0, lr1, ns0, ns1;
  float one_minus_alpha, prior_sig, sigma2, n_data, mu, ca, cb;
  uint64_t seed, chain, step;
  const float* __restrict__ clip;  // (total_norm, coef) from the clip finalize, or null
  int32_t* __restrict__ nonfinite;  // set to 1 if a written theta / grad value is not finite (or null)
  uint64_t goff;  // Philox counter offset in float4 groups (a launch over a sub-range)
  uint32_t cgroups;  // stacked chains: float4 groups per chain (0 = one chain)
  // Adam-preconditioned SGHMC only (bdl_adam_step)
  float* __restrict__ adam_m;
  float* __restrict__ adam_v;
  float* __restrict__ sgd_buf;
  float b1, omb1, b2, omb2, bc1, bc2, aeps, two_alpha, nd, temp;
  // scalar-divisor reciprocals for BDL_FLAG_RECIP_DIV (host-rounded fl32(1/s64))
  float inv_s2, inv_nd, inv_ca, inv_cb, inv_temp, inv_bc1, inv_bc2;
};

// The kernel's KArgs re-read from the kernarg segment at the point of use:
// scalar loads behind a laundered segment pointer, which the compiler can
// neither hoist out of the sweep loop nor keep in SGPRs across it.  Every
// step / Adam kernel takes its KArgs as the first kernel argument, at offset
// 0 of the segment.  The sweep's device functions are templates over the
// argument view A (KArgs, or this address-space-4 view), so one body serves
// both.
typedef __attribute__((address_space(4))) const KArgs ckargs;

__device__ __forceinline__ ckargs& fresh_kargs() {
  ckargs* ap = (ckargs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ap));
  return *ap;
}

// The Philox draw for float4 group gi of a launch.  The counter is the group
// index within its chain: with stacked chains (cgroups > 0, chain k's elements
// at [4*cgroups*k, 4*cgroups*(k+1))) chain k is keyed chain + k and draws what
// a one-chain launch with that chain id draws.  The host keeps every group
// index below 2^32 in that mode, so the split is a 32-bit division.
// noise_from: the draw from the generator inputs of `a` as given.
template <class A>
__device__ __forceinline__ f4v noise_from(const A& a, int64_t gi) {
  uint64_t g = (uint64_t)gi + a.goff, c = a.chain;
  if (a.cgroups) {
    const uint32_t k = (uint32_t)g / a.cgroups;
    g -= (uint64_t)k * a.cgroups;
    c += k;
  }
  return philox_normal4(g, a.seed, c, a.step);
}

template <class A>
__device__ __forceinline__ f4v step_noise4(const A& a0, int64_t gi) {
#ifdef BDL_PHILOX_KEYS_PER_CALL
  // the generator's inputs (seed, chain, step, offset, chain split) re-read
  // from the kernarg segment per call (scalar loads) instead of being held in
  // SGPRs across the sweep (see philox4x32_10).  Every kernel that draws
  // step noise takes its KArgs as the first kernel argument, at offset 0 of
  // the segment.  (Spelled out rather than through fresh_kargs(): that form
  // changed the Adam unit's register allocation, 34 -> 108 SGPR spills.)
  (void)a0;
  ckargs* ap = (ckargs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ap));
  return noise_from(*ap, gi);
#else
  return noise_from(a0, gi);
#endif
}

// HELD: the inputs as the caller's argument view holds them (no per-call
// re-read; chunk_fast's kHeldNoise).
template <bool HELD, class A>
__device__ __forceinline__ f4v step_noise4_held(const A& a0, int64_t gi) {
  if constexpr (HELD)
    return noise_from(a0, gi);
  else
    return step_noise4(a0, gi);
}

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

// grad_base mode: the per-run gradient bases live in LDS right after the runs.
__device__ __forceinline__ int64_t* lds_gbase(int nruns) {
  return reinterpret_cast<int64_t*>(s_runs + nruns);
}

// Stage the run table (and the gradient bases) in LDS; dynamic LDS bytes =
// nruns * (sizeof(bdl_run) + (gbase ? 8 : 0)), see run_lds_bytes.
__device__ __forceinline__ void stage_runs(const KArgs& a) {
  for (int i = threadIdx.x; i < a.nruns; i += kBlock) s_runs[i] = a.runs[i];
  if (a.gbase) {
    int64_t* g = lds_gbase(a.nruns);
    for (int i = threadIdx.x; i < a.nruns; i += kBlock) g[i] = a.gbase[i];
  }
  __syncthreads();
}

// Where run r's gradient lives: the flat vector, or its own tensor.
template <class A>
__device__ __forceinline__ float* run_grad(const A& a, int r) {
  return a.gbase ? reinterpret_cast<float*>(lds_gbase(a.nruns)[r]) : a.grad;
}

// A block iteration may take the fast path only inside one run whose
// gradient is 16-B addressable.
constexpr uint32_t kNoFastPath = BDL_ATTR_SKIP | BDL_ATTR_GUNALIGNED;

// Divergence guard: any element of the vector not finite (NaN / +-Inf)?
__device__ __forceinline__ uint32_t nonfinite4(f4v v) {
  return (uint32_t)(!__builtin_isfinite(v.x) | !__builtin_isfinite(v.y) |
                    !__builtin_isfinite(v.z) | !__builtin_isfinite(v.w));
}

// End of a step launch: report divergence with one atomic per offending lane
// (never taken on a healthy chain, so the guard costs a compare per element).
__device__ __forceinline__ void report_nonfinite(const KArgs& a, uint32_t bad) {
  if (bad && a.nonfinite) atomicOr(a.nonfinite, 1);
}

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

// The cSGHMC sweep with its arithmetic removed (measurement only,
// bdl_sgmcmc_step_bare): the same loop, run table, loads and stores as the
// production cSGHMC kernel of a collect kind, the update and the noise draw
// gone (theta, mom, m1, m2 written back as loaded; the init kinds' m1 = theta,
// m2 = 0 / theta^2 kept: they are copies).  Its time is the ceiling of that
// kernel's own access schedule.  Not a public method id.
constexpr int kMethodBare = 100;

template <int METHOD>
constexpr bool is_csghmc_sweep() {
  return METHOD == BDL_CSGHMC || METHOD == kMethodBare;
}

// the collect arithmetic a METHOD applies: for the bare sweep's steady-state
// kinds none — m1 / m2 go back as loaded, laundered through an empty asm so
// that the compiler keeps the load and the store (a store of the value just
// loaded from the same address is otherwise deleted as dead)
constexpr int kCollectLaunder = 99;

template <int METHOD, int COLLECT>
constexpr int collect_op() {
  return (METHOD == kMethodBare &&
          (COLLECT == BDL_COLLECT_WELFORD || COLLECT == BDL_COLLECT_MEAN))
             ? kCollectLaunder
             : COLLECT;
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
template <int METHOD, int NOISE, bool RECIP, bool PRIOR, bool GR, class A>
__device__ __forceinline__ void update_core(const A& a, const StepConst& c, float eta,
                                            float ns, float& th, float& g, float& v, float th0,
                                            float eps) {
  if constexpr (METHOD == kMethodBare) {
    // loaded values go back unchanged, through an empty asm (collect_op)
    (void)a, (void)c, (void)eta, (void)ns, (void)th0, (void)eps;
    asm volatile("" : "+v"(th), "+v"(g), "+v"(v));
  } else if constexpr (GR) {
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
template <int COLLECT, bool RECIP, class A>
__device__ __forceinline__ void collect_core(const A& a, const StepConst& c, float th,
                                             float& m1, float& m2) {
  if constexpr (COLLECT == kCollectLaunder) {
    (void)a, (void)c, (void)th;
    asm volatile("" : "+v"(m1), "+v"(m2));
  } else if constexpr (COLLECT == BDL_COLLECT_WELFORD_INIT) {
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
  static constexpr bool kReadPrior = !is_csghmc_sweep<METHOD>();
  static constexpr bool kMom = (is_csghmc_sweep<METHOD>() || METHOD == BDL_SGHMC ||
                                METHOD == BDL_SGHMC_GRAD);
  static constexpr bool kWriteTheta =
      (is_csghmc_sweep<METHOD>() || METHOD == BDL_SGHMC || METHOD == BDL_SGLD);
  static constexpr bool kWriteGrad = (METHOD == BDL_SGHMC_GRAD || METHOD == BDL_SGLD_GRAD);
  static constexpr bool kCollect = (COLLECT != BDL_COLLECT_NONE);
  static constexpr bool kReadMoments =
      (COLLECT == BDL_COLLECT_WELFORD || COLLECT == BDL_COLLECT_MEAN);
};

// Is A the re-read kernarg view (fresh_kargs) rather than the kernel's KArgs?
template <class A>
constexpr bool is_fresh_args = !__is_same(__remove_cv(A), KArgs);

// Which step instances run their sweep on the re-read argument view (stream
// bases, scalars and flags loaded per iteration) with the slow path rolled:
// the SGLD / SGHMC collect and buffer-noise instances at depth 2 and 4.
// Those spilled 2-16 SGPRs, and the reloads sat in the sweep loop (16-42
// v_readlane per loop; 0 with this, tools/hot_loop_spills.py).  Same
// process, builds alternating (profiles/round6/ab_spills/): ResNet-101 SGLD
// collect 0.3079 ms (1 x 4) vs 0.3102 (best, 2 x 1), SGHMC collect 0.2970 vs
// 0.3026 at 1 x 2, ViT-L/32 SGLD collect equal.  At depth 1 the per-iteration
// scalar loads cost 5-21 % (the wave waits on them once per group), so the
// depth-1 instances keep SGPR-resident arguments, as do the cSGHMC sweeps
// (0 spills in every Philox instance).
template <int METHOD, int NOISE, int COLLECT, int UNROLL>
constexpr bool fresh_step_args() {
  return !is_csghmc_sweep<METHOD>() && UNROLL >= 2 &&
         (COLLECT != BDL_COLLECT_NONE || NOISE == BDL_NOISE_BUFFER);
}

// FAST PATH: a whole block-iteration (kBlock*UNROLL float4 groups) in range
// and inside one non-skip run.  eta / ns are scalars, PRIOR / GR compile-time:
// no branch inside, no bounds checks, every load issued before any arithmetic.
template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL, bool PRIOR, bool GR, class A>
__device__ __forceinline__ void chunk_fast(const A& a, const StepConst& c, int64_t gb,
                                           float eta, float ns, float* gp, uint32_t& bad) {
  using T = StepTraits<METHOD, COLLECT>;
  constexpr bool kPriorLoad = T::kReadPrior && PRIOR && !GR;
  // the depth-1 SGLD / SGHMC collect instances draw their noise from the
  // generator inputs held in SGPRs (the kernel's KArgs), not re-read per call:
  // at one group per lane the per-call scalar loads' wait is one per group and
  // sits in front of the draw.  Same process, builds alternating
  // (profiles/round6/ab_held/): ResNet-101 SGLD collect 0.3042 ms at 1 x 1
  // against the previous best 0.3107 (1 x 4), ViT-L/32 SGLD collect on
  // per-tensor gradients 2.1473 vs 2.2072, SGHMC collect equal.  The plain
  // depth-1 steps keep the per-call re-read: held, SGLD at its tuned 2 x 1 ran
  // 0.1749 vs 0.1697 ms (its SGPR spills 0 -> 12).
  constexpr bool kHeldNoise = UNROLL == 1 && COLLECT != BDL_COLLECT_NONE &&
                              (METHOD == BDL_SGLD || METHOD == BDL_SGHMC);
  f4v th[UNROLL], g[UNROLL], v[UNROLL], t0[UNROLL], ep[UNROLL], m1[UNROLL], m2[UNROLL];
  const f4v z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
    v[u] = t0[u] = ep[u] = m1[u] = m2[u] = z;
    th[u] = vload(a.theta + e);
    // SGLD and SGHMC read their gradient through the global address space:
    // the per-call Philox inputs are scalar loads, and with the gradient as a
    // flat_load their lgkmcnt wait would also wait for it.  Same process,
    // builds alternating: ResNet-101 SGLD equal at 2 x 1 and 4 % faster at
    // 1 x 4, its collect 1-2.4 % and ViT-L/32's 4.3 % faster
    // (profiles/round5/ab_noise/); SGHMC with its keys per call as well 3.8 %
    // (ResNet-101) and 5.3 % (ViT-L/32, per-tensor gradients) faster at the
    // best geometry (profiles/round5/ab_sghmc/).  The cSGHMC explore (no
    // noise) ran 2.7 % slower with it.
    if constexpr (METHOD == BDL_SGLD || METHOD == BDL_SGHMC)
      g[u] = gvload(gp + e);
    else
      g[u] = vload(gp + e);
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
      ep[u] = step_noise4_held<kHeldNoise>(a, gi);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xt = th[u][j], xg = g[u][j], xv = v[u][j], x1 = m1[u][j], x2 = m2[u][j];
      update_core<METHOD, NOISE, RECIP, PRIOR, GR>(a, c, eta, ns, xt, xg, xv, t0[u][j], ep[u][j]);
      collect_core<collect_op<METHOD, COLLECT>(), RECIP>(a, c, xt, x1, x2);
      th[u][j] = xt;
      g[u][j] = xg;
      v[u][j] = xv;
      m1[u][j] = x1;
      m2[u][j] = x2;
    }
    if constexpr (T::kWriteTheta) {
      bad |= nonfinite4(th[u]);
      vstore(a.theta + e, th[u]);
    }
    if constexpr (T::kWriteGrad) {
      bad |= nonfinite4(g[u]);
      vstore(gp + e, g[u]);
    }
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

template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL, class A>
__device__ __forceinline__ void chunk_fast_dispatch(const A& a, const StepConst& c,
                                                    int64_t gb, uint32_t attr, float* gp,
                                                    uint32_t& bad) {
  const bool head = (attr & BDL_ATTR_HEAD) != 0;
  const float eta = head ? a.lr1 : a.lr0;
  const float ns = head ? a.ns1 : a.ns0;
  if constexpr (is_csghmc_sweep<METHOD>()) {
    chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, false, false>(a, c, gb, eta, ns, gp, bad);
  } else {
    if constexpr (METHOD == BDL_SGLD || METHOD == BDL_SGHMC) {
      if (c.grad_ready) {
        chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, false, true>(a, c, gb, eta, ns, gp, bad);
        return;
      }
    }
    if (attr & BDL_ATTR_PRIOR)
      chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, true, false>(a, c, gb, eta, ns, gp, bad);
    else
      chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, false, false>(a, c, gb, eta, ns, gp, bad);
  }
}

// The fast iterations of one run (the cSGHMC sweep, step_body): every full
// block iteration from gb on whose groups all lie in the run (gb + kIter <=
// lim), with the run's attributes and gradient base resolved once — no LDS
// access, no run search between them.  Returns the first iteration not taken.
template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL, bool PRIOR, bool GR>
__device__ __forceinline__ int64_t fast_run(const KArgs& a, const StepConst& c, int64_t gb,
                                            int64_t lim, int64_t gstep, float eta, float ns,
                                            float* gp, uint32_t& bad) {
  constexpr int64_t kIter = (int64_t)kBlock * UNROLL;
  do {
    chunk_fast<METHOD, NOISE, COLLECT, RECIP, UNROLL, PRIOR, GR>(a, c, gb, eta, ns, gp, bad);
    gb += gstep;
  } while (gb + kIter <= lim);
  return gb;
}

// Element-wise update for the slow path: attribute-dependent branches allowed.
template <int METHOD, int NOISE, int COLLECT, bool RECIP, class A>
__device__ __forceinline__ void update_elem(const A& a, const StepConst& c, uint32_t attr,
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
  collect_core<collect_op<METHOD, COLLECT>(), RECIP>(a, c, th, m1, m2);
}

// SLOW PATH: an iteration that reaches the end of the vector / span, crosses a
// run boundary or covers a skipped parameter.  Per-lane predicates, guarded
// partial groups, a per-element run search (in LDS).  Taken for
// O(#runs + #blocks) iterations per launch.
template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL, class A>
__device__ __forceinline__ void chunk_slow(const A& a, const StepConst& c, int64_t gb,
                                           int64_t gend, int r0, uint32_t& bad) {
  using T = StepTraits<METHOD, COLLECT>;
  const int64_t n = a.n;
  int rr = r0;  // run of the chunk's first element; a lane's elements only move forward
  // rolled in the fresh-argument instances (fresh_step_args): the path is
  // rare, and unrolled, its nested guards' lane masks filled their SGPR file
  constexpr int kSlowUnroll = is_fresh_args<A> ? 1 : UNROLL;
#pragma unroll kSlowUnroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    if (gi >= gend) continue;
    const int64_t e = gi * 4;
    const f4v z = {0.f, 0.f, 0.f, 0.f};
    const bool gt = a.gbase != nullptr;  // gradient per tensor
    f4v th = ld4(a.theta, e, n), g = gt ? z : ld4(a.grad, e, n), v = z, t0 = z, ep = z, m1 = z,
        m2 = z;
    // per-tensor gradient: one 16-B load when the group lies in one run whose
    // base is 16-B addressable (run offsets are multiples of 4 on every
    // backbone here), else element by element below
    bool gvec = false;
    if (gt) {
      while (rr < a.nruns - 1 && run_end(rr) <= e) ++rr;
      if (e + 4 <= n && run_end(rr) >= e + 4 && !(run_attr(rr) & kNoFastPath)) {
        g = vload(run_grad(a, rr) + e);
        gvec = true;
      }
    }
    if (T::kMom || (METHOD == BDL_SGLD && c.sgd_mom_read)) v = ld4(a.mom, e, n);
    if (T::kReadPrior) t0 = ld4(a.prior_mean, e, n);
    if (NOISE == BDL_NOISE_BUFFER) ep = ld4(a.noise, e, n);
    if (NOISE == BDL_NOISE_PHILOX) ep = step_noise4(a, gi);
    if (T::kReadMoments) {
      m1 = ld4(a.mom1, e, n);
      if (c.has_m2) m2 = ld4(a.mom2, e, n);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (e + j >= n) break;
      while (rr < a.nruns - 1 && run_end(rr) <= e + j) ++rr;
      const uint32_t at = run_attr(rr);
      float* gpr = gt ? run_grad(a, rr) : nullptr;
      if (gt && !gvec && !(at & BDL_ATTR_SKIP)) g[j] = sload(gpr + e + j);
      float xt = th[j], xg = g[j], xv = v[j], x1 = m1[j], x2 = m2[j];
      update_elem<METHOD, NOISE, COLLECT, RECIP>(a, c, at, xt, xg, xv, t0[j], ep[j], x1, x2);
      if (T::kWriteGrad && gt && !(at & BDL_ATTR_SKIP)) sstore(gpr + e + j, xg);
      th[j] = xt;
      g[j] = xg;
      v[j] = xv;
      m1[j] = x1;
      m2[j] = x2;
    }
    if (T::kWriteTheta) {
      bad |= nonfinite4(th);  // lanes past n hold 0: never flagged
      st4(a.theta, e, n, th);
    }
    if (T::kWriteGrad) bad |= nonfinite4(g);  // SKIP elements hold 0 here
    if (T::kWriteGrad && !gt) st4(a.grad, e, n, g);
    if (T::kMom || (METHOD == BDL_SGLD && c.sgd_mom)) st4(a.mom, e, n, v);
    if (T::kCollect) {
      st4(a.mom1, e, n, m1);
      if (c.has_m2) st4(a.mom2, e, n, m2);
    }
  }
}


// Block-uniform test for the multi-run path: the full iteration whose
// elements end at e_end starts in run r and ends in a later run; every run it
// touches must allow the fast path (no SKIP, gradient base 16-B addressable)
// and every run boundary inside it must fall on a float4 group boundary, so
// that each lane's group lies in one run.
__device__ __forceinline__ bool multi_run_ok(int nruns, int r, int64_t e_end) {
  for (; r < nruns; ++r) {
    if (run_attr(r) & kNoFastPath) return false;
    const int64_t end = run_end(r);
    if (end >= e_end) return true;
    if (end & 3) return false;
  }
  return false;
}

// MULTI-RUN PATH: a whole block iteration in range that crosses run
// boundaries (multi_run_ok).  Each lane finds the run of each of its groups
// in the LDS table and applies that run's attributes (lr group, prior) per
// element, reading the gradient from that run's own base; as on the fast
// path every access is a 16-B access and every load is issued before any
// arithmetic.  Where it is taken: iterations that straddle a tensor boundary
// when each tensor's gradient is read from its own autograd allocation (one
// run per tensor: ~300 of the ~75 K iterations of a ViT-L/32 step), which
// the guarded slow path used to take with its loads serialised per group.
template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL, class A>
__device__ __forceinline__ void chunk_multi(const A& a, const StepConst& c, int64_t gb,
                                            int r0, uint32_t& bad) {
  using T = StepTraits<METHOD, COLLECT>;
  f4v th[UNROLL], g[UNROLL], v[UNROLL], t0[UNROLL], ep[UNROLL], m1[UNROLL], m2[UNROLL];
  uint32_t at[UNROLL];
  float* gq[UNROLL];
  const f4v z = {0.f, 0.f, 0.f, 0.f};
  int rr = r0;  // a lane's groups only move forward; multi_run_ok bounds the search
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
    while (run_end(rr) <= e) ++rr;
    at[u] = run_attr(rr);
    gq[u] = run_grad(a, rr);
    v[u] = t0[u] = ep[u] = m1[u] = m2[u] = z;
    th[u] = vload(a.theta + e);
    g[u] = vload(gq[u] + e);
    if (T::kMom || (METHOD == BDL_SGLD && c.sgd_mom_read)) v[u] = vload(a.mom + e);
    if (T::kReadPrior) t0[u] = vload(a.prior_mean + e);
    if (NOISE == BDL_NOISE_BUFFER) ep[u] = vload(a.noise + e);
    if (T::kReadMoments) {
      m1[u] = vload(a.mom1 + e);
      if (c.has_m2) m2[u] = vload(a.mom2 + e);
    }
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    if constexpr (NOISE == BDL_NOISE_PHILOX) ep[u] = step_noise4(a, gi);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xt = th[u][j], xg = g[u][j], xv = v[u][j], x1 = m1[u][j], x2 = m2[u][j];
      update_elem<METHOD, NOISE, COLLECT, RECIP>(a, c, at[u], xt, xg, xv, t0[u][j], ep[u][j], x1,
                                                 x2);
      th[u][j] = xt;
      g[u][j] = xg;
      v[u][j] = xv;
      m1[u][j] = x1;
      m2[u][j] = x2;
    }
    if constexpr (T::kWriteTheta) {
      bad |= nonfinite4(th[u]);
      vstore(a.theta + e, th[u]);
    }
    if constexpr (T::kWriteGrad) {
      bad |= nonfinite4(g[u]);
      vstore(gq[u] + e, g[u]);
    }
    if (T::kMom || (METHOD == BDL_SGLD && c.sgd_mom)) vstore(a.mom + e, v[u]);
    if constexpr (T::kCollect) {
      vstore(a.mom1 + e, m1[u]);
      if (c.has_m2) vstore(a.mom2 + e, m2[u]);
    }
  }
}

// Variants of a step body, fixed per launch (step_variant): the SGD step on
// an already formed gradient (BDL_FLAG_GRAD_READY) and the clipped SGLD
// gradient (bdl_sgld_step_clipped); kVarRuntime reads both from the launch.
constexpr int kVarGradReady = 1, kVarClip = 2, kVarRuntime = -1;

// The cSGHMC cycle-init collects (m1 = theta, m2 written, nothing of the
// moments read) at depth 1 take the plain sweep's per-run loop too: same
// process, builds alternating (profiles/round6/ab_csg_per_run/), the Welford
// init 1.5814 vs 1.5913 ms and 1.5697 vs 1.5843 (flat / per-tensor
// gradients, each build's best geometry); the steady collect ran 3.5-5 %
// slower that way at 1 x 1 and keeps the per-iteration lookup.
template <int COLLECT, int UNROLL>
constexpr bool csg_collect_per_run() {
  return UNROLL == 1 &&
         (COLLECT == BDL_COLLECT_WELFORD_INIT || COLLECT == BDL_COLLECT_MEAN_INIT);
}

// The launch's per-step constants (flags, clip coefficient, reciprocals).
template <int METHOD, int COLLECT, int VAR, class A>
__device__ __forceinline__ StepConst make_step_const(const A& a) {
  StepConst c;
  c.sgd_mom = (METHOD == BDL_SGLD) && (a.flags & BDL_FLAG_MOMENTUM);
  c.sgd_mom_read = c.sgd_mom && !(a.flags & BDL_FLAG_FIRST_STEP);
  c.has_m2 = (COLLECT != BDL_COLLECT_NONE) && (a.mom2 != nullptr);
  if constexpr (VAR == kVarRuntime) {
    c.grad_ready = (METHOD == BDL_SGLD || METHOD == BDL_SGHMC) && (a.flags & BDL_FLAG_GRAD_READY);
    c.clip = (METHOD == BDL_SGLD) && a.clip != nullptr;
  } else {
    c.grad_ready = (VAR & kVarGradReady) != 0;
    c.clip = (VAR & kVarClip) != 0;
  }
  c.clip_coef = c.clip ? a.clip[1] : 1.0f;
  c.inv_s2 = a.inv_s2;
  c.inv_nd = a.inv_nd;
  c.inv_ca = a.inv_ca;
  c.inv_cb = a.inv_cb;
  return c;
}

template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL, int VAR>
__device__ __forceinline__ void step_body(const KArgs& a) {
  const StepConst c = make_step_const<METHOD, COLLECT, VAR>(a);

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

  // stage the run table (and gradient bases) in LDS
  stage_runs(a);
  if (g0 >= g1) return;

  int r = find_run_lds(a.nruns, g0 * 4);
  uint32_t bad = 0;
  // Two loop shapes, chosen per kernel from same-process A/Bs
  // (profiles/round5/ab_loop/): the plain cSGHMC sweep (explore / sample
  // steps) resolves a run once and loops over its full iterations with no LDS
  // access between them (explore 1.0387 vs 1.0493 ms with the per-iteration
  // loop); the SGLD / SGHMC sweeps and the collect steps keep the
  // per-iteration run lookup, which needs fewer registers (with the per-run
  // loop: SGLD SGPR spills 0 -> 2-14 and ResNet-101 SGLD at 2 x 1 0.1793 vs
  // 0.1716 ms; cSGHMC depth-4 collects 0 -> 2-6 spills).
  if constexpr (fresh_step_args<METHOD, NOISE, COLLECT, UNROLL>()) {
  for (int64_t gb = g0; gb < g1; gb += gstep) {
    // the iteration's arguments, flags included, from the re-read view
    ckargs& fa = fresh_kargs();
    const StepConst fc = make_step_const<METHOD, COLLECT, VAR>(fa);
    while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
    const int64_t gend = min(gb + kIter, g1);
    const uint32_t attr = run_attr(r);
    const bool full = gend == gb + kIter && gend <= nfull;
    if (full && run_end(r) >= gend * 4 && !(attr & kNoFastPath))
      chunk_fast_dispatch<METHOD, NOISE, COLLECT, RECIP, UNROLL>(fa, fc, gb, attr, run_grad(fa, r),
                                                                  bad);
    else if (full && multi_run_ok(a.nruns, r, gend * 4))
      chunk_multi<METHOD, NOISE, COLLECT, RECIP, UNROLL>(fa, fc, gb, r, bad);
    else
      chunk_slow<METHOD, NOISE, COLLECT, RECIP, UNROLL>(fa, fc, gb, gend, r, bad);
  }
  } else if constexpr (!is_csghmc_sweep<METHOD>() ||
                       (COLLECT != BDL_COLLECT_NONE && !csg_collect_per_run<COLLECT, UNROLL>())) {
  for (int64_t gb = g0; gb < g1; gb += gstep) {
    while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
    const int64_t gend = min(gb + kIter, g1);
    const uint32_t attr = run_attr(r);
    const bool full = gend == gb + kIter && gend <= nfull;
    if (full && run_end(r) >= gend * 4 && !(attr & kNoFastPath))
      chunk_fast_dispatch<METHOD, NOISE, COLLECT, RECIP, UNROLL>(a, c, gb, attr, run_grad(a, r),
                                                                  bad);
    else if (full && multi_run_ok(a.nruns, r, gend * 4))
      chunk_multi<METHOD, NOISE, COLLECT, RECIP, UNROLL>(a, c, gb, r, bad);
    else
      chunk_slow<METHOD, NOISE, COLLECT, RECIP, UNROLL>(a, c, gb, gend, r, bad);
  }
  } else {
  for (int64_t gb = g0; gb < g1;) {
    while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
    const uint32_t attr = run_attr(r);
    // the full iterations from gb on whose groups all lie in run r
    const int64_t lim = min(min(run_end(r) >> 2, nfull), g1);
    if (!(attr & kNoFastPath) && gb + kIter <= lim) {
      const bool head = (attr & BDL_ATTR_HEAD) != 0;
      gb = fast_run<METHOD, NOISE, COLLECT, RECIP, UNROLL, false, false>(
          a, c, gb, lim, gstep, head ? a.lr1 : a.lr0, head ? a.ns1 : a.ns0, run_grad(a, r), bad);
      continue;
    }
    const int64_t gend = min(gb + kIter, g1);
    if (gend == gb + kIter && gend <= nfull && multi_run_ok(a.nruns, r, gend * 4))
      chunk_multi<METHOD, NOISE, COLLECT, RECIP, UNROLL>(a, c, gb, r, bad);
    else
      chunk_slow<METHOD, NOISE, COLLECT, RECIP, UNROLL>(a, c, gb, gend, r, bad);
    gb += gstep;
  }
  }
  report_nonfinite(a, bad);
}

// In the plain (non-collect) SGLD / SGHMC sweeps — the steps of a run — the
// rarely taken variants get bodies of their own, chosen once per launch: a
// runtime flag tested inside the sweep keeps what it needs live across all of
// it (SGPR spills: 6-13 per SGLD Philox instance with runtime flags, 0 with
// variant bodies).  The collect instances (one step in `thin`) keep the
// runtime flags: three bodies there cost more registers than they save.
template <int METHOD, int NOISE, int COLLECT, bool RECIP, int UNROLL>
__device__ __forceinline__ void step_variant(const KArgs& a) {
  if constexpr (COLLECT != BDL_COLLECT_NONE || !(METHOD == BDL_SGLD || METHOD == BDL_SGHMC)) {
    step_body<METHOD, NOISE, COLLECT, RECIP, UNROLL, kVarRuntime>(a);
  } else {
    if (a.flags & BDL_FLAG_GRAD_READY)
      step_body<METHOD, NOISE, COLLECT, RECIP, UNROLL, kVarGradReady>(a);
    else if (METHOD == BDL_SGLD && a.clip != nullptr)
      step_body<METHOD, NOISE, COLLECT, RECIP, UNROLL, kVarClip>(a);
    else
      step_body<METHOD, NOISE, COLLECT, RECIP, UNROLL, 0>(a);
  }
}

template <int METHOD, int NOISE, int COLLECT, int UNROLL>
__global__ __launch_bounds__(kBlock) void bdl_step_kernel(const KArgs a) {
  if (a.flags & BDL_FLAG_RECIP_DIV)
    step_variant<METHOD, NOISE, COLLECT, true, UNROLL>(a);
  else
    step_variant<METHOD, NOISE, COLLECT, false, UNROLL>(a);
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

template <int NOISE, bool RECIP, bool PRIOR, bool GRADONLY, class A>
__device__ __forceinline__ void adam_core(const A& a, const AdamConst& c, float eta, float& th,
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
                                          float eta, float* gp, uint32_t& bad) {
  constexpr bool kReadMoments = (COLLECT == BDL_COLLECT_MEAN);
  const f4v z = {0.f, 0.f, 0.f, 0.f};
  f4v th[U], g[U], vm[U], m[U], v[U], buf[U], t0[U], ep[U], m1[U], m2[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    buf[u] = t0[u] = ep[u] = m1[u] = m2[u] = z;
    th[u] = vload(a.theta + e);
    g[u] = vload(gp + e);
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
  // the update's scalars re-read from the kernarg segment (as in
  // adam_pipe_compute): held across the sweep they spilled 89-132 SGPRs in
  // the plain-loop (GRADONLY) instances, 12-30 this way
  ckargs& ka = fresh_kargs();
  AdamConst c2 = c;
  c2.inv_s2 = ka.inv_s2;
  c2.inv_nd = ka.inv_nd;
  c2.inv_temp = ka.inv_temp;
  c2.inv_bc1 = ka.inv_bc1;
  c2.inv_bc2 = ka.inv_bc2;
  c2.inv_ca = ka.inv_ca;
  c2.inv_cb = ka.inv_cb;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    if constexpr (NOISE == BDL_NOISE_PHILOX) ep[u] = step_noise4(a, gi);
    StepConst cc;  // collect_core only reads inv_ca / inv_cb
    cc.inv_ca = c2.inv_ca;
    cc.inv_cb = c2.inv_cb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xt = th[u][j], xg = g[u][j], xvm = vm[u][j], xm = m[u][j], xv = v[u][j],
            xb = buf[u][j], x1 = m1[u][j], x2 = m2[u][j];
      adam_core<NOISE, RECIP, PRIOR, GRADONLY>(ka, c2, eta, xt, xg, xvm, xm, xv, xb, t0[u][j],
                                               ep[u][j]);
      collect_core<COLLECT, RECIP>(ka, cc, xt, x1, x2);
      th[u][j] = xt;
      g[u][j] = xg;
      vm[u][j] = xvm;
      m[u][j] = xm;
      v[u][j] = xv;
      buf[u][j] = xb;
      m1[u][j] = x1;
      m2[u][j] = x2;
    }
    if constexpr (GRADONLY) {
      bad |= nonfinite4(g[u]);
      vstore(gp + e, g[u]);
    } else {
      bad |= nonfinite4(th[u]);
      vstore(a.theta + e, th[u]);
    }
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
                                          int64_t gend, int r0, uint32_t& bad) {
  const int64_t n = a.n;
  int rr = r0;  // run of the chunk's first element; a lane's elements only move forward
  const f4v z = {0.f, 0.f, 0.f, 0.f};
  StepConst cc;
  cc.inv_ca = c.inv_ca;
  cc.inv_cb = c.inv_cb;
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    if (gi >= gend) continue;
    const int64_t e = gi * 4;
    const bool gt = a.gbase != nullptr;  // gradient per tensor (as in chunk_slow)
    f4v th = ld4(a.theta, e, n), g = gt ? z : ld4(a.grad, e, n), vm = ld4(a.mom, e, n);
    bool gvec = false;
    if (gt) {
      while (rr < a.nruns - 1 && run_end(rr) <= e) ++rr;
      if (e + 4 <= n && run_end(rr) >= e + 4 && !(run_attr(rr) & kNoFastPath)) {
        g = vload(run_grad(a, rr) + e);
        gvec = true;
      }
    }
    f4v m = ld4(a.adam_m, e, n), v = ld4(a.adam_v, e, n), t0 = ld4(a.prior_mean, e, n);
    f4v buf = z, ep = z, m1 = z, m2 = z;
    if (!GRADONLY && c.sgd_mom_read) buf = ld4(a.sgd_buf, e, n);
    if (NOISE == BDL_NOISE_BUFFER) ep = ld4(a.noise, e, n);
    if (NOISE == BDL_NOISE_PHILOX) ep = step_noise4(a, gi);
    if (COLLECT == BDL_COLLECT_MEAN) {
      m1 = ld4(a.mom1, e, n);
      if (c.has_m2) m2 = ld4(a.mom2, e, n);
    }
    for (int j = 0; j < 4; ++j) {
      if (e + j >= n) break;
      while (rr < a.nruns - 1 && run_end(rr) <= e + j) ++rr;
      const uint32_t at = run_attr(rr);
      float* gpr = gt ? run_grad(a, rr) : nullptr;
      if (gt && !gvec && !(at & BDL_ATTR_SKIP)) g[j] = sload(gpr + e + j);
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
      if (GRADONLY && gt && !(at & BDL_ATTR_SKIP)) sstore(gpr + e + j, xg);
      th[j] = xt;
      g[j] = xg;
      vm[j] = xvm;
      m[j] = xm;
      v[j] = xv;
      buf[j] = xb;
      m1[j] = x1;
      m2[j] = x2;
    }
    if (GRADONLY) {
      bad |= nonfinite4(g);
      if (!gt) st4(a.grad, e, n, g);
    } else {
      bad |= nonfinite4(th);
      st4(a.theta, e, n, th);
    }
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


// Multi-run iteration of the Adam sweep (as chunk_multi for the step sweep):
// a full block iteration across run boundaries that multi_run_ok admits; each
// lane takes its group's run (gradient base, lr group, prior) from the LDS
// table, every access 16-B, all loads first.
template <int NOISE, int COLLECT, bool RECIP, bool GRADONLY, int U>
__device__ __forceinline__ void adam_multi(const KArgs& a, const AdamConst& c, int64_t gb, int r0,
                                           uint32_t& bad) {
  constexpr bool kReadMoments = (COLLECT == BDL_COLLECT_MEAN);
  const f4v z = {0.f, 0.f, 0.f, 0.f};
  f4v th[U], g[U], vm[U], m[U], v[U], buf[U], t0[U], ep[U], m1[U], m2[U];
  uint32_t at[U];
  float* gq[U];
  int rr = r0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t e = (gb + (int64_t)u * kBlock + threadIdx.x) * 4;
    while (run_end(rr) <= e) ++rr;
    at[u] = run_attr(rr);
    gq[u] = run_grad(a, rr);
    buf[u] = ep[u] = m1[u] = m2[u] = z;
    th[u] = vload(a.theta + e);
    g[u] = vload(gq[u] + e);
    vm[u] = vload(a.mom + e);
    m[u] = vload(a.adam_m + e);
    v[u] = vload(a.adam_v + e);
    if (!GRADONLY && c.sgd_mom_read) buf[u] = vload(a.sgd_buf + e);
    t0[u] = vload(a.prior_mean + e);
    if constexpr (NOISE == BDL_NOISE_BUFFER) ep[u] = vload(a.noise + e);
    if constexpr (kReadMoments) {
      m1[u] = vload(a.mom1 + e);
      if (c.has_m2) m2[u] = vload(a.mom2 + e);
    }
  }
  StepConst cc;  // collect_core only reads inv_ca / inv_cb
  cc.inv_ca = c.inv_ca;
  cc.inv_cb = c.inv_cb;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    if constexpr (NOISE == BDL_NOISE_PHILOX) ep[u] = step_noise4(a, gi);
    const float eta = (at[u] & BDL_ATTR_HEAD) ? a.lr1 : a.lr0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xt = th[u][j], xg = g[u][j], xvm = vm[u][j], xm = m[u][j], xv = v[u][j],
            xb = buf[u][j], x1 = m1[u][j], x2 = m2[u][j];
      if (at[u] & BDL_ATTR_PRIOR)
        adam_core<NOISE, RECIP, true, GRADONLY>(a, c, eta, xt, xg, xvm, xm, xv, xb, t0[u][j],
                                                ep[u][j]);
      else
        adam_core<NOISE, RECIP, false, GRADONLY>(a, c, eta, xt, xg, xvm, xm, xv, xb, t0[u][j],
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
    if constexpr (GRADONLY) {
      bad |= nonfinite4(g[u]);
      vstore(gq[u] + e, g[u]);
    } else {
      bad |= nonfinite4(th[u]);
      vstore(a.theta + e, th[u]);
    }
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

// ---------------------------------------------------------------------------
// Software-pipelined Adam sweep (not GRADONLY): the next block iteration's loads are issued
// before this iteration's arithmetic, so the ~420 VALU instructions per float4
// group (IEEE divide / sqrt x2 each, Philox) run while the next seven streams
// are in flight.  One process, same buffers, alternating builds
// (tools/step_ab.py, profiles/round4/check_b/adam_pipe_ab.jsonl): best
// geometry 2.406 ms (1 workgroup/CU x 4) vs 2.429 ms unpipelined (4 x 4); at
// 1 x 4, where one wave per SIMD would otherwise wait out its own arithmetic,
// 2.406 vs 3.074 ms.  Two register sets take turns (the
// loop body is written twice with the roles swapped: no copies); an iteration
// that needs the guarded path drains the pipeline.  Same per-element update as
// adam_fast / adam_slow, so results are bit-identical.
// Register budget (round 5): the compute re-reads the update's scalars, and
// (BDL_PHILOX_KEYS_PER_CALL, set for this unit) the Philox inputs, from the
// kernarg segment per iteration, and the next iteration's gradient is loaded
// through the global address space (gvload) so those scalar loads' lgkmcnt
// waits do not wait for it: SGPR spills 189 -> 34 in the production instance
// <PHILOX, NONE, false, 4>; ViT-L/32 Adam-SGHMC + SGD, same process, builds
// alternating (profiles/round5/ab_adam/): 2.5862 vs 2.6615 ms at the best
// geometry (flat gradient), 2.6104 vs 2.6455 (per-tensor gradients).  Either
// change alone was slower.
// ---------------------------------------------------------------------------
template <int U>
struct AdamRegs {
  f4v th[U], g[U], vm[U], m[U], v[U], buf[U], t0[U], ep[U], m1[U], m2[U];
};

template <int NOISE, int COLLECT, int U>
__device__ __forceinline__ void adam_pipe_load(const KArgs& a, const AdamConst& c, int64_t gb,
                                               const float* gp, bool prior, AdamRegs<U>& R) {
  const f4v z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    R.th[u] = vload(a.theta + e);
    R.g[u] = gvload(gp + e);
    R.vm[u] = vload(a.mom + e);
    R.m[u] = vload(a.adam_m + e);
    R.v[u] = vload(a.adam_v + e);
    R.buf[u] = c.sgd_mom_read ? vload(a.sgd_buf + e) : z;
    R.t0[u] = prior ? vload(a.prior_mean + e) : z;
    R.ep[u] = z;
    if constexpr (NOISE == BDL_NOISE_BUFFER) R.ep[u] = vload(a.noise + e);
    R.m1[u] = R.m2[u] = z;
    if constexpr (COLLECT == BDL_COLLECT_MEAN) {
      R.m1[u] = vload(a.mom1 + e);
      if (c.has_m2) R.m2[u] = vload(a.mom2 + e);
    }
  }
}

template <int NOISE, int COLLECT, bool RECIP, bool PRIOR, int U>
__device__ __forceinline__ void adam_pipe_compute(const KArgs& a, const AdamConst& c, int64_t gb,
                                                  float eta, float* gp, AdamRegs<U>& R,
                                                  uint32_t& bad) {
  // the update's scalars (Adam / SGD / prior coefficients and their
  // reciprocals) re-read from the kernarg segment per iteration (scalar loads
  // behind a laundered segment pointer, so they are not hoisted), like the
  // Philox inputs (step_noise4): held in SGPRs across the sweep they spilled
  // 92-197 SGPRs into VGPR lanes in the Philox instances, read here 24-76
  // (tools/resource_usage.py).  The kernel's KArgs is its first argument, at
  // offset 0 of the segment.
  typedef __attribute__((address_space(4))) const KArgs ckargs;
  ckargs* ap = (ckargs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ap));
  const ckargs& ka = *ap;
  AdamConst c2 = c;
  c2.inv_s2 = ka.inv_s2;
  c2.inv_nd = ka.inv_nd;
  c2.inv_temp = ka.inv_temp;
  c2.inv_bc1 = ka.inv_bc1;
  c2.inv_bc2 = ka.inv_bc2;
  c2.inv_ca = ka.inv_ca;
  c2.inv_cb = ka.inv_cb;
  StepConst cc;  // collect_core only reads inv_ca / inv_cb
  cc.inv_ca = c2.inv_ca;
  cc.inv_cb = c2.inv_cb;
  (void)gp;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t gi = gb + (int64_t)u * kBlock + threadIdx.x;
    const int64_t e = gi * 4;
    if constexpr (NOISE == BDL_NOISE_PHILOX) R.ep[u] = step_noise4(a, gi);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xt = R.th[u][j], xg = R.g[u][j], xvm = R.vm[u][j], xm = R.m[u][j], xv = R.v[u][j],
            xb = R.buf[u][j], x1 = R.m1[u][j], x2 = R.m2[u][j];
      adam_core<NOISE, RECIP, PRIOR, false>(ka, c2, eta, xt, xg, xvm, xm, xv, xb, R.t0[u][j],
                                            R.ep[u][j]);
      collect_core<COLLECT, RECIP>(ka, cc, xt, x1, x2);
      R.th[u][j] = xt;
      R.vm[u][j] = xvm;
      R.m[u][j] = xm;
      R.v[u][j] = xv;
      R.buf[u][j] = xb;
      R.m1[u][j] = x1;
      R.m2[u][j] = x2;
    }
    bad |= nonfinite4(R.th[u]);
    vstore(a.theta + e, R.th[u]);
    vstore(a.mom + e, R.vm[u]);
    vstore(a.adam_m + e, R.m[u]);
    vstore(a.adam_v + e, R.v[u]);
    if (c.sgd_mom) vstore(a.sgd_buf + e, R.buf[u]);
    if constexpr (COLLECT != BDL_COLLECT_NONE) {
      vstore(a.mom1 + e, R.m1[u]);
      if (c.has_m2) vstore(a.mom2 + e, R.m2[u]);
    }
  }
}

// Cursor of the pipelined sweep: the current block iteration, its run and
// whether its data already sit in the current register set.
struct AdamPipeCursor {
  int64_t gb;
  int r;
  uint32_t attr;
  bool fast, loaded;
};

template <int U>
__device__ __forceinline__ bool adam_pipe_fast(const KArgs& a, int64_t gb, int& r,
                                               uint32_t& attr) {
  constexpr int64_t kIter = (int64_t)kBlock * U;
  const int64_t ngroups = (a.n + 3) >> 2, nfull = a.n >> 2;
  if (gb >= ngroups) return false;
  while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
  const int64_t gend = min(gb + kIter, ngroups);
  attr = run_attr(r);
  return gend == gb + kIter && gend <= nfull && run_end(r) >= gend * 4 && !(attr & kNoFastPath);
}

// One block iteration with X as the current register set and Y as the next;
// false when the block's span is done.
template <int NOISE, int COLLECT, bool RECIP, int U>
__device__ __forceinline__ bool adam_pipe_iter(const KArgs& a, const AdamConst& c,
                                               AdamPipeCursor& k, AdamRegs<U>& X,
                                               AdamRegs<U>& Y, uint32_t& bad) {
  constexpr int64_t kIter = (int64_t)kBlock * U;
  const int64_t ngroups = (a.n + 3) >> 2;
  const int64_t gstep = (int64_t)gridDim.x * kIter;
  if (k.gb >= ngroups) return false;
  if (!k.fast) {
    const int64_t gend = min(k.gb + kIter, ngroups);
    if (gend == k.gb + kIter && gend <= (a.n >> 2) && multi_run_ok(a.nruns, k.r, gend * 4))
      adam_multi<NOISE, COLLECT, RECIP, false, U>(a, c, k.gb, k.r, bad);
    else
      adam_slow<NOISE, COLLECT, RECIP, false, U>(a, c, k.gb, gend, k.r, bad);
    k.gb += gstep;
    k.fast = adam_pipe_fast<U>(a, k.gb, k.r, k.attr);
    k.loaded = false;
    return true;
  }
  const bool prior = (k.attr & BDL_ATTR_PRIOR) != 0;
  float* gp = run_grad(a, k.r);
  if (!k.loaded) adam_pipe_load<NOISE, COLLECT, U>(a, c, k.gb, gp, prior, X);
  // the next iteration: classify it and issue its loads before this one's math
  const int64_t nx = k.gb + gstep;
  int rn = k.r;
  uint32_t attrn = 0;
  const bool fastn = adam_pipe_fast<U>(a, nx, rn, attrn);
  if (fastn)
    adam_pipe_load<NOISE, COLLECT, U>(a, c, nx, run_grad(a, rn), (attrn & BDL_ATTR_PRIOR) != 0, Y);
  const float eta = (k.attr & BDL_ATTR_HEAD) ? a.lr1 : a.lr0;
  if (prior)
    adam_pipe_compute<NOISE, COLLECT, RECIP, true, U>(a, c, k.gb, eta, gp, X, bad);
  else
    adam_pipe_compute<NOISE, COLLECT, RECIP, false, U>(a, c, k.gb, eta, gp, X, bad);
  k.gb = nx;
  k.r = rn;
  k.attr = attrn;
  k.fast = fastn;
  k.loaded = fastn;
  return true;
}

template <int NOISE, int COLLECT, bool RECIP, int U>
__device__ __forceinline__ void adam_pipe_sweep(const KArgs& a, const AdamConst& c,
                                                uint32_t& bad) {
  constexpr int64_t kIter = (int64_t)kBlock * U;
  AdamPipeCursor k;
  k.gb = (int64_t)blockIdx.x * kIter;
  k.r = find_run_lds(a.nruns, k.gb * 4);
  k.attr = 0;
  k.fast = adam_pipe_fast<U>(a, k.gb, k.r, k.attr);
  k.loaded = false;
  AdamRegs<U> A, B;
  for (;;) {
    if (!adam_pipe_iter<NOISE, COLLECT, RECIP, U>(a, c, k, A, B, bad)) break;
    if (!adam_pipe_iter<NOISE, COLLECT, RECIP, U>(a, c, k, B, A, bad)) break;
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
  stage_runs(a);
  if constexpr (!GRADONLY) {  // the software-pipelined sweep
    uint32_t bad = 0;
    adam_pipe_sweep<NOISE, COLLECT, RECIP, U>(a, c, bad);
    report_nonfinite(a, bad);
    return;
  }
  int r = find_run_lds(a.nruns, (int64_t)blockIdx.x * kIter * 4);
  uint32_t bad = 0;
  for (int64_t gb = (int64_t)blockIdx.x * kIter; gb < ngroups; gb += (int64_t)gridDim.x * kIter) {
    while (r < a.nruns - 1 && run_end(r) <= gb * 4) ++r;
    const int64_t gend = min(gb + kIter, ngroups);
    const uint32_t attr = run_attr(r);
    if (gend == gb + kIter && gend <= nfull && run_end(r) >= gend * 4 && !(attr & kNoFastPath)) {
      const float eta = (attr & BDL_ATTR_HEAD) ? a.lr1 : a.lr0;
      if (attr & BDL_ATTR_PRIOR)
        adam_fast<NOISE, COLLECT, RECIP, GRADONLY, true, U>(a, c, gb, eta, run_grad(a, r), bad);
      else
        adam_fast<NOISE, COLLECT, RECIP, GRADONLY, false, U>(a, c, gb, eta, run_grad(a, r), bad);
    } else {
      if (gend == gb + kIter && gend <= nfull && multi_run_ok(a.nruns, r, gend * 4))
        adam_multi<NOISE, COLLECT, RECIP, GRADONLY, U>(a, c, gb, r, bad);
      else
        adam_slow<NOISE, COLLECT, RECIP, GRADONLY, U>(a, c, gb, gend, r, bad);
    }
  }
  report_nonfinite(a, bad);
}

template <int NOISE, int COLLECT, bool GRADONLY, int U>
__global__ __launch_bounds__(kBlock) void bdl_adam_kernel(const KArgs a) {
  if (a.flags & BDL_FLAG_RECIP_DIV)
    adam_body<NOISE, COLLECT, true, GRADONLY, U>(a);
  else
    adam_body<NOISE, COLLECT, false, GRADONLY, U>(a);
}

// ---------------------------------------------------------------------------
// Kernel selection: one function pointer per (method, noise, collect, unroll)
// instance; each method's instances live in their own translation unit
// (bdl_step_*.hip, bdl_adam.hip) so the library compiles in parallel.
// ---------------------------------------------------------------------------
using StepKernel = void (*)(const KArgs);

template <int METHOD, int NOISE, int COLLECT>
StepKernel pick_unroll(int unroll) {
  // Every unroll depth for cSGHMC and for the noise-bearing SGHMC / SGLD
  // production kernels; the *_GRAD and test-only noise-free variants use the
  // default depth to keep build time down.
  constexpr bool kAllDepths =
      is_csghmc_sweep<METHOD>() ||
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

StepKernel pick_step_csghmc(int noise, int collect, int unroll);
StepKernel pick_step_csghmc_bare(int collect, int unroll);
StepKernel pick_step_sghmc(int method, int noise, int collect, int unroll);
StepKernel pick_step_sgld(int method, int noise, int collect, int unroll);
StepKernel pick_adam(int noise, int collect, bool grad_only, int unroll);

}  // namespace bdl
