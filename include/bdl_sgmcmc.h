/*
 * bdl_sgmcmc.h — C-ABI of the MI355X-native fused SG-MCMC parameter update.
 *
 * This is the drop-in boundary for the per-step update of the reference's
 * methods/{csghmc,sghmc,csgld,sgld}.py Runner/Model step loop (and of its
 * variants methods/{csghmc_fs,adam_sghmc,adam_csghmc}.py).  The Python host
 * package (bayesdll_amd) binds these symbols with ctypes; any other host
 * (C, C++, another FFI) can bind them the same way — no torch types cross
 * this boundary, only plain device pointers, sizes and scalars.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repo root):
 *
 *   bdl_sgmcmc_step  replaces, in one launch over flat fp32 vectors,
 *     - methods/csghmc.py:747-778  per-tensor cSGHMC momentum + theta update
 *     - methods/sghmc.py:482-510   SGHMC grad_U / momentum / p.grad = g + v
 *       followed by torch.optim.SGD(momentum=0).step()  (methods/sghmc.py:229)
 *     - methods/sgld.py:469-484    SGLD p.grad = g + prior + noise
 *       followed by torch.optim.SGD(momentum=mu).step() (methods/sgld.py:226)
 *     - methods/csgld.py:665-680   same as sgld under the cyclical lr
 *       (methods/csgld.py:253 for the SGD step)
 *     - the posterior-moment accumulation that follows on thinned steps:
 *       methods/csghmc.py:327-345 (Welford), methods/sgld.py:239-246 and
 *       methods/sghmc.py:242-249 (running mean), methods/csgld.py:280-293
 *       (per-cycle running mean)
 *   bdl_sgld_step_clipped replaces methods/csgld.py:248-253 with args.clip_grad
 *     (Model.forward, torch.nn.utils.clip_grad_norm_, optimizer.step()).
 *   bdl_adam_step replaces methods/adam_sghmc.py:500-553 (+ SGD step, :229)
 *     and methods/adam_csghmc.py:812-860 (+ SGD step, :322).
 *   bdl_moments_update replaces the stand-alone moment updates
 *     (methods/sgld.py:95-102 burn-in seeding; the same formulas as above
 *     when the caller does not fuse them into the step).
 *   bdl_posterior_sample replaces the per-tensor posterior draw
 *     p.copy_(mean + var.sqrt() * randn_like(p))  (methods/sgld.py:292-296,
 *     methods/csghmc.py:466-468) and the variance-from-moments formulas
 *     (methods/sgld.py:337-345, methods/csghmc.py:451-459).
 *   bdl_philox_normal exposes the in-kernel N(0,1) generator (the stream the
 *     step kernel uses in BDL_NOISE_PHILOX mode), replacing torch.randn_like
 *     (methods/csghmc.py:766) for statistical testing and host inspection.
 *   bdl_build_runs is host-only: it turns the per-tensor segment table
 *     (named_parameters order, readout_name, 'bias' names — the selection
 *     logic of methods/csghmc.py:750-762 / methods/sgld.py:471-484) into the
 *     merged run table the kernels read.
 *
 * Conventions
 *   - Return 0 on success, a negative bdl_status on failure; a thread-local
 *     message is available through bdl_last_error().  No exception crosses
 *     the ABI.
 *   - All vector pointers are device pointers (hipMalloc / torch HIP tensors),
 *     16-byte aligned, fp32, contiguous, n elements, in the canonical flat
 *     order of nn.utils.parameters_to_vector(net.parameters()).
 *   - Launches are asynchronous on the given hipStream_t (pass torch's
 *     current stream); no host synchronisation, no allocation.
 */
#ifndef BDL_SGMCMC_H
#define BDL_SGMCMC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* v8: the Adam state-tiling fields (bdl_adam_args.tile_*) and the placement
 * probe flag are gone (measured, not adopted: DESIGN.md §4). */
#define BDL_ABI_VERSION 8

typedef enum bdl_status {
  BDL_OK = 0,
  BDL_ERR_NULL = -1,       /* a required pointer is null                    */
  BDL_ERR_ALIGN = -2,      /* a vector pointer is not 16-byte aligned        */
  BDL_ERR_ARG = -3,        /* inconsistent sizes / enum out of range         */
  BDL_ERR_LAUNCH = -4,     /* HIP launch error                               */
  BDL_ERR_RUNS = -5        /* run table does not cover [0, n) monotonically  */
} bdl_status;

/* Which update rule (and which reference code path) a step applies. */
typedef enum bdl_method {
  BDL_CSGHMC = 0,      /* methods/csghmc.py:747-778; theta and mom updated    */
  BDL_SGHMC = 1,       /* methods/sghmc.py:482-510 + SGD(momentum 0) step     */
  BDL_SGLD = 2,        /* methods/sgld.py:469-484 (and csgld) + SGD(mu) step  */
  BDL_SGHMC_GRAD = 3,  /* sghmc Model.forward only: grad <- g + v', mom <- v' */
  BDL_SGLD_GRAD = 4,   /* sgld Model.forward only: grad <- g + prior + noise  */
  BDL_ADAM_SGHMC = 5,  /* Adam-preconditioned SGHMC + SGD step (bdl_adam_step only):
                          methods/adam_sghmc.py:500-553 and adam_csghmc.py:812-860 */
  BDL_ADAM_SGHMC_GRAD = 6 /* its Model.forward only: grad, v_mom, m, v written    */
} bdl_method;

typedef enum bdl_noise_mode {
  BDL_NOISE_NONE = 0,    /* no noise term (cSGHMC exploration steps)          */
  BDL_NOISE_BUFFER = 1,  /* eps read from args.noise (torch-RNG parity mode)  */
  BDL_NOISE_PHILOX = 2   /* eps from in-kernel Philox4x32-10 + Box-Muller     */
} bdl_noise_mode;

/* Posterior-moment accumulation fused after the update (on the new theta). */
typedef enum bdl_collect {
  BDL_COLLECT_NONE = 0,
  BDL_COLLECT_WELFORD_INIT = 1, /* m1 = theta, m2 = 0    (csghmc.py:333-337)  */
  BDL_COLLECT_WELFORD = 2,      /* d=t-m1; m1+=d/a; d2=t-m1; m2+=d*d2 (:340-345) */
  BDL_COLLECT_MEAN_INIT = 3,    /* m1 = theta, m2 = theta^2 (csgld.py:282-284)  */
  BDL_COLLECT_MEAN = 4          /* m = (x + a*m) / b, x in {t, t^2} (sgld.py:242-245) */
} bdl_collect;

/* Per-element attribute bits carried by a run. */
#define BDL_ATTR_HEAD 0x1     /* readout_name in pname -> lr group 1          */
#define BDL_ATTR_PRIOR 0x2    /* prior term applied (not an uninformative bias)*/
#define BDL_ATTR_SKIP 0x4     /* parameter has no grad: left untouched          */
#define BDL_ATTR_GUNALIGNED 0x8 /* grad_base mode: this run's gradient base is not
                                 16-byte aligned (element-wise loads only)       */

/* Flags for bdl_step_args.flags. */
#define BDL_FLAG_FIRST_STEP 0x1  /* SGD momentum buffer does not exist yet: buf = grad */
#define BDL_FLAG_RECIP_DIV 0x2   /* divide by a scalar as x*(1/s) (torch-on-GPU), else x/s (torch CPU) */
#define BDL_FLAG_MOMENTUM 0x4    /* SGD momentum != 0: maintain args.mom as SGD buffer */
#define BDL_FLAG_GRAD_READY 0x8  /* BDL_SGLD/BDL_SGHMC: grad already holds the sampler gradient
                                    (e.g. clipped after a *_GRAD call): apply the SGD step only */

/* One parameter tensor in named_parameters order (host input to bdl_build_runs). */
typedef struct bdl_segment {
  int64_t offset;   /* element offset in the flat vector                      */
  int64_t numel;    /* element count                                          */
  uint32_t attr;    /* BDL_ATTR_* bits                                        */
  uint32_t pad;
} bdl_segment;

/* A maximal run of consecutive elements with identical attributes.
 * Runs are sorted; run i covers [runs[i-1].end, runs[i].end). Device-resident. */
typedef struct bdl_run {
  int64_t end;
  uint32_t attr;
  uint32_t pad;
} bdl_run;

typedef struct bdl_step_args {
  /* vectors (device, fp32, n elements) */
  float* theta;            /* in/out                                               */
  float* grad;             /* in (out for *_GRAD methods)                           */
  float* mom;              /* csghmc/sghmc momentum v, or SGD momentum buffer       */
  const float* prior_mean; /* theta0 (sghmc/sgld); may be null for csghmc           */
  const float* noise;      /* BDL_NOISE_BUFFER only                                 */
  float* mom1;             /* collect only                                          */
  float* mom2;             /* collect only; may be null (nst == 0)                  */
  const bdl_run* runs;     /* device run table                                      */
  int32_t nruns;
  int32_t method;          /* bdl_method      */
  int32_t noise_mode;      /* bdl_noise_mode  */
  int32_t collect;         /* bdl_collect     */
  int32_t flags;           /* BDL_FLAG_*      */
  int32_t pad0;
  int64_t n;
  /* scalars, already rounded from the host's float64 to fp32 exactly as torch
   * casts a Python scalar at the op (index 0 = body group, 1 = head group). */
  float lr[2];             /* eta                                                   */
  float noise_scale[2];    /* csghmc: nd*sqrt(2*a*eta)/N; sghmc: nd*sqrt(2a/(N eta)); sgld: nd*sqrt(2/(N eta)) */
  float one_minus_alpha;   /* fl32(1 - momentum_decay)                             */
  float prior_sig;         /* csghmc: the sigma multiplying theta (quirk Q1)        */
  float sigma2;            /* sghmc/sgld: fl32(prior_sig**2)                        */
  float n_data;            /* fl32(ND * Ninflate)                                   */
  float mu;                /* SGD momentum                                          */
  float collect_a;         /* WELFORD: n; MEAN: multiplier of the old moment        */
  float collect_b;         /* MEAN: divisor                                          */
  /* Reciprocals of the scalar divisors, fl32(1/s) of the host's float64 s: what
   * torch on a HIP device multiplies by for tensor / Python-scalar (used with
   * BDL_FLAG_RECIP_DIV; 0 means 1.0f/fl32(s)). */
  float inv_sigma2;
  float inv_n_data;
  float inv_collect_a;
  float inv_collect_b;
  float pad1;
  uint64_t seed;           /* Philox key                                            */
  uint64_t chain;          /* chain id (rank)                                        */
  uint64_t step;           /* global step counter                                    */
  /* Gradient in place, per tensor (null: the flat `grad` vector is used).
   * Device array of nruns byte addresses: run r's gradient for flat element i
   * is ((float*)grad_base[r])[i], i.e. grad_base[r] = (address of the tensor's
   * own .grad) - 4 * (flat offset of the tensor).  autograd's per-parameter
   * gradient tensors are then read (and, for *_GRAD methods, written) where
   * autograd left them — no flat gradient buffer, no zero-fill and no
   * accumulation pass before the step (torch's AccumulateGrad steals the
   * fresh gradient when .grad is None).  Runs must not span two tensors;
   * SKIP runs may hold 0; a base that is not 16-byte aligned needs
   * BDL_ATTR_GUNALIGNED on its run.  `grad` may be null in this mode. */
  const int64_t* grad_base;
  /* Divergence guard (nullable): set to 1 (atomic OR) when the step writes a
   * theta value (or, for *_GRAD methods, a gradient value) that is NaN or
   * +-Inf.  Never written on a healthy chain; the host reads it when it likes
   * (e.g. once per epoch), so the guard adds no synchronisation. */
  int32_t* nonfinite;
  /* Philox counter offset, in float4 groups: a launch over the sub-range
   * [4*philox_offset, 4*philox_offset + n) of a chain's flat vectors (all
   * pointers and the run table shifted to it) draws exactly the noise the
   * whole-vector launch draws there.  0 for whole-vector launches. */
  uint64_t philox_offset;
  /* Stacked chains (0: the vectors hold one chain).  > 0: they hold
   * consecutive chains of 4*chain_groups elements each — chain k's element j
   * at 4*chain_groups*k + j, the tail of each chain's slot beyond its own n
   * covered by a BDL_ATTR_SKIP run — and chain k draws its Philox noise keyed
   * chain + k with the element index inside its slot: exactly the noise of a
   * one-chain launch with chain id chain + k.  The run table spans all chains
   * (one run per chain and tensor in grad_base mode).  Requires n/4 +
   * philox_offset < 2^32.  Replaces running K reference processes, one chain
   * each, on one device. */
  uint64_t chain_groups;
} bdl_step_args;

/* Extra state and scalars of the Adam-preconditioned SGHMC step.  Per element,
 * in the reference's op order (every op separately rounded; "/s" is a scalar
 * division, rounded per BDL_FLAG_RECIP_DIV):
 *   gs  = g / temperature                     (adam_csghmc.py:834; 1.0 for adam_sghmc)
 *   gU  = gs + (theta - theta0)/sigma2/N      (uninformative bias: gs)
 *   m   = m*beta1 + gU*(1-beta1);   v = v*beta2 + (gU*gU)*(1-beta2)
 *   d   = sqrt(v/bias_corr2) + eps;  pg = (m/bias_corr1) / d;  pt = 1/d
 *   vm  = (vm*(1-alpha) + pg*lr) + (sqrt(pt*two_alpha/N)*nd) * eps
 *   grad = grad_is_mom ? vm : g + vm          (adam_csghmc.py:860 / adam_sghmc.py:553)
 *   then torch.optim.SGD (momentum mu, buffer sgd_buf) steps theta with grad.
 * bdl_step_args supplies theta, grad, prior_mean, noise, runs, lr, one_minus_alpha
 * (= fl32(1 - momentum_decay)), sigma2, n_data, mu, flags, collect, Philox key;
 * args->mom is v_mom (Model.momentum_buffer). */
typedef struct bdl_adam_args {
  float* adam_m;           /* Model.m (first moment)                                */
  float* adam_v;           /* Model.v (second moment)                               */
  float* sgd_buf;          /* SGD momentum buffer; required iff BDL_FLAG_MOMENTUM   */
  float beta1, one_minus_beta1, beta2, one_minus_beta2;
  float bias_corr1;        /* fl32(1 - beta1**t)                                    */
  float bias_corr2;        /* fl32(1 - beta2**t)                                    */
  float eps;               /* Adam epsilon                                          */
  float two_alpha;         /* fl32(2 * momentum_decay)                              */
  float nd;                /* noise discount                                        */
  float temperature;       /* adam_csghmc temperature (1.0 otherwise)               */
  float inv_bias_corr1;    /* reciprocals as in bdl_step_args.inv_* (0 -> 1/fl32(s)) */
  float inv_bias_corr2;
  float inv_temperature;
  float pad2;
  int32_t grad_is_mom;     /* 1: p.grad = v_mom (adam_csghmc); 0: g + v_mom         */
} bdl_adam_args;

/* Stand-alone posterior-moment update (no parameter update). */
typedef struct bdl_moments_args {
  const float* theta;
  float* mom1;
  float* mom2;             /* may be null */
  int64_t n;
  int32_t collect;         /* bdl_collect */
  int32_t flags;           /* BDL_FLAG_RECIP_DIV */
  float collect_a;
  float collect_b;
  float inv_collect_a;     /* see bdl_step_args.inv_*                                 */
  float inv_collect_b;
} bdl_moments_args;

/* Variance form used by bdl_posterior_sample. */
typedef enum bdl_var_mode {
  BDL_VAR_GIVEN = 0,       /* mom2 already holds the variance                        */
  BDL_VAR_RAW_MOMENTS = 1, /* var = ratio*(m2 - m1^2)  (sgld.py:337-345, csgld.py:396-400) */
  BDL_VAR_WELFORD = 2      /* var = M2 / ratio_div      (csghmc.py:451-459)           */
} bdl_var_mode;

typedef struct bdl_sample_args {
  float* out;              /* theta sample                                            */
  const float* mom1;       /* posterior mean                                          */
  const float* mom2;       /* variance source (see var_mode)                          */
  const float* noise;      /* eps buffer (BDL_NOISE_BUFFER) or null (Philox)          */
  int64_t n;
  int32_t var_mode;
  int32_t noise_mode;      /* BDL_NOISE_BUFFER or BDL_NOISE_PHILOX                    */
  float ratio;             /* RAW_MOMENTS multiplier / WELFORD divisor                */
  float var_floor;         /* clamp_(min=...) — 1e-12 in the reference                 */
  float inv_ratio;         /* WELFORD: nonzero -> multiply by it (torch-on-GPU rounding) */
  int32_t blocks_per_cu;   /* workgroups per CU, 1-8 (0: 2); the caller may tune it (ABI v7) */
  uint64_t seed, chain, step;
  uint64_t chain_groups;   /* stacked chains, as bdl_step_args.chain_groups (0: one) */
  int32_t unroll;          /* float4 groups per lane in flight: 0 (= 4), 1 or 4 (ABI v7) */
  int32_t pad;
} bdl_sample_args;

int bdl_version(void);
const char* bdl_last_error(void);

/* Host-only: merge segments into runs. out_runs must hold >= nseg+1 entries
 * (gaps between segments become BDL_ATTR_SKIP runs). Returns the run count
 * (>= 0) or a negative bdl_status. */
int bdl_build_runs(const bdl_segment* segs, int32_t nseg, int64_t n,
                   bdl_run* out_runs, int32_t max_runs);

/* One fused SG-MCMC step (update + optional noise + optional moment collect). */
int bdl_sgmcmc_step(const bdl_step_args* args, void* hip_stream);

/* Stand-alone moment update. */
int bdl_moments_update(const bdl_moments_args* args, void* hip_stream);

/* cSGLD with gradient clipping: replaces methods/csgld.py:248-253
 * (Model.forward's p.grad = g + prior + noise, then
 * torch.nn.utils.clip_grad_norm_(net.parameters(), clip_grad), then
 * optimizer.step()).  args->method must be BDL_SGLD.  Three launches, no host
 * synchronisation:
 *   1. the sampler gradient G is recomputed element-wise (never stored: Philox
 *      noise is a pure function of its counter) and sum(G^2) is reduced with
 *      wavefront shuffles + LDS into one partial per workgroup (skipped
 *      parameters excluded, as their .grad is None in the reference);
 *   2. one workgroup sums the partials in a fixed order (deterministic),
 *      total_norm = sqrt(sum), coef = min(1, max_norm / (total_norm + 1e-6));
 *   3. the SGLD + SGD step on G * coef (moment collect allowed).
 * workspace: device memory of bdl_clip_workspace_bytes(n) bytes; its first
 * two floats receive (total_norm, coef) for inspection. */
int64_t bdl_clip_workspace_bytes(int64_t n);
int bdl_sgld_step_clipped(const bdl_step_args* args, float max_norm, void* workspace,
                          void* hip_stream);

/* One fused Adam-preconditioned SGHMC step: replaces the per-tensor loop of
 * methods/adam_sghmc.py:500-553 / adam_csghmc.py:812-860 and the following
 * optimizer.step().  args->method: BDL_ADAM_SGHMC (update + SGD step, collect
 * NONE / MEAN_INIT / MEAN) or BDL_ADAM_SGHMC_GRAD (grad, v_mom, m, v only).
 * 40 B/element (theta, v_mom, m, v r/w; g, theta0 r), +8 with an SGD buffer. */
int bdl_adam_step(const bdl_step_args* args, const bdl_adam_args* adam, void* hip_stream);

/* theta_s = mean + sqrt(clamp(var)) * eps. */
int bdl_posterior_sample(const bdl_sample_args* args, void* hip_stream);

/* out[i] = the N(0,1) value the step kernel would draw for element i. */
int bdl_philox_normal(float* out, int64_t n, uint64_t seed, uint64_t chain,
                      uint64_t step, void* hip_stream);

/* Launch geometry override for tuning (0 = default): workgroups per CU, float4
 * groups in flight per lane (1, 2, 4: the production kernels of every method;
 * *_GRAD and noise-free test variants keep 2), and the sweep
 * order (0 = one contiguous span per workgroup, 1 = grid-stride).  Returns the
 * previous value packed as (grid_stride << 24) | (blocks_per_cu << 8) | unroll.
 * Process-global, not thread-safe; for tuning and tests. */
int bdl_set_launch_config(int32_t blocks_per_cu, int32_t unroll, int32_t grid_stride);

/* HIP-graph node binding, for a step captured inside a HIP graph (the
 * graph-mode update / backward overlap, bayesdll_amd/_base.py).  No reference
 * counterpart: the reference has no graph mode.
 * bdl_graph_find_step_node: in a captured (not yet destroyed) graph, the one
 * kernel node of a bdl_sgmcmc_step launched during a capture over the vector
 * at `theta` of `n` elements (BDL_ERR_ARG unless exactly one).
 * bdl_graph_redirect: while graph_exec is non-null, the calling
 * thread's bdl_sgmcmc_step calls launch nothing; each rewrites `node`'s kernel
 * arguments in the instantiated graph (hipGraphExecKernelNodeSetParams) with
 * the step it describes, which must select the kernel the node was captured
 * with (checked first: else BDL_ERR_ARG, nothing changed).  graph_exec = null ends the redirect.
 * While a redirect is set, the thread's other launching entry points
 * (bdl_sgld_step_clipped, bdl_adam_step, bdl_moments_update,
 * bdl_posterior_sample, bdl_philox_normal, bdl_stream_mix) launch nothing and
 * return BDL_ERR_ARG. */
int bdl_graph_find_step_node(void* graph, const void* theta, int64_t n, void** node);
/* The arguments a captured step node launches with (a diagnostic, read
 * before the first replay): out[0..9] = theta, grad, mom, runs, grad_base,
 * nruns, n, flags, mom1, mom2 (pointers as integers); nout >= 10. */
int bdl_graph_node_step_args(void* node, int64_t* out, int32_t nout);
int bdl_graph_redirect(void* graph_exec, void* node);

#ifdef __cplusplus
}
#endif

#endif /* BDL_SGMCMC_H */
