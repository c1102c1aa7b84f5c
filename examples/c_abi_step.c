/*
 * A plain C host (gcc, no Python, no torch) driving the fused SG-MCMC step
 * through the C-ABI of include/bdl_sgmcmc.h, with device memory from the HIP
 * runtime's C API — the same boundary a cgo / JNI / N-API binding uses.
 *
 * Five cSGHMC steps (methods/csghmc.py:759-778; two lr groups, the head as
 * the trailing segment, a ragged n) on the GPU, then the same update in this
 * program on the CPU, op by op in fp32 (compiled with -ffp-contract=off):
 * theta and v must agree bit for bit.  Prints "OK <n> <steps>" and exits 0.
 */
#define __HIP_PLATFORM_AMD__
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bdl_sgmcmc.h"

#define HIP_OK(x)                                                        \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 2;                                                          \
    }                                                                    \
  } while (0)

static uint64_t s = 0x9E3779B97F4A7C15ull;
static float urand(void) { /* xorshift64*, uniform in [-1, 1) */
  s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
  return (float)((s * 2685821657736338717ull) >> 40) / (float)(1 << 23) - 1.0f;
}

int main(void) {
  const int64_t n = (1 << 22) + 13, head = 1000;
  const int steps = 5;
  const float lr[2] = {1e-3f, 1e-2f}, prior_sig = 1.0f, one_minus_alpha = 0.82f;
  float* th = (float*)malloc(n * sizeof(float));
  float* g = (float*)malloc(n * sizeof(float));
  float* v = (float*)calloc(n, sizeof(float));
  float* out = (float*)malloc(n * sizeof(float));
  for (int64_t i = 0; i < n; ++i) { th[i] = 0.02f * urand(); g[i] = 1e-3f * urand(); }

  /* segment table -> run table (host-only entry point) */
  bdl_segment segs[2] = {{0, n - head, BDL_ATTR_PRIOR, 0},
                         {n - head, head, BDL_ATTR_PRIOR | BDL_ATTR_HEAD, 0}};
  bdl_run runs[8];
  const int nr = bdl_build_runs(segs, 2, n, runs, 8);
  if (nr < 1) { fprintf(stderr, "build_runs: %s\n", bdl_last_error()); return 1; }

  float *d_th, *d_g, *d_v;
  bdl_run* d_runs;
  HIP_OK(hipMalloc((void**)&d_th, n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&d_g, n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&d_v, n * sizeof(float)));
  HIP_OK(hipMalloc((void**)&d_runs, nr * sizeof(bdl_run)));
  HIP_OK(hipMemcpy(d_th, th, n * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_g, g, n * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_v, v, n * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_runs, runs, nr * sizeof(bdl_run), hipMemcpyHostToDevice));

  bdl_step_args a;
  memset(&a, 0, sizeof a);
  a.theta = d_th; a.grad = d_g; a.mom = d_v; a.runs = d_runs; a.nruns = nr;
  a.method = BDL_CSGHMC; a.noise_mode = BDL_NOISE_NONE; a.collect = BDL_COLLECT_NONE;
  a.n = n; a.lr[0] = lr[0]; a.lr[1] = lr[1];
  a.one_minus_alpha = one_minus_alpha; a.prior_sig = prior_sig;
  for (int k = 0; k < steps; ++k) {
    a.step = (uint64_t)k;
    const int rc = bdl_sgmcmc_step(&a, NULL);  /* NULL = the default stream */
    if (rc != BDL_OK) { fprintf(stderr, "step: %d %s\n", rc, bdl_last_error()); return 1; }
  }
  HIP_OK(hipDeviceSynchronize());

  /* the reference update on the CPU, op by op (csghmc.py:759-778) */
  for (int k = 0; k < steps; ++k) {
    for (int64_t i = 0; i < n; ++i) {
      const float eta = i >= n - head ? lr[1] : lr[0];
      const float t = prior_sig * th[i];
      const float gu = g[i] + t;
      const float x = v[i] * one_minus_alpha;
      const float y = eta * gu;
      const float vn = x - y;
      v[i] = vn;
      th[i] = th[i] + vn;
    }
  }
  HIP_OK(hipMemcpy(out, d_th, n * sizeof(float), hipMemcpyDeviceToHost));
  if (memcmp(out, th, n * sizeof(float)) != 0) { fprintf(stderr, "theta differs\n"); return 1; }
  HIP_OK(hipMemcpy(out, d_v, n * sizeof(float), hipMemcpyDeviceToHost));
  if (memcmp(out, v, n * sizeof(float)) != 0) { fprintf(stderr, "v differs\n"); return 1; }
  printf("OK %lld %d\n", (long long)n, steps);
  hipFree(d_th); hipFree(d_g); hipFree(d_v); hipFree(d_runs);
  free(th); free(g); free(v); free(out);
  return 0;
}
