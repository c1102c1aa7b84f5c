// placement_probe2.cpp — why does the same fused cSGHMC explore sweep (ViT-L/32,
// 306,535,400 fp32) run 0.97 ms on one (theta, grad, mom) allocation set and
// 1.05-1.13 ms on another?  (tooling, not product; links libbdl_sgmcmc.so and
// times the production kernel through the C-ABI with hipEvents)
//
// Strategies (argv[1]):
//   separate  : hipMalloc per vector (what torch's caching allocator does for
//               blocks this large), S sets side by side
//   contig    : hipExtMallocWithFlags(hipDeviceMallocContiguous) per vector
//               (one physically contiguous range per vector)
//   vmm       : hipMemCreate + hipMemMap per vector with chunk size argv[3] MB
//               (physical chunks of a chosen size mapped into one VA range)
//   slab      : one hipMalloc for the three vectors of a set, carved at
//               offsets 0, s, 2s with s = round_up(4n, 2 MiB) + argv[3] bytes
//   mix       : argv[2] separate vectors; every ordered triple of distinct vectors
//               timed as (theta, grad, mom) — is the slowness a property of one
//               vector, of a pair, or of the triple?
// argv[2] = number of sets.  Prints one JSON line per set: VAs, per-pass ms.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bdl_sgmcmc.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

static const int64_t N = 306535400, HEAD = 1025000;

struct Set {
  float *th, *g, *v;
};

__global__ void fill(float* p, int64_t n, float a, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = a * ((float)(h & 0xffffff) / 16777216.f - 0.5f);
  }
}

static float* vmm_alloc(size_t bytes, size_t chunk) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  if (chunk < gran) chunk = gran;
  chunk = (chunk + gran - 1) / gran * gran;
  const size_t total = (bytes + chunk - 1) / chunk * chunk;
  void* va = nullptr;
  CK(hipMemAddressReserve(&va, total, 0, nullptr, 0));
  for (size_t off = 0; off < total; off += chunk) {
    hipMemGenericAllocationHandle_t h;
    CK(hipMemCreate(&h, chunk, &prop, 0));
    CK(hipMemMap((char*)va + off, chunk, 0, h, 0));
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, total, &acc, 1));
  return (float*)va;
}

static bdl_run* device_runs(int* nr) {
  bdl_segment segs[2] = {{0, N - HEAD, BDL_ATTR_PRIOR, 0},
                         {N - HEAD, HEAD, BDL_ATTR_PRIOR | BDL_ATTR_HEAD, 0}};
  bdl_run runs[8];
  *nr = bdl_build_runs(segs, 2, N, runs, 8);
  bdl_run* d_runs;
  CK(hipMalloc((void**)&d_runs, sizeof runs));
  CK(hipMemcpy(d_runs, runs, *nr * sizeof(bdl_run), hipMemcpyHostToDevice));
  return d_runs;
}

static int mix(int nv, const std::vector<long long>& deltas) {
  const size_t bytes = (size_t)N * 4, slack = (size_t)1100 << 20;
  std::vector<float*> V(nv);
  for (int i = 0; i < nv; ++i) {
    CK(hipMalloc((void**)&V[i], bytes + slack));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, V[i], N, 2e-3f, 7u + i);
  }
  CK(hipDeviceSynchronize());
  int nr = 0;
  bdl_run* d_runs = device_runs(&nr);
  bdl_set_launch_config(1, 4, 1);
  bdl_step_args a;
  memset(&a, 0, sizeof a);
  a.runs = d_runs; a.nruns = nr; a.method = BDL_CSGHMC; a.noise_mode = BDL_NOISE_NONE;
  a.collect = BDL_COLLECT_NONE; a.n = N; a.lr[0] = 1e-7f; a.lr[1] = 1e-6f;
  a.one_minus_alpha = 0.5f; a.prior_sig = 0.0f;  // values stay bounded over many launches
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (long long d : deltas)
  for (int i = 0; i < nv; ++i)
    for (int j = 0; j < nv; ++j)
      for (int k = 0; k < nv; ++k) {
        if (i == j || j == k || i == k) continue;
        // with offsets: one grad vector per (theta, mom) pair is enough
        if (deltas.size() > 1 && j != (i != 0 && k != 0 ? 0 : (i != 1 && k != 1 ? 1 : 2))) continue;
        a.theta = V[i]; a.grad = V[j]; a.mom = (float*)((char*)V[k] + d);
        for (int w = 0; w < 2; ++w) bdl_sgmcmc_step(&a, nullptr);
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < 8; ++r) bdl_sgmcmc_step(&a, nullptr);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        printf("{\"delta\": %lld, \"th\": %d, \"g\": %d, \"v\": %d, \"ms\": %.4f}\n", d, i,
               j, k, t / 8);
      }
  fflush(stdout);
  return 0;
}

// map: allocate nv vectors in order; time (theta = ref, mom = V[k]) for two
// reference vectors (the first and the last) -> the class sequence of the
// allocations, in allocation order
static int classmap(int nv, size_t elems) {
  const size_t bytes = elems * 4;
  std::vector<float*> V(nv);
  for (int i = 0; i < nv; ++i) {
    if (hipMalloc((void**)&V[i], bytes) != hipSuccess) { nv = i; break; }
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, V[i], (int64_t)elems, 2e-3f, 7u + i);
  }
  CK(hipDeviceSynchronize());
  bdl_segment seg = {0, (int64_t)elems, BDL_ATTR_PRIOR, 0};
  bdl_run runs[4];
  const int nr = bdl_build_runs(&seg, 1, (int64_t)elems, runs, 4);
  bdl_run* d_runs;
  CK(hipMalloc((void**)&d_runs, sizeof runs));
  CK(hipMemcpy(d_runs, runs, nr * sizeof(bdl_run), hipMemcpyHostToDevice));
  bdl_set_launch_config(1, 4, 1);
  bdl_step_args a;
  memset(&a, 0, sizeof a);
  a.runs = d_runs; a.nruns = nr; a.method = BDL_CSGHMC; a.noise_mode = BDL_NOISE_NONE;
  a.collect = BDL_COLLECT_NONE; a.n = (int64_t)elems; a.lr[0] = 1e-7f; a.lr[1] = 1e-6f;
  a.one_minus_alpha = 0.5f; a.prior_sig = 0.0f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int refs[2] = {0, nv - 1};
  for (int k = 0; k < nv; ++k) {
    float ms[2] = {0, 0};
    for (int r = 0; r < 2; ++r) {
      const int ref = refs[r];
      if (k == ref) continue;
      int g = 1;
      while (g == k || g == ref) ++g;
      a.theta = V[ref]; a.grad = V[g]; a.mom = V[k];
      for (int w = 0; w < 2; ++w) bdl_sgmcmc_step(&a, nullptr);
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < 6; ++q) bdl_sgmcmc_step(&a, nullptr);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[r], e0, e1));
      ms[r] /= 6;
    }
    printf("{\"k\": %d, \"va\": \"%p\", \"ms_ref0\": %.4f, \"ms_reflast\": %.4f}\n", k,
           (void*)V[k], ms[0], ms[1]);
  }
  fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "separate";
  const int sets = argc > 2 ? atoi(argv[2]) : 6;
  const long long param = argc > 3 ? atoll(argv[3]) : 0;
  const int passes = 3, reps = 20;
  const size_t bytes = (size_t)N * 4;
  if (mode == "vmm") {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    size_t gmin = 0, grec = 0;
    CK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
    CK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
    printf("{\"granularity_min\": %zu, \"granularity_rec\": %zu}\n", gmin, grec);
  }
  if (mode == "map") return classmap(sets, argc > 3 ? (size_t)atoll(argv[3]) : (size_t)N);
  if (mode == "mix") {  // argv[3...]: byte offsets of the momentum vector
    std::vector<long long> deltas;
    for (int i = 3; i < argc; ++i) deltas.push_back(atoll(argv[i]));
    if (deltas.empty()) deltas.push_back(0);
    return mix(sets, deltas);
  }
  std::vector<Set> S(sets);
  for (int s = 0; s < sets; ++s) {
    if (mode == "separate") {
      CK(hipMalloc((void**)&S[s].th, bytes));
      CK(hipMalloc((void**)&S[s].g, bytes));
      CK(hipMalloc((void**)&S[s].v, bytes));
    } else if (mode == "contig") {
      CK(hipExtMallocWithFlags((void**)&S[s].th, bytes, hipDeviceMallocContiguous));
      CK(hipExtMallocWithFlags((void**)&S[s].g, bytes, hipDeviceMallocContiguous));
      CK(hipExtMallocWithFlags((void**)&S[s].v, bytes, hipDeviceMallocContiguous));
    } else if (mode == "vmm") {
      const size_t chunk = (size_t)(param > 0 ? param : 2) << 20;
      S[s].th = vmm_alloc(bytes, chunk);
      S[s].g = vmm_alloc(bytes, chunk);
      S[s].v = vmm_alloc(bytes, chunk);
    } else if (mode == "slab") {
      const size_t two_mb = (size_t)2 << 20;
      const size_t stride = (bytes + two_mb - 1) / two_mb * two_mb + (size_t)param;
      char* base = nullptr;
      CK(hipMalloc((void**)&base, 3 * stride));
      S[s].th = (float*)base;
      S[s].g = (float*)(base + stride);
      S[s].v = (float*)(base + 2 * stride);
    } else {
      fprintf(stderr, "unknown mode %s\n", mode.c_str());
      return 1;
    }
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, S[s].th, N, 0.04f, 1u + s);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, S[s].g, N, 2e-3f, 101u + s);
    CK(hipMemset(S[s].v, 0, bytes));
  }
  CK(hipDeviceSynchronize());

  bdl_segment segs[2] = {{0, N - HEAD, BDL_ATTR_PRIOR, 0},
                         {N - HEAD, HEAD, BDL_ATTR_PRIOR | BDL_ATTR_HEAD, 0}};
  bdl_run runs[8];
  const int nr = bdl_build_runs(segs, 2, N, runs, 8);
  bdl_run* d_runs;
  CK(hipMalloc((void**)&d_runs, sizeof runs));
  CK(hipMemcpy(d_runs, runs, nr * sizeof(bdl_run), hipMemcpyHostToDevice));
  if (argc > 4) {  // blocks_per_cu unroll
    bdl_set_launch_config(atoi(argv[4]), argc > 5 ? atoi(argv[5]) : 4, 1);
  } else {
    bdl_set_launch_config(1, 4, 1);
  }

  bdl_step_args a;
  memset(&a, 0, sizeof a);
  a.runs = d_runs; a.nruns = nr; a.method = BDL_CSGHMC; a.noise_mode = BDL_NOISE_NONE;
  a.collect = BDL_COLLECT_NONE; a.n = N; a.lr[0] = 1e-7f; a.lr[1] = 1e-6f;
  a.one_minus_alpha = 0.82f; a.prior_sig = 1.0f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(sets);
  uint64_t step = 0;
  auto run = [&](int s) {
    a.theta = S[s].th; a.grad = S[s].g; a.mom = S[s].v; a.step = step++;
    const int rc = bdl_sgmcmc_step(&a, nullptr);
    if (rc) { fprintf(stderr, "step %d: %s\n", rc, bdl_last_error()); exit(1); }
  };
  for (int s = 0; s < sets; ++s)
    for (int w = 0; w < 3; ++w) run(s);
  for (int p = 0; p < passes; ++p) {
    for (int s = 0; s < sets; ++s) {
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) run(s);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[s].push_back(t / reps);
    }
  }
  for (int s = 0; s < sets; ++s) {
    double mean = 0;
    for (float t : ms[s]) mean += t;
    mean /= ms[s].size();
    printf("{\"mode\": \"%s\", \"param\": %lld, \"set\": %d, \"th\": \"%p\", \"g\": \"%p\", "
           "\"v\": \"%p\", \"ms\": [%.4f, %.4f, %.4f], \"mean\": %.4f, \"tbs\": %.3f}\n",
           mode.c_str(), param, s, (void*)S[s].th, (void*)S[s].g, (void*)S[s].v, ms[s][0],
           ms[s][1], ms[s][2], mean, 20.0 * N / (mean * 1e-3) / 1e12);
  }
  fflush(stdout);
  return 0;
}
