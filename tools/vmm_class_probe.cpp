// vmm_class_probe.cpp — can the placement class of the explore sweep be chosen
// chunk by chunk?  (tooling, not product; links libbdl_sgmcmc.so and times the
// production cSGHMC explore kernel through the C-ABI with hipEvents)
//
// Phase 1: M physical chunks (hipMemCreate, argv[1] MB each, argv[2] of them),
// each mapped at its own VA.  The chunk-sized explore sweep is timed with
// theta = chunk r, mom = chunk k, grad = a third chunk, for r = 0 and r = M-1:
// the relation of every chunk to the two references (fast / slow pairing).
// Phase 2: ViT-L/32-sized composite vectors, each mapped from ceil(4N/chunk)
// chunks (the same physical chunk may be mapped at several VAs), with theta's
// chunks and mom's chunks taken from chosen relation groups; full-size sweep
// timed.  Prints one JSON line per measurement.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

static const int64_t N = 306535400;

__global__ void fill(float* p, int64_t n, float a, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = a * ((float)(h & 0xffffff) / 16777216.f - 0.5f);
  }
}

static hipMemAllocationProp g_prop;
static size_t g_chunk;

static float* map_chunks(const std::vector<hipMemGenericAllocationHandle_t>& hs) {
  void* va = nullptr;
  const size_t total = hs.size() * g_chunk;
  CK(hipMemAddressReserve(&va, total, 0, nullptr, 0));
  for (size_t i = 0; i < hs.size(); ++i) CK(hipMemMap((char*)va + i * g_chunk, g_chunk, 0, hs[i], 0));
  hipMemAccessDesc acc = {};
  acc.location = g_prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, total, &acc, 1));
  return (float*)va;
}

struct Timer {
  bdl_step_args a;
  bdl_run* d_runs = nullptr;
  hipEvent_t e0, e1;
  int64_t n_alloc = 0;
  void init(int64_t n) {
    if (d_runs == nullptr) CK(hipMalloc((void**)&d_runs, 4 * sizeof(bdl_run)));
    bdl_segment seg = {0, n, BDL_ATTR_PRIOR, 0};
    bdl_run runs[4];
    const int nr = bdl_build_runs(&seg, 1, n, runs, 4);
    CK(hipMemcpy(d_runs, runs, nr * sizeof(bdl_run), hipMemcpyHostToDevice));
    memset(&a, 0, sizeof a);
    a.runs = d_runs; a.nruns = nr; a.method = BDL_CSGHMC; a.noise_mode = BDL_NOISE_NONE;
    a.collect = BDL_COLLECT_NONE; a.n = n; a.lr[0] = 1e-7f; a.lr[1] = 1e-7f;
    a.one_minus_alpha = 0.5f; a.prior_sig = 0.0f;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
  }
  float time(float* th, float* g, float* v, int reps) {
    a.theta = th; a.grad = g; a.mom = v;
    for (int w = 0; w < 2; ++w) bdl_sgmcmc_step(&a, nullptr);
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) {
      const int rc = bdl_sgmcmc_step(&a, nullptr);
      if (rc) { fprintf(stderr, "step %d: %s\n", rc, bdl_last_error()); exit(1); }
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t = 0;
    CK(hipEventElapsedTime(&t, e0, e1));
    return t / reps;
  }
};

int main(int argc, char** argv) {
  const size_t chunk_mb = argc > 1 ? atoll(argv[1]) : 1024;
  const int M = argc > 2 ? atoi(argv[2]) : 16;
  g_chunk = chunk_mb << 20;
  memset(&g_prop, 0, sizeof g_prop);
  g_prop.type = hipMemAllocationTypePinned;
  g_prop.location.type = hipMemLocationTypeDevice;
  g_prop.location.id = 0;
  bdl_set_launch_config(1, 4, 1);

  std::vector<hipMemGenericAllocationHandle_t> H(M);
  std::vector<float*> C(M);
  const int64_t nc = (int64_t)(g_chunk / 4);
  for (int i = 0; i < M; ++i) {
    CK(hipMemCreate(&H[i], g_chunk, &g_prop, 0));
    C[i] = map_chunks({H[i]});
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, C[i], nc, 2e-3f, 7u + i);
  }
  CK(hipDeviceSynchronize());

  // phase 1: chunk-sized pair times against two references
  Timer T;
  T.init(nc);
  std::vector<float> t0(M, 0), t1(M, 0);
  for (int k = 0; k < M; ++k) {
    const int refs[2] = {0, M - 1};
    float* out[2] = {&t0[k], &t1[k]};
    for (int r = 0; r < 2; ++r) {
      if (k == refs[r]) continue;
      int g = 1;
      while (g == k || g == refs[r]) ++g;
      *out[r] = T.time(C[refs[r]], C[g], C[k], 6);
    }
    printf("{\"phase\": 1, \"chunk\": %d, \"va\": \"%p\", \"ms_ref0\": %.4f, \"ms_reflast\": %.4f}\n",
           k, (void*)C[k], t0[k], t1[k]);
    fflush(stdout);
  }

  // groups by relation to chunk 0: split the sorted times at gaps > 3 %
  std::vector<int> order;
  for (int k = 1; k < M; ++k) order.push_back(k);
  std::sort(order.begin(), order.end(), [&](int x, int y) { return t0[x] < t0[y]; });
  std::vector<std::vector<int>> groups(1);
  for (size_t i = 0; i < order.size(); ++i) {
    if (i > 0 && t0[order[i]] > 1.03f * t0[order[i - 1]]) groups.emplace_back();
    groups.back().push_back(order[i]);
  }
  printf("{\"phase\": 1, \"groups\": [");
  for (size_t gi = 0; gi < groups.size(); ++gi) {
    printf("%s[", gi ? ", " : "");
    for (size_t j = 0; j < groups[gi].size(); ++j) printf("%s%d", j ? ", " : "", groups[gi][j]);
    printf("]");
  }
  printf("]}\n");
  fflush(stdout);

  // phase 2: full-size composite vectors.  theta = {chunk 0, + chunks of the
  // slowest group (the same relation to 0 as 0 itself)}; mom from group gm;
  // grad from whatever is left (chunks may repeat across roles only if needed)
  const int per = (int)((4 * N + g_chunk - 1) / g_chunk);
  T.init(N);
  std::vector<int> same = groups.back();  // slowest pairing with 0 = same class as 0
  std::vector<int> th_ids = {0};
  for (int k : same) if ((int)th_ids.size() < per) th_ids.push_back(k);
  if ((int)th_ids.size() < per) { printf("{\"phase\": 2, \"error\": \"not enough same-class chunks\"}\n"); return 0; }
  for (size_t gm = 0; gm < groups.size(); ++gm) {
    std::vector<int> mom_ids, g_ids;
    for (int k : groups[gm]) {
      if (std::find(th_ids.begin(), th_ids.end(), k) != th_ids.end()) continue;
      if ((int)mom_ids.size() < per) mom_ids.push_back(k);
    }
    if ((int)mom_ids.size() < per) continue;
    for (int k = 0; k < M && (int)g_ids.size() < per; ++k) {
      if (std::find(th_ids.begin(), th_ids.end(), k) != th_ids.end()) continue;
      if (std::find(mom_ids.begin(), mom_ids.end(), k) != mom_ids.end()) continue;
      g_ids.push_back(k);
    }
    while ((int)g_ids.size() < per) g_ids.push_back(th_ids[g_ids.size() % th_ids.size()]);
    auto pick = [&](const std::vector<int>& ids) {
      std::vector<hipMemGenericAllocationHandle_t> hs;
      for (int k : ids) hs.push_back(H[k]);
      return map_chunks(hs);
    };
    float *th = pick(th_ids), *g = pick(g_ids), *v = pick(mom_ids);
    float ms[3];
    for (int p = 0; p < 3; ++p) ms[p] = T.time(th, g, v, 10);
    printf("{\"phase\": 2, \"mom_group\": %zu, \"theta\": [", gm);
    for (size_t j = 0; j < th_ids.size(); ++j) printf("%s%d", j ? ", " : "", th_ids[j]);
    printf("], \"mom\": [");
    for (size_t j = 0; j < mom_ids.size(); ++j) printf("%s%d", j ? ", " : "", mom_ids[j]);
    printf("], \"grad\": [");
    for (size_t j = 0; j < g_ids.size(); ++j) printf("%s%d", j ? ", " : "", g_ids[j]);
    printf("], \"ms\": [%.4f, %.4f, %.4f]}\n", ms[0], ms[1], ms[2]);
    fflush(stdout);
    // mixed mom: half from this group, half same-class
    if (gm + 1 < groups.size() && per >= 2) {
      std::vector<int> mix = mom_ids;
      mix[per - 1] = -1;
      for (int k : same)
        if (std::find(th_ids.begin(), th_ids.end(), k) == th_ids.end() &&
            std::find(mix.begin(), mix.end(), k) == mix.end()) { mix[per - 1] = k; break; }
      if (mix[per - 1] >= 0) {
        float* vm = pick(mix);
        for (int p = 0; p < 3; ++p) ms[p] = T.time(th, g, vm, 10);
        printf("{\"phase\": 2, \"mom_group\": %zu, \"mixed_last_same\": %d, \"ms\": [%.4f, %.4f, %.4f]}\n",
               gm, mix[per - 1], ms[0], ms[1], ms[2]);
        fflush(stdout);
      }
    }
  }
  return 0;
}
