// phase_probe.hip — does aligning every CU's read and write bursts to a
// chip-wide clock help the explore sweep (tooling)?
//
// The explore step's 3 reads + 2 writes per element run at ~94 % of the
// serialised read / write bound: the rest is DRAM read / write
// turnaround.  Each wave already alternates a read burst (U float4 groups x
// theta, grad, mom) with a write burst, but the 256 CUs are out of phase, so
// every HBM channel sees reads and writes mixed.  Here the phases are tied to
// the SoC's constant 100 MHz real-time counter (the same for every CU, no
// communication): loads are issued only in the first R ticks of each period
// of R + W ticks, stores only in the last W.  If the channels then see
// mostly-read and mostly-write stretches, the sweep approaches the serialised
// bound; the cost is idle time when a burst does not fill its slot.
// Variants, same arithmetic and bytes as the cSGHMC explore step (20 B /
// element): base (the production loop shape) and phased at a sweep of
// (workgroups/CU, R, W).  theta / mom = the fastest pair of NV allocations
// under base (the placement effect).  Each phased variant's
// output is checked bit for bit against base.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ f4 ld(const f4* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(f4* p, f4 v) { __builtin_nontemporal_store(v, p); }

struct A {
  f4* th;
  const f4* g;
  f4* v;
  long n4;
  float oma, eta, sig;
  unsigned rt, wt;  // read / write slot lengths in real-time ticks
};

__device__ __forceinline__ void upd(const A& a, f4& th, f4 g, f4& v) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float t = a.sig * th[j];
    const float gu = g[j] + t;
    const float x = v[j] * a.oma;
    const float y = a.eta * gu;
    const float vn = x - y;
    v[j] = vn;
    th[j] = th[j] + vn;
  }
}

template <int U>
__global__ __launch_bounds__(256) void k_base(const A a) {
  const long stepi = (long)gridDim.x * 256 * U;
  for (long b = (long)blockIdx.x * 256 * U; b + 256 * U <= a.n4; b += stepi) {
    f4 th[U], g[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = b + u * 256 + threadIdx.x;
      th[u] = ld(a.th + i);
      g[u] = ld(a.g + i);
      v[u] = ld(a.v + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = b + u * 256 + threadIdx.x;
      upd(a, th[u], g[u], v[u]);
      st(a.th + i, th[u]);
      st(a.v + i, v[u]);
    }
  }
}

// position inside the current period of rt + wt ticks
__device__ __forceinline__ unsigned phase_pos(const A& a) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  return (unsigned)(t % (unsigned long long)(a.rt + a.wt));
}

template <int U>
__global__ __launch_bounds__(256) void k_phase(const A a) {
  const long stepi = (long)gridDim.x * 256 * U;
  for (long b = (long)blockIdx.x * 256 * U; b + 256 * U <= a.n4; b += stepi) {
    // wait for a read slot (positions [0, rt))
    while (phase_pos(a) >= a.rt) __builtin_amdgcn_s_sleep(1);
    f4 th[U], g[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = b + u * 256 + threadIdx.x;
      th[u] = ld(a.th + i);
      g[u] = ld(a.g + i);
      v[u] = ld(a.v + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) upd(a, th[u], g[u], v[u]);
    // wait for a write slot (positions [rt, rt + wt))
    while (phase_pos(a) < a.rt) __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = b + u * 256 + threadIdx.x;
      st(a.th + i, th[u]);
      st(a.v + i, v[u]);
    }
  }
}

__global__ void k_fill(f4* x, long n4, unsigned seed, float scale) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    const float f = ((float)(h & 0xFFFF) - 32768.f) * scale;
    x[i] = f4{f, -f, 0.5f * f, f * 0.25f};
  }
}

__global__ void k_cmp(const f4* x, const f4* y, long n4, unsigned long long* bad) {
  unsigned long long c = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    for (int j = 0; j < 4; ++j) c += __float_as_uint(x[i][j]) != __float_as_uint(y[i][j]);
  if (c) atomicAdd(bad, c);
}

template <typename K>
float timeit(K k, int grid, A a, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) k<<<grid, 256>>>(a);
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) k<<<grid, 256>>>(a);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms / reps;
}

int main() {
  const long n4 = 306535400 / 4 / (256 * 4) * (256 * 4);
  int cus = 0, rate_khz = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  printf("{\"cus\": %d, \"wall_clock_khz\": %d}\n", cus, rate_khz);
  fflush(stdout);
  const int NV = getenv("NV") ? atoi(getenv("NV")) : 6;
  std::vector<f4*> V(NV);
  for (auto& p : V) {
    CHECK(hipMalloc(&p, n4 * sizeof(f4)));
    k_fill<<<cus * 4, 256>>>(p, n4, 7u, 1e-6f);
  }
  f4 *g, *th_ref, *v_ref;
  unsigned long long* bad;
  CHECK(hipMalloc(&g, n4 * sizeof(f4)));
  CHECK(hipMalloc(&th_ref, n4 * sizeof(f4)));
  CHECK(hipMalloc(&v_ref, n4 * sizeof(f4)));
  CHECK(hipMalloc(&bad, 8));
  k_fill<<<cus * 4, 256>>>(g, n4, 11u, 1e-7f);
  int bi = 0, bj = 1;
  float best = 1e9f;
  for (int i = 0; i < NV; ++i)
    for (int j = 0; j < NV; ++j) {
      if (i == j) continue;
      A a{V[i], g, V[j], n4, 0.82f, 1e-9f, 0.f, 1, 1};
      const float ms = timeit(k_base<4>, cus, a, 3);
      if (ms < best) best = ms, bi = i, bj = j;
    }
  printf("{\"theta\": %d, \"mom\": %d, \"pair_ms\": %.4f}\n", bi, bj, best);
  fflush(stdout);
  A a{V[bi], g, V[bj], n4, 0.82f, 1e-4f, 1.0f, 175, 140};
  {  // correctness: one phased launch from the same start, vs base
    k_fill<<<cus * 4, 256>>>(V[bi], n4, 3u, 1e-4f);
    k_fill<<<cus * 4, 256>>>(V[bj], n4, 5u, 1e-5f);
    k_base<4><<<cus, 256>>>(a);
    CHECK(hipMemcpy(th_ref, V[bi], n4 * sizeof(f4), hipMemcpyDeviceToDevice));
    CHECK(hipMemcpy(v_ref, V[bj], n4 * sizeof(f4), hipMemcpyDeviceToDevice));
    k_fill<<<cus * 4, 256>>>(V[bi], n4, 3u, 1e-4f);
    k_fill<<<cus * 4, 256>>>(V[bj], n4, 5u, 1e-5f);
    k_phase<4><<<cus, 256>>>(a);
    CHECK(hipMemset(bad, 0, 8));
    k_cmp<<<cus * 4, 256>>>(V[bi], th_ref, n4, bad);
    k_cmp<<<cus * 4, 256>>>(V[bj], v_ref, n4, bad);
    unsigned long long b = 0;
    CHECK(hipMemcpy(&b, bad, 8, hipMemcpyDeviceToHost));
    printf("{\"variant\": \"phase4\", \"mismatches\": %llu}\n", b);
    fflush(stdout);
  }
  // slot lengths in ticks (10 ns at 100 MHz): per-iteration chip volume at
  // 1 wg/CU x 4 is ~12.6 MB read + 8.4 MB written
  const unsigned slots[][2] = {{60, 50},   {100, 80},  {140, 110}, {175, 140}, {220, 175},
                               {280, 220}, {350, 280}, {450, 360}, {175, 100}, {175, 180}};
  const int NS = sizeof(slots) / sizeof(slots[0]);
  const int reps = getenv("REPS") ? atoi(getenv("REPS")) : 2;
  for (int r = 0; r < reps; ++r) {
    for (int bpc = 1; bpc <= 2; ++bpc) {
      const int grid = cus * bpc;
      const float tb = timeit(k_base<4>, grid, a, 10);
      printf("{\"round\": %d, \"variant\": \"base4\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"frac\": %.4f}\n",
             r, bpc, tb, 20.0 * 4 * n4 / (tb * 1e-3) / 8e12);
      fflush(stdout);
      for (int s = 0; s < NS; ++s) {
        A p = a;
        p.rt = slots[s][0] * bpc;
        p.wt = slots[s][1] * bpc;
        const float t = timeit(k_phase<4>, grid, p, 10);
        printf("{\"round\": %d, \"variant\": \"phase4\", \"blocks_per_cu\": %d, \"rt\": %u, \"wt\": %u, "
               "\"ms\": %.4f, \"frac\": %.4f}\n",
               r, bpc, p.rt, p.wt, t, 20.0 * 4 * n4 / (t * 1e-3) / 8e12);
        fflush(stdout);
      }
    }
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
