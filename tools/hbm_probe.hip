// hbm_probe.hip — HBM ceilings on this GPU for the access mix of the fused
// SG-MCMC step (tooling, not product).  Times, with hipEvents, over 1.2 GB fp32
// vectors (far beyond the 256 MiB Infinity Cache):
//   read1   : 1 read stream  (sum, one atomic per block)
//   write1  : 1 write stream
//   copy    : 1 read + 1 write
//   r3w2    : 3 reads + 2 writes (the explore step's mix, trivial arithmetic)
//   r2w1    : 2 reads + 1 write to a third vector (the posterior-sample mix)
// each with temporal / non-temporal access and several grid sizes, grid-stride,
// 256-thread blocks, `U` float4 per lane in flight.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// XCD remap (XCD=1): workgroups are dispatched round-robin over the 8 XCDs
// (block b runs on XCD b % 8); remapped, XCD x sweeps the logical blocks
// [x*G/8, (x+1)*G/8) of every grid-stride window, i.e. one contiguous 1/8 of it.
template <bool XCD>
__device__ __forceinline__ long logical_block() {
  if constexpr (!XCD) return blockIdx.x;
  const long g = gridDim.x, per = g / 8;
  const long b = blockIdx.x;
  return (g % 8 == 0) ? (b % 8) * per + b / 8 : b;
}

template <int MODE, bool NT, int U, bool XCD = false>
__global__ __launch_bounds__(256) void probe(const f4* __restrict__ a, const f4* __restrict__ b,
                                             const f4* __restrict__ c, f4* __restrict__ x,
                                             f4* __restrict__ y, long n4, float* sink) {
  const long step = (long)gridDim.x * 256 * U;
  f4 acc = {0, 0, 0, 0};
  for (long base = logical_block<XCD>() * 256 * U; base < n4; base += step) {
    f4 ra[U], rb[U], rc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * 256 + threadIdx.x;
      if (i < n4) {
        if (MODE != 1) ra[u] = ld<NT>(a + i);
        if (MODE >= 3) rb[u] = ld<NT>(b + i);
        if (MODE == 3 || MODE == 4) rc[u] = ld<NT>(c + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * 256 + threadIdx.x;
      if (i >= n4) continue;
      if (MODE == 0) acc += ra[u];
      if (MODE == 1) st<NT>(x + i, f4{1.f, 2.f, 3.f, 4.f});
      if (MODE == 2) st<NT>(x + i, ra[u]);
      if (MODE == 5) st<NT>(x + i, ra[u] + rb[u] * 0.5f);
      if (MODE == 3 || MODE == 4) {
        const f4 v = rc[u] * 0.82f - (ra[u] + rb[u]) * 1e-4f;
        // MODE 3: results to two other buffers; MODE 4: in place (a, c), as the sampler
        st<NT>(MODE == 3 ? x + i : const_cast<f4*>(a) + i, ra[u] + v);
        st<NT>(MODE == 3 ? y + i : const_cast<f4*>(c) + i, v);
      }
    }
  }
  if (MODE == 0 && (acc.x + acc.y + acc.z + acc.w) == 12345.f) sink[0] = 1.f;
}

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

template <int MODE, bool NT, int U, bool XCD = false>
float run(int grid, const f4* a, const f4* b, const f4* c, f4* x, f4* y, long n4, float* sink,
          int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) probe<MODE, NT, U, XCD><<<grid, 256>>>(a, b, c, x, y, n4, sink);
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) probe<MODE, NT, U, XCD><<<grid, 256>>>(a, b, c, x, y, n4, sink);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms / reps;
}

template <int MODE, bool NT, int U, bool XCD = false>
void sweep(const char* name, int cus, const f4* a, const f4* b, const f4* c, f4* x, f4* y, long n4,
           float* sink) {
  const double bytes_per_el = (MODE == 0 || MODE == 1) ? 4 : (MODE == 2 ? 8 : (MODE == 5 ? 12 : 20));
  const int bpcs[] = {1, 2, 3, 4};
  for (int bpc : bpcs) {
    const float ms = run<MODE, NT, U, XCD>(cus * bpc, a, b, c, x, y, n4, sink, 20);
    printf("{\"pattern\": \"%s\", \"nt\": %d, \"unroll\": %d, \"blocks_per_cu\": %d, "
           "\"xcd_remap\": %d, \"ms\": %.4f, \"gbs\": %.1f}\n",
           name, NT ? 1 : 0, U, bpc, XCD ? 1 : 0, ms, bytes_per_el * n4 * 4 / ms / 1e6);
    fflush(stdout);
  }
}

int main() {
  const long n = 306535400;  // ViT-L/32 parameter count
  const long n4 = n / 4;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  f4 *a, *b, *c, *x, *y;
  float* sink;
  CHECK(hipMalloc(&a, n4 * sizeof(f4)));
  CHECK(hipMalloc(&b, n4 * sizeof(f4)));
  CHECK(hipMalloc(&c, n4 * sizeof(f4)));
  CHECK(hipMalloc(&x, n4 * sizeof(f4)));
  CHECK(hipMalloc(&y, n4 * sizeof(f4)));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(a, 0, n4 * sizeof(f4)));
  CHECK(hipMemset(b, 0, n4 * sizeof(f4)));
  CHECK(hipMemset(c, 0, n4 * sizeof(f4)));
  const char* which = getenv("PROBE") ? getenv("PROBE") : "all";
  const bool all = !strcmp(which, "all");
  if (!strcmp(which, "xcd")) {  // XCD-remapped vs round-robin block order, the explore mix
    for (int rep = 0; rep < 2; ++rep) {
      sweep<4, true, 4, false>("r3w2_inplace", cus, a, b, c, x, y, n4, sink);
      sweep<4, true, 4, true>("r3w2_inplace", cus, a, b, c, x, y, n4, sink);
      sweep<4, true, 2, false>("r3w2_inplace", cus, a, b, c, x, y, n4, sink);
      sweep<4, true, 2, true>("r3w2_inplace", cus, a, b, c, x, y, n4, sink);
    }
    CHECK(hipDeviceSynchronize());
    return 0;
  }
  if (!strcmp(which, "r2w1")) {  // the posterior-sample mix
    for (int rep = 0; rep < 2; ++rep) {
      sweep<5, true, 1>("r2w1", cus, a, b, c, x, y, n4, sink);
      sweep<5, true, 2>("r2w1", cus, a, b, c, x, y, n4, sink);
      sweep<5, true, 4>("r2w1", cus, a, b, c, x, y, n4, sink);
      sweep<5, false, 2>("r2w1", cus, a, b, c, x, y, n4, sink);
      sweep<5, false, 4>("r2w1", cus, a, b, c, x, y, n4, sink);
    }
    CHECK(hipDeviceSynchronize());
    return 0;
  }
  if (all) {
    sweep<0, false, 2>("read1", cus, a, b, c, x, y, n4, sink);
    sweep<0, true, 2>("read1", cus, a, b, c, x, y, n4, sink);
    sweep<1, false, 2>("write1", cus, a, b, c, x, y, n4, sink);
    sweep<1, true, 2>("write1", cus, a, b, c, x, y, n4, sink);
    sweep<2, false, 2>("copy", cus, a, b, c, x, y, n4, sink);
    sweep<2, true, 2>("copy", cus, a, b, c, x, y, n4, sink);
    sweep<3, false, 2>("r3w2", cus, a, b, c, x, y, n4, sink);
  }
  sweep<3, true, 1>("r3w2", cus, a, b, c, x, y, n4, sink);
  sweep<3, true, 2>("r3w2", cus, a, b, c, x, y, n4, sink);
  sweep<3, true, 4>("r3w2", cus, a, b, c, x, y, n4, sink);
  sweep<4, true, 1>("r3w2_inplace", cus, a, b, c, x, y, n4, sink);
  sweep<4, true, 2>("r3w2_inplace", cus, a, b, c, x, y, n4, sink);
  sweep<4, true, 4>("r3w2_inplace", cus, a, b, c, x, y, n4, sink);
  CHECK(hipDeviceSynchronize());
  return 0;
}
