// Minimal repro of the round-2 virtual-range aliasing finding (DESIGN.md §4
// "Virtual ranges"), in plain HIP: no torch, no product code.  ONE scenario
// per process (argv[1]), so no earlier scenario's recycled ranges leak in.
//
// Setup: 4 physical chunks (hipMemCreate), each also mapped alone as a "view"
// (as the placement search keeps them), all zero.  Round 1 maps chunks 0, 1
// back to back into one reserved range R1 and writes 1.0 through it.  The
// scenario then tears R1 down and round 2 maps chunks 2, 3 into a range R2
// and writes 2.0 through it.  The views must then read 1, 1, 2, 2.
//
//   free_reuse       hipMemUnmap(R1, whole); hipMemAddressFree(R1); R2 = new
//                    reservation (the round-2 product: it gets R1's address)
//   free_reuse_sync  the same with hipDeviceSynchronize around the unmap
//   per_chunk_free   one hipMemUnmap per chunk instead of one over the range
//   remap_in_place   R1 stays reserved; chunks 2, 3 mapped into R1 itself
//   fresh_range      R1 stays reserved (unmapped); R2 = new reservation
//                    (the round-2 fix)
//   late_views       as free_reuse but no views during rounds 1 and 2 (the
//                    chunks are mapped once each, like an ordinary vector);
//                    views are created only for the final read
//   after_hipfree    R1 stays reserved; R2 is reserved at the address of a
//                    hipMalloc'd block (filled with 7, then hipFree'd) —
//                    hinted, so the reservation can land there: can memory
//                    torch's allocator used and freed be mapped safely?
//   arena            R1 and R2 are consecutive sub-ranges of ONE large
//                    reservation made at the start, never reused (the
//                    product's scheme since round 4: bdl_vmm_map bump-allocates
//                    from an arena)
//
// Output: one JSON line (scenario, whether R2 == R1, each chunk's min / max
// over 257 strided samples, "ok").  Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x,          \
                   hipGetErrorString(e_));                                      \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void fill_kernel(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// out[k] = p[k * stride] for k < m, out[m] = p[n - 1]
__global__ void gather_kernel(const float* p, size_t n, size_t stride, size_t m, float* out) {
  const size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (k < m) out[k] = p[k * stride];
  if (k == m) out[m] = p[n - 1];
}

static int g_dev = 0;
static size_t g_cb = 0;
static hipMemAllocationProp g_prop;

static void set_rw(void* va, size_t bytes) {
  hipMemAccessDesc acc;
  std::memset(&acc, 0, sizeof acc);
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = g_dev;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, bytes, &acc, 1));
}

static void fill(void* p, size_t nfloat, float v) {
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, (float*)p, nfloat, v);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
}

static void* map_range(const hipMemGenericAllocationHandle_t* h, int k) {
  void* va = nullptr;
  CK(hipMemAddressReserve(&va, k * g_cb, 2 << 20, nullptr, 0));
  for (int c = 0; c < k; ++c) CK(hipMemMap((char*)va + c * g_cb, g_cb, 0, h[c], 0));
  set_rw(va, k * g_cb);
  return va;
}

static void minmax(const void* p, size_t n, float* lo, float* hi) {
  const size_t m = 256;
  static float* dout = nullptr;
  if (!dout) CK(hipMalloc(&dout, (m + 1) * sizeof(float)));
  std::vector<float> host(m + 1);
  hipLaunchKernelGGL(gather_kernel, dim3(2), dim3(256), 0, 0, (const float*)p, n, n / m, m, dout);
  CK(hipGetLastError());
  CK(hipMemcpy(host.data(), dout, (m + 1) * sizeof(float), hipMemcpyDeviceToHost));
  *lo = *hi = host[0];
  for (float v : host) {
    if (v < *lo) *lo = v;
    if (v > *hi) *hi = v;
  }
}

int main(int argc, char** argv) {
  const std::string sc = argc > 1 ? argv[1] : "free_reuse";
  const size_t chunk_mb = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 64;
  CK(hipSetDevice(g_dev));
  std::memset(&g_prop, 0, sizeof g_prop);
  g_prop.type = hipMemAllocationTypePinned;
  g_prop.location.type = hipMemLocationTypeDevice;
  g_prop.location.id = g_dev;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &g_prop, hipMemAllocationGranularityRecommended));
  g_cb = ((chunk_mb << 20) + gran - 1) / gran * gran;
  const size_t nf = g_cb / sizeof(float);
  const bool views_early = sc != "late_views";

  hipMemGenericAllocationHandle_t h[4];
  void* view[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int c = 0; c < 4; ++c) {
    CK(hipMemCreate(&h[c], g_cb, &g_prop, 0));
    if (views_early) {
      view[c] = map_range(&h[c], 1);
      fill(view[c], nf, 0.0f);
    }
  }
  if (!views_early) {  // zero the chunks through a temporary range each, kept reserved
    for (int c = 0; c < 4; ++c) {
      void* t = map_range(&h[c], 1);
      fill(t, nf, 0.0f);
      CK(hipMemUnmap(t, g_cb));  // never freed: no recycling from here
    }
  }
  void* arena = nullptr;
  if (sc == "arena") CK(hipMemAddressReserve(&arena, 64 * g_cb, 2 << 20, nullptr, 0));
  void* r1 = nullptr;
  if (sc == "arena") {
    r1 = arena;
    for (int c = 0; c < 2; ++c) CK(hipMemMap((char*)r1 + c * g_cb, g_cb, 0, h[c], 0));
    set_rw(r1, 2 * g_cb);
  } else {
    r1 = map_range(&h[0], 2);
  }
  fill(r1, 2 * nf, 1.0f);
  void* freed = nullptr;  // after_hipfree: the address of a freed hipMalloc block
  if (sc == "after_hipfree") {
    CK(hipMalloc(&freed, 2 * g_cb));
    fill(freed, 2 * nf, 7.0f);
    CK(hipFree(freed));
    CK(hipDeviceSynchronize());
  }

  void* r2 = nullptr;
  const bool sync = sc == "free_reuse_sync";
  if (sync) CK(hipDeviceSynchronize());
  if (sc == "per_chunk_free") {
    for (int c = 0; c < 2; ++c) CK(hipMemUnmap((char*)r1 + c * g_cb, g_cb));
  } else {
    CK(hipMemUnmap(r1, 2 * g_cb));
  }
  if (sync) CK(hipDeviceSynchronize());
  if (sc == "remap_in_place") {
    for (int c = 0; c < 2; ++c) CK(hipMemMap((char*)r1 + c * g_cb, g_cb, 0, h[2 + c], 0));
    set_rw(r1, 2 * g_cb);
    r2 = r1;
  } else if (sc == "fresh_range") {
    r2 = map_range(&h[2], 2);
  } else if (sc == "arena") {
    r2 = (char*)arena + 2 * g_cb;  // the next sub-range: never mapped before
    for (int c = 0; c < 2; ++c) CK(hipMemMap((char*)r2 + c * g_cb, g_cb, 0, h[2 + c], 0));
    set_rw(r2, 2 * g_cb);
  } else if (sc == "after_hipfree") {
    CK(hipMemAddressReserve(&r2, 2 * g_cb, 2 << 20, freed, 0));
    for (int c = 0; c < 2; ++c) CK(hipMemMap((char*)r2 + c * g_cb, g_cb, 0, h[2 + c], 0));
    set_rw(r2, 2 * g_cb);
  } else {
    CK(hipMemAddressFree(r1, 2 * g_cb));
    r2 = map_range(&h[2], 2);
  }
  fill(r2, 2 * nf, 2.0f);

  if (!views_early)
    for (int c = 0; c < 4; ++c) view[c] = map_range(&h[c], 1);
  float lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
  for (int c = 0; c < 4; ++c) minmax(view[c], nf, &lo[c], &hi[c]);
  bool ok = true;
  for (int c = 0; c < 4; ++c) {
    const float want = c < 2 ? 1.0f : 2.0f;
    ok = ok && lo[c] == want && hi[c] == want;
  }
  std::printf("{\"scenario\":\"%s\",\"chunk_bytes\":%zu,\"r2_is_r1\":%s,"
              "\"r2_at_freed_hipmalloc\":%s,\"chunks_minmax\":"
              "[[%g,%g],[%g,%g],[%g,%g],[%g,%g]],\"ok\":%s}\n",
              sc.c_str(), g_cb, r2 == r1 ? "true" : "false",
              (freed && r2 == freed) ? "true" : "false", lo[0], hi[0], lo[1], hi[1], lo[2],
              hi[2], lo[3], hi[3], ok ? "true" : "false");
  std::fflush(stdout);
  CK(hipDeviceSynchronize());
  return 0;  // the process exit returns every mapping and chunk to the driver
}
