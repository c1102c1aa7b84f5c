// layout_probe.hip — does interleaving a sampler's INTERNAL state streams in one
// allocation (tiles of T float4 groups per stream, stream-major inside a tile)
// make the sweep independent of where the allocations land physically?
// (tooling, not product).  Each trial allocates fresh buffers (kept until the
// end, so every trial lands on other physical memory) for the separate layout
// (one hipMalloc per stream, as torch's allocator gives them) and for every
// tile size, then times each layout (hipEvents, 10 launches, trivial
// arithmetic, nt loads / stores, 256-thread blocks, 2 float4 per lane).
//   PROBE=adam    theta rw, g r, prior r (external) + 4 rw internal (v_mom, m, v, buf)
//   PROBE=draw    out w (external) + 2 r internal (m1, m2)
//   PROBE=collect theta rw, g r (external) + 3 rw internal (mom, m1, m2)
//   PROBE=sgld    theta rw, g r (external) + prior r, buf rw internal
//   PROBE=explore theta rw, g r (external) + mom rw internal (no interleave possible)
//   PROBE=pair    g r (external) + theta, mom rw internal: the explore mix with
//                 theta / mom interleaved (not shippable: theta is the
//                 parameters' storage) — tests the placement hypothesis
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr int kU = 2;
constexpr int kMaxS = 4;

struct Args {
  f4* ext_rw;             // theta or null
  const f4* ext_r[2];     // g, prior (null if absent)
  f4* ext_w;              // write-only (draw output) or null
  f4* in[kMaxS];          // separate layout: one pointer per internal stream
  f4* tiled;              // tiled layout base
  long tile;              // float4 groups per stream per tile (0 = separate)
  int ns;                 // internal streams
  unsigned rwmask;        // bit s: internal stream s is written back
  long n4;
  long nseg;              // sweep: 1 = grid-stride over the whole vector; S = S segments,
                          // block b sweeping segment b % S (grid-stride inside it)
};

__device__ __forceinline__ f4* in_ptr(const Args& a, int s, long i) {
  if (a.tile == 0) return a.in[s] + i;
  const long t = i / a.tile, r = i - t * a.tile;
  return a.tiled + (t * a.ns + s) * a.tile + r;
}

template <int NS, bool RW, int NR, bool W>
__global__ __launch_bounds__(256) void probe(const Args a) {
  const long kIt = 256 * kU;
  const long seg = blockIdx.x % a.nseg, per = gridDim.x / a.nseg;
  const long slen = ((a.n4 + a.nseg - 1) / a.nseg + kIt - 1) / kIt * kIt;
  const long lo = seg * slen, hi = lo + slen < a.n4 ? lo + slen : a.n4;
  const long step = per * kIt;
  for (long base = lo + (long)(blockIdx.x / a.nseg) * kIt; base < hi; base += step) {
    f4 th[kU], gr[kU][2], st[kU][NS > 0 ? NS : 1];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const long i = base + u * 256 + threadIdx.x;
      if (i >= hi) continue;
      if (RW) th[u] = __builtin_nontemporal_load(a.ext_rw + i);
#pragma unroll
      for (int r = 0; r < NR; ++r) gr[u][r] = __builtin_nontemporal_load(a.ext_r[r] + i);
#pragma unroll
      for (int s = 0; s < NS; ++s) st[u][s] = __builtin_nontemporal_load(in_ptr(a, s, i));
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const long i = base + u * 256 + threadIdx.x;
      if (i >= hi) continue;
      f4 acc = RW ? th[u] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < NR; ++r) acc += gr[u][r] * 1e-4f;
#pragma unroll
      for (int s = 0; s < NS; ++s) acc += st[u][s] * 0.5f;
      if (RW) __builtin_nontemporal_store(acc, a.ext_rw + i);
      if (W) __builtin_nontemporal_store(acc, a.ext_w + i);
#pragma unroll
      for (int s = 0; s < NS; ++s)
        if (a.rwmask & (1u << s)) __builtin_nontemporal_store(st[u][s] * 0.9f + acc, in_ptr(a, s, i));
    }
  }
}

template <int NS, bool RW, int NR, bool W>
float timeit(const Args& a, int grid, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) probe<NS, RW, NR, W><<<grid, 256>>>(a);
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) probe<NS, RW, NR, W><<<grid, 256>>>(a);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms / reps;
}

static f4* alloc(long n4) {
  f4* p = nullptr;
  CHECK(hipMalloc(&p, n4 * sizeof(f4)));
  CHECK(hipMemset(p, 0, n4 * sizeof(f4)));
  return p;
}

template <int NS, bool RW, int NR, bool W>
void run(const char* name, unsigned rwmask, int trials) {
  const long n = 306535400;  // ViT-L/32 parameter count
  const long n4 = n / 4;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // float4 groups: separate, 16 B, 1 KiB, 4 KiB, 16 KiB (TILES=big: 64 KiB, 1 MiB, 16 MiB, 64 MiB)
  const long small[] = {0, 1, 64, 256, 1024}, big[] = {0, 1024, 65536, 1048576, 4194304};
  const long* tiles = getenv("TILES") && !strcmp(getenv("TILES"), "big") ? big : small;
  int nbytes = 0;
  nbytes += RW ? 8 : 0;
  nbytes += NR * 4 + (W ? 4 : 0);
  for (int s = 0; s < NS; ++s) nbytes += (rwmask & (1u << s)) ? 8 : 4;
  for (int t = 0; t < trials; ++t) {
    Args base{};
    base.n4 = n4;
    base.ns = NS;
    base.rwmask = rwmask;
    if (RW) base.ext_rw = alloc(n4);
    for (int r = 0; r < NR; ++r) base.ext_r[r] = alloc(n4);
    if (W) base.ext_w = alloc(n4);
    for (int ti = 0; ti < 5; ++ti) {
      const long tile = tiles[ti];
      Args a = base;
      a.tile = tile;
      a.nseg = 1;
      if (tile == 0) {
        for (int s = 0; s < NS; ++s) a.in[s] = alloc(n4);
      } else {
        const long nt = (n4 + tile - 1) / tile;
        a.tiled = alloc(nt * tile * NS);
      }
      float best = 1e9f;
      int bbpc = 0;
      char buf[256];
      int len = 0;
      for (int bpc = 1; bpc <= 2; ++bpc) {
        const float ms = timeit<NS, RW, NR, W>(a, cus * bpc, 10);
        len += snprintf(buf + len, sizeof(buf) - len, "%s%.4f", bpc > 1 ? ", " : "", ms);
        if (ms < best) best = ms, bbpc = bpc;
      }
      printf("{\"probe\": \"%s\", \"trial\": %d, \"tile_f4\": %ld, \"ms_by_bpc\": [%s], "
             "\"best_ms\": %.4f, \"bpc\": %d, \"frac\": %.4f}\n",
             name, t, tile, buf, best, bbpc, (double)nbytes * n / (best * 1e-3) / 8e12);
      fflush(stdout);
    }
  }
}

// SWEEP=1: the mix over separate allocations, grid-stride vs segmented sweeps
template <int NS, bool RW, int NR, bool W>
void run_sweeps(const char* name, unsigned rwmask, int trials, long tile) {
  const long n = 306535400, n4 = n / 4;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int nbytes = (RW ? 8 : 0) + NR * 4 + (W ? 4 : 0);
  for (int s = 0; s < NS; ++s) nbytes += (rwmask & (1u << s)) ? 8 : 4;
  for (int t = 0; t < trials; ++t) {
    Args a{};
    a.n4 = n4;
    a.ns = NS;
    a.rwmask = rwmask;
    a.tile = tile;
    if (RW) a.ext_rw = alloc(n4);
    for (int r = 0; r < NR; ++r) a.ext_r[r] = alloc(n4);
    if (W) a.ext_w = alloc(n4);
    if (tile == 0)
      for (int s = 0; s < NS; ++s) a.in[s] = alloc(n4);
    else
      a.tiled = alloc((n4 + tile - 1) / tile * tile * NS);
    for (int bpc = 1; bpc <= 2; ++bpc) {
      const long segs[] = {1, 2, 4, 8, 32, (long)cus * bpc};
      for (long ns : segs) {
        a.nseg = ns;
        const float ms = timeit<NS, RW, NR, W>(a, cus * bpc, 10);
        printf("{\"probe\": \"%s\", \"trial\": %d, \"tile_f4\": %ld, \"bpc\": %d, \"nseg\": %ld, "
               "\"ms\": %.4f, \"frac\": %.4f}\n",
               name, t, tile, bpc, ns, ms, (double)nbytes * n / (ms * 1e-3) / 8e12);
        fflush(stdout);
      }
    }
  }
}

int main() {
  if (getenv("SWEEP")) {
    const char* w = getenv("PROBE") ? getenv("PROBE") : "explore";
    const int trials = getenv("TRIALS") ? atoi(getenv("TRIALS")) : 5;
    if (!strcmp(w, "explore")) run_sweeps<1, true, 1, false>("explore", 0x1, trials, 0);
    else if (!strcmp(w, "pair")) run_sweeps<2, false, 1, false>("pair", 0x3, trials, 64);
    else if (!strcmp(w, "adam")) run_sweeps<4, true, 2, false>("adam", 0xF, trials, 0);
    else if (!strcmp(w, "draw")) run_sweeps<2, false, 0, true>("draw", 0x0, trials, 0);
    CHECK(hipDeviceSynchronize());
    return 0;
  }
  const char* which = getenv("PROBE") ? getenv("PROBE") : "adam";
  const int trials = getenv("TRIALS") ? atoi(getenv("TRIALS")) : 5;
  if (!strcmp(which, "adam")) run<4, true, 2, false>("adam", 0xF, trials);
  else if (!strcmp(which, "draw")) run<2, false, 0, true>("draw", 0x0, trials);
  else if (!strcmp(which, "collect")) run<3, true, 1, false>("collect", 0x7, trials);
  else if (!strcmp(which, "sgld")) run<2, true, 1, false>("sgld", 0x2, trials);
  else if (!strcmp(which, "explore")) run<1, true, 1, false>("explore", 0x1, trials);
  else if (!strcmp(which, "pair")) run<2, false, 1, false>("pair", 0x3, trials);
  else {
    fprintf(stderr, "unknown PROBE %s\n", which);
    return 2;
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
