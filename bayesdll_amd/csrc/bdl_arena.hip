// bdl_arena.hip — the gradient arena (include/bdl_arena.h): one device
// reservation per device that torch.cuda.MemPool carves its segments from,
// so the per-tensor gradients a backward pass produces are sub-ranges of ONE
// allocation (the update then reads them as it reads a flat vector: same
// physical placement class).  Host code only.
//
// The caching allocator above it asks for whole segments (2 MiB multiples, or
// 20 MiB for the 1-10 MiB size class) and keeps them cached for the lifetime
// of the pool, so in steady state this code is not called at all: a step's
// gradients come back at the same addresses from the pool's cache.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "bdl_arena.h"
#include "bdl_sgmcmc.h"

namespace bdl {
void set_last_error(const std::string& msg);  // bdl_api.hip
}

namespace {

constexpr int64_t kAlign = 2 << 20;  // carve granularity: the caching allocator's large page

struct Region {
  char* base = nullptr;
  int64_t size = 0;
  int64_t bump = 0;  // bytes carved, from the top: [base + size - bump, base + size) is in use
  int64_t live = 0;  // carvings not yet freed
};

struct DeviceArena {
  std::vector<Region> regions;  // regions.back() is current
  int64_t carvings = 0;
  int64_t grown = 0;
};

// never destroyed: the caching allocator above may return segments while the
// process exits, after this library's static destructors would have run
std::mutex& g_mu = *new std::mutex;
DeviceArena* const g_dev = new DeviceArena[64];

int64_t round_up(int64_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

// hipMalloc on `device`, restoring the caller's current device.
char* device_malloc(int device, int64_t bytes) {
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != device && hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  void* p = nullptr;
  const hipError_t err = hipMalloc(&p, (size_t)bytes);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  if (err != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return (char*)p;
}

void device_free(int device, void* p) {
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != device) (void)hipSetDevice(device);
  (void)hipFree(p);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  (void)hipGetLastError();
}

bool new_region(int device, int64_t bytes) {
  DeviceArena& d = g_dev[device];
  const int64_t sz = round_up(std::max<int64_t>(bytes, kAlign));
  char* p = device_malloc(device, sz);
  if (!p) return false;
  // the old current region is retired: released as soon as it holds nothing
  if (!d.regions.empty() && d.regions.back().live == 0) {
    device_free(device, d.regions.back().base);
    d.regions.pop_back();
  }
  Region r;
  r.base = p;
  r.size = sz;
  d.regions.push_back(r);
  return true;
}

bool valid_device(int device) { return device >= 0 && device < 64; }

}  // namespace

extern "C" {

int bdl_arena_reserve(int32_t device, int64_t bytes) {
  if (!valid_device(device) || bytes <= 0) {
    bdl::set_last_error("bdl_arena_reserve: bad device or size");
    return BDL_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  if (!new_region(device, bytes)) {
    bdl::set_last_error("bdl_arena_reserve: hipMalloc of " + std::to_string(bytes) +
                        " bytes failed");
    return BDL_ERR_LAUNCH;
  }
  return BDL_OK;
}

void* bdl_arena_alloc(size_t size, int device, void* hip_stream) {
  (void)hip_stream;  // the pool above orders reuse on streams; carving is stream-free
  if (!valid_device(device)) return nullptr;
  const int64_t want = round_up(std::max<int64_t>((int64_t)size, 1));
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& d = g_dev[device];
  if (d.regions.empty() || d.regions.back().bump + want > d.regions.back().size) {
    const int64_t cur = d.regions.empty() ? 0 : d.regions.back().size;
    if (!new_region(device, std::max<int64_t>(2 * want, cur))) return nullptr;
    ++d.grown;
  }
  // carved top-down: a backward pass allocates the last layers' gradients
  // first, so the parameters' gradients land in increasing address order
  // with the parameter index, as in the flat vector (the explore sweep over
  // reverse-ordered gradient tensors ran 0.7-1.3 % slower at its 1 x 4
  // geometry on two boxes, tools/grad_layout_probe.py)
  Region& r = d.regions.back();
  r.bump += want;
  char* p = r.base + r.size - r.bump;
  ++r.live;
  ++d.carvings;
  return p;
}

void bdl_arena_free(void* ptr, size_t size, int device, void* hip_stream) {
  (void)size;
  (void)hip_stream;
  if (!ptr || !valid_device(device)) return;
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceArena& d = g_dev[device];
  for (size_t i = 0; i < d.regions.size(); ++i) {
    Region& r = d.regions[i];
    if ((char*)ptr < r.base || (char*)ptr >= r.base + r.size) continue;
    if (--r.live > 0) return;
    if (i + 1 == d.regions.size()) {
      r.bump = 0;  // the current region is empty again: carve it from the start
    } else {
      device_free(device, r.base);
      d.regions.erase(d.regions.begin() + (long)i);
    }
    return;
  }
}

int bdl_arena_stats(int32_t device, int64_t* out, int32_t nout) {
  if (!out) {
    bdl::set_last_error("bdl_arena_stats: null out");
    return BDL_ERR_NULL;
  }
  if (!valid_device(device) || nout < 8) {
    bdl::set_last_error("bdl_arena_stats: bad device or nout < 8");
    return BDL_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  const DeviceArena& d = g_dev[device];
  int64_t reserved = 0, carved = 0, live = 0;
  for (const Region& r : d.regions) {
    reserved += r.size;
    carved += r.bump;
    live += r.live;
  }
  out[0] = (int64_t)d.regions.size();
  out[1] = reserved;
  out[2] = carved;
  out[3] = live;
  out[4] = d.carvings;
  out[5] = d.grown;
  out[6] = d.regions.empty() ? 0 : (int64_t)(uintptr_t)d.regions.back().base;
  out[7] = d.regions.empty() ? 0 : d.regions.back().size;
  return BDL_OK;
}

int bdl_arena_contains(int32_t device, const void* ptr, int64_t bytes) {
  if (!valid_device(device) || !ptr || bytes < 0) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  for (const Region& r : g_dev[device].regions)
    if ((const char*)ptr >= r.base + r.size - r.bump && (const char*)ptr + bytes <= r.base + r.size)
      return 1;
  return 0;
}

}  // extern "C"
