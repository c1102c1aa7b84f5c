// vmm_arena_probe.cpp — how far into one hipMemAddressReserve'd range can
// hipMemMap place chunks? (tooling, not product).  Reserves ARENA_GB of address
// space once, then maps one physical chunk of CHUNK_MB at successive fresh
// offsets (bump pointer, like bdl_vmm_map), touches it, unmaps it, and prints
// the first offset whose map fails (or the end of the arena).
//   hipcc --offload-arch=gfx950 -O2 -o tools/bin/vmm_arena_probe tools/vmm_arena_probe.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

int main() {
  const size_t arena_gb = getenv("ARENA_GB") ? atol(getenv("ARENA_GB")) : 4096;
  const size_t chunk = (getenv("CHUNK_MB") ? atol(getenv("CHUNK_MB")) : 586) << 20;
  const size_t stride = (getenv("STRIDE_GB") ? atol(getenv("STRIDE_GB")) : 8) << 30;
  hipMemAllocationProp prop;
  memset(&prop, 0, sizeof prop);
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
  size_t rgran = 0;
  hipMemGetAllocationGranularity(&rgran, &prop, hipMemAllocationGranularityRecommended);
  void* base = nullptr;
  hipError_t e = hipMemAddressReserve(&base, arena_gb << 30, 2 << 20, nullptr, 0);
  printf("{\"reserve_gb\": %zu, \"rc\": \"%s\", \"base\": \"%p\", \"gran_min\": %zu, \"gran_rec\": %zu}\n",
         arena_gb, hipGetErrorString(e), base, gran, rgran);
  if (e != hipSuccess) return 1;
  hipMemGenericAllocationHandle_t h;
  e = hipMemCreate(&h, chunk, &prop, 0);
  if (e != hipSuccess) {
    printf("{\"create\": \"%s\"}\n", hipGetErrorString(e));
    return 1;
  }
  hipMemAccessDesc acc;
  memset(&acc, 0, sizeof acc);
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = 0;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  size_t off = 0, ok = 0;
  for (; off + chunk <= (arena_gb << 30); off += stride) {
    char* p = (char*)base + off;
    e = hipMemMap(p, chunk, 0, h, 0);
    if (e == hipSuccess) e = hipMemSetAccess(p, chunk, &acc, 1);
    if (e == hipSuccess) e = hipMemset(p, 1, 4096);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
      printf("{\"fail_offset_gb\": %.1f, \"va\": \"%p\", \"rc\": \"%s\", \"ok_maps\": %zu}\n",
             off / 1073741824.0, (void*)p, hipGetErrorString(e), ok);
      (void)hipGetLastError();
      return 0;
    }
    hipMemUnmap(p, chunk);
    ++ok;
  }
  printf("{\"all_ok\": true, \"ok_maps\": %zu, \"last_offset_gb\": %.1f}\n", ok,
         off / 1073741824.0);
  // further reservations of the same size (an arena that ran out is followed
  // by another): map one chunk at the start, middle and end of each
  const int extra = getenv("ARENAS") ? atoi(getenv("ARENAS")) - 1 : 3;
  for (int k = 0; k < extra; ++k) {
    void* b2 = nullptr;
    e = hipMemAddressReserve(&b2, arena_gb << 30, 2 << 20, nullptr, 0);
    printf("{\"arena\": %d, \"reserve\": \"%s\", \"base\": \"%p\"", k + 1, hipGetErrorString(e), b2);
    if (e != hipSuccess) {
      printf("}\n");
      (void)hipGetLastError();
      break;
    }
    const size_t offs[] = {0, (arena_gb << 29), (arena_gb << 30) - chunk};
    for (size_t o : offs) {
      char* p = (char*)b2 + (o & ~(size_t)((2 << 20) - 1));
      e = hipMemMap(p, chunk, 0, h, 0);
      if (e == hipSuccess) e = hipMemSetAccess(p, chunk, &acc, 1);
      if (e == hipSuccess) e = hipMemset(p, 1, 4096);
      if (e == hipSuccess) e = hipDeviceSynchronize();
      printf(", \"map_at_%.0fgb\": \"%s\"", (p - (char*)b2) / 1073741824.0, hipGetErrorString(e));
      if (e == hipSuccess) hipMemUnmap(p, chunk);
      (void)hipGetLastError();
    }
    printf("}\n");
    fflush(stdout);
  }
  return 0;
}
