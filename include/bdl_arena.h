/* bdl_arena.h — gradient arena of the fused SG-MCMC library.
 *
 * Not part of the reference's interface.  The reference reads each
 * parameter's gradient where autograd leaves it (`p.grad`,
 * methods/csghmc.py:741-778); so do the product Runners ("tensor" gradient
 * mode, bdl_step_args.grad_base).  Left to torch's caching allocator, the
 * ~300 gradient tensors of a ViT-L/32 backward land in ~100 separately
 * hipMalloc'd segments wherever the allocator finds them, and the update's
 * sweep over them ran up to 1.8 % behind the same sweep over one allocation
 * (DESIGN.md §3).  The arena is one device reservation that a
 * torch.cuda.MemPool carves its segments from (torch.cuda.memory.
 * CUDAPluggableAllocator with bdl_arena_alloc / bdl_arena_free); the Runners
 * route the backward pass's allocations to that pool
 * (bayesdll_amd/arena.py), so every gradient tensor is a sub-range of one
 * reservation, step after step the same one.
 *
 * Regions: bdl_arena_reserve makes a new region of at least `bytes` current
 * on a device.  An allocation is carved from the current region (2 MiB
 * aligned, bump pointer from the top down: a backward pass allocates the last
 * layers' gradients first, so they land in the flat vector's address order);
 * when it does not fit, a new region of max(2 x the
 * request, the current region's size) becomes current.  A region whose
 * carvings are all freed is reset (current) or released (hipFree, otherwise).
 * Thread-safe.  Errors: negative bdl_status (bdl_sgmcmc.h), bdl_last_error(). */
#ifndef BDL_ARENA_H
#define BDL_ARENA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Reserve a region of at least `bytes` (rounded up to 2 MiB) on `device` and
 * make it the device's current region.  Returns BDL_OK or an error. */
int bdl_arena_reserve(int32_t device, int64_t bytes);

/* torch.cuda.memory.CUDAPluggableAllocator entry points (its
 * `void* alloc(size_t, int, stream)` / `void free(void*, size_t, int, stream)`
 * signatures).  The caching allocator of the MemPool asks for whole segments
 * (2 MiB multiples) and caches them; bdl_arena_alloc returns NULL only when
 * the device is out of memory. */
void* bdl_arena_alloc(size_t size, int device, void* hip_stream);
void bdl_arena_free(void* ptr, size_t size, int device, void* hip_stream);

/* Per-device statistics into out[0..nout): [0] regions, [1] bytes reserved,
 * [2] bytes carved, [3] live carvings, [4] carvings so far, [5] regions
 * created because the current one was full, [6] base address of the current
 * region, [7] its size.  Needs nout >= 8. */
int bdl_arena_stats(int32_t device, int64_t* out, int32_t nout);

/* 1 if [ptr, ptr + bytes) lies inside one live region of `device`, else 0. */
int bdl_arena_contains(int32_t device, const void* ptr, int64_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* BDL_ARENA_H */
