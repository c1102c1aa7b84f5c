/* bdl_placement.h — physical-chunk placement of the chain's swept vectors.
 *
 * Not part of the reference's interface: the reference keeps every vector in
 * torch's caching allocator (methods/csghmc.py:727-730 momentum_buffer,
 * methods/sgld.py:98 parameters_to_vector).  On MI355X the fused step's HBM
 * rate depends on which PHYSICAL memory the two vectors it rewrites in place
 * (theta and the momentum / SGD buffer) land on: the same sweep runs ~0.95 ms
 * or ~1.05 ms for ViT-L/32 depending on the pair of physical regions
 * (profiles/round2/placement/, DESIGN.md §4 "Placement").  These entry points
 * let the host allocate physical chunks (hipMemCreate), time pairs of them,
 * and map the chosen chunks into one contiguous virtual range per vector
 * (hipMemAddressReserve + hipMemMap), so the pairing is chosen chunk by chunk
 * instead of drawn by the allocator.
 *
 * Ownership: a chunk handle is released with bdl_chunk_release once it is
 * mapped where it is needed (the physical memory lives until its last mapping
 * is unmapped); a mapping is removed with bdl_vmm_unmap after all work that
 * reads it has completed (the caller synchronises).  Errors: negative
 * bdl_status (bdl_sgmcmc.h) and bdl_last_error(). */
#ifndef BDL_PLACEMENT_H
#define BDL_PLACEMENT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Allocation granularity (bytes) of physical chunks on `device`; chunk sizes
 * passed below must be multiples of it. */
int bdl_chunk_granularity(int32_t device, uint64_t* bytes);

/* Create one physical chunk of `bytes` on `device` (not yet mapped). */
int bdl_chunk_create(int32_t device, uint64_t bytes, uint64_t* handle);

/* Drop the caller's reference to a chunk (freed when no mapping remains). */
int bdl_chunk_release(uint64_t handle);

/* Take nchunks * chunk_bytes (chunk_bytes a multiple of 2 MiB) of virtual
 * address space from the library's arena — one large reservation made at the
 * first call, bump-allocated, no sub-range ever handed out twice — map
 * handles[i] at offset i * chunk_bytes, grant `device` read/write; *va
 * receives the base.  A chunk may be mapped at several places. */
int bdl_vmm_map(int32_t device, const uint64_t* handles, int32_t nchunks, uint64_t chunk_bytes,
                void** va);

/* Unmap a range returned by bdl_vmm_map (total = nchunks * chunk_bytes); its
 * physical chunks are freed once unmapped everywhere and released.  The
 * virtual sub-range is never handed out again: on this driver stack an
 * address mapped once keeps translating to its first backing after the unmap
 * (measured, tools/vmm_alias_repro.cpp). */
int bdl_vmm_unmap(void* va, uint64_t total_bytes);

/* Virtual address space the arena holds (*reserved_bytes) and the sub-ranges
 * handed out so far (*mapped_bytes); either pointer may be null. */
int bdl_vmm_arena_info(uint64_t* reserved_bytes, uint64_t* mapped_bytes);

/* Measurement: the bare access mix of a sweep — nreads 16-B streams read and
 * nwrites written per float4 group over n fp32 elements, no arithmetic beyond
 * a sum, in the step kernels' loop shape and launch geometry (blocks_per_cu
 * workgroups of 256 per CU, unroll 1 / 2 / 4 groups per lane in flight).
 * Timed on a kernel's own buffers (writes may alias reads, as a step's
 * in-place vectors do) it is the HBM ceiling of that exact access pattern on
 * that exact memory.  Supported (nreads, nwrites): (2,1) posterior draw,
 * (3,2) explore / moments, (4,2) SGLD, (3,4) Welford init, (5,4) Welford
 * collect, (7,5) Adam-SGHMC + SGD.  The written vectors receive reads[0]
 * (+ 0 * the others): their contents are destroyed. */
int bdl_stream_mix(const float* const* reads, int32_t nreads, float* const* writes,
                   int32_t nwrites, int64_t n, int32_t blocks_per_cu, int32_t unroll,
                   void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* BDL_PLACEMENT_H */
