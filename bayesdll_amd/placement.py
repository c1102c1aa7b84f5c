"""Physical-chunk placement of a chain's swept vectors (include/bdl_placement.h).

Why: the fused step rewrites two vectors in place — theta and the momentum /
SGD buffer — and on MI355X its HBM rate depends on which physical memory
those two land on.  For ViT-L/32 the explore sweep runs ~0.95 ms when the
pair of physical regions is a "fast" pair and ~1.05 ms otherwise; the
relation is a property of the physical regions (moving a vector by 256 B ...
1 GB inside its allocation never changes it; regions come in runs of several
GB, with more than two levels of pair time), invisible from user space, and
torch's allocator hands out whatever
comes next (profiles/round2/placement/, tools/vmm_class_probe.cpp).

How: instead of drawing whole allocations and hoping, each vector is built
from `per` physical chunks (hipMemCreate, ~<= 1 GiB each) mapped back to back
into one virtual range (hipMemMap), so the pairing is chosen chunk by chunk:

  1. allocate K = roles * per + spare chunks, each also mapped on its own;
  2. time the method's production kernel on every ordered chunk pair
     (theta = chunk i, momentum = chunk j, the other roles on further
     chunks) — chunk-sized sweeps, a few launches each;
  3. if the pair times show no clearly fast pair, allocate more spares
     (bounded) first;
  4. candidate assignments: the allocation order, up to COMPOSITES
     greedy ones (seeded by each of the fastest pairs, completed with the
     fastest disjoint pairs; theta / momentum from the pairs, the other roles
     from the remaining chunks in allocation order); each is mapped and timed
     at FULL size — chunk-pair times only rank the seeds; and, competing
     with them, the roles plus TORCH_EXTRA more vectors allocated plainly by
     torch, with up to TORCH_PAIRINGS (theta, mom) pairings among them (on
     some boxes hipMalloc'd memory pairs faster than any chunk composite).
     The fastest is kept; the per-chunk views are unmapped and every handle
     released (unchosen chunks return to the driver at once — nothing is
     parked in torch's cache).

Results never depend on placement (the kernels read the same values from any
address).  The mapped ranges are exposed to torch through
__cuda_array_interface__; a range is unmapped when the last tensor viewing it
is freed — after a device synchronisation, and never inside a HIP-graph
capture (it is then queued and unmapped at the next release point)."""
from __future__ import annotations

import ctypes as C
import itertools
import math
import os

import torch

from . import _lib as L

# chunk size bound: vectors of up to CHUNK_TARGET bytes are one chunk
# (BDL_CHUNK_MB overrides, for placement A/Bs)
CHUNK_TARGET = int(os.environ.get("BDL_CHUNK_MB", "1024")) << 20
ALIGN = 2 << 20          # chunk sizes are multiples of 2 MiB (large-page mappings)
FAST_PAIR = 0.97         # a pair this much faster than the median pair is worth taking
SPARE_ROUNDS = 2         # at most this many rounds of extra chunks while none is seen
COMPOSITES = 6           # full-size candidate assignments timed besides allocation order
# plain torch allocations competing with the chunk composites: TORCH_VECTORS
# of them (the roles + extras; BDL_PLACEMENT_TORCH overrides), every unordered
# pair tried as (theta, mom), up to TORCH_PAIRINGS — consecutive allocations
# often sit in one physical group, and a few more of them reach the next
TORCH_EXTRA = int(os.environ.get("BDL_PLACEMENT_TORCH", "2"))
TORCH_PAIRINGS = 10

_pending = []  # (device index, va, total bytes) whose unmap was deferred (graph capture)


def _unmap_now(dev_index, va, total):
    with torch.cuda.device(dev_index):
        torch.cuda.synchronize()
    L.check(L.lib().bdl_vmm_unmap(C.c_void_p(va), total), "bdl_vmm_unmap")


def release_pending():
    """Unmap ranges whose last tensor died during a graph capture."""
    if not _pending or torch.cuda.is_current_stream_capturing():
        return
    while _pending:
        _unmap_now(*_pending.pop())


class Mapping:
    """One contiguous virtual range mapped from physical chunks (bdl_vmm_map),
    seen by torch as a flat fp32 tensor.  Torch's tensor keeps this object
    alive (from_blob with a reference to it); when it goes, the range is
    unmapped."""

    def __init__(self, dev_index, handles, chunk_bytes, nelem):
        arr = (C.c_uint64 * len(handles))(*handles)
        va = C.c_void_p()
        L.check(L.lib().bdl_vmm_map(dev_index, arr, len(handles), chunk_bytes, C.byref(va)),
                "bdl_vmm_map")
        self.dev_index = dev_index
        self.va = int(va.value)
        self.total = len(handles) * int(chunk_bytes)
        if nelem * 4 > self.total:
            raise ValueError("bayesdll_amd.placement: mapping smaller than its tensor")
        self.__cuda_array_interface__ = {"shape": (int(nelem),), "typestr": "<f4",
                                         "data": (self.va, False), "version": 2}

    def tensor(self):
        with torch.cuda.device(self.dev_index):
            t = torch.as_tensor(self, device=torch.device("cuda", self.dev_index))
        if t.data_ptr() != self.va or t.device.index != self.dev_index:
            raise RuntimeError("bayesdll_amd.placement: torch did not wrap the mapped range")
        return t

    def __del__(self):
        va, self.va = getattr(self, "va", 0), 0
        if not va:
            return
        try:
            if torch.cuda.is_current_stream_capturing():
                _pending.append((self.dev_index, va, self.total))
            else:
                _unmap_now(self.dev_index, va, self.total)
                release_pending()
        except Exception:  # noqa: BLE001 - interpreter shutdown: the driver reclaims it
            pass


class _Chunks:
    """Physical chunks of one size on one device, each also mapped alone."""

    def __init__(self, dev_index, chunk_bytes):
        self.dev_index = dev_index
        self.chunk_bytes = chunk_bytes
        self.handles, self.views = [], []

    def add(self, k):
        lib = L.lib()
        for _ in range(k):
            h = C.c_uint64()
            L.check(lib.bdl_chunk_create(self.dev_index, self.chunk_bytes, C.byref(h)),
                    "bdl_chunk_create")
            self.handles.append(int(h.value))
            m = Mapping(self.dev_index, [int(h.value)], self.chunk_bytes, self.chunk_bytes // 4)
            self.views.append(m.tensor().zero_())

    def release(self):
        """Drop the per-chunk views and every handle (chunks mapped into a
        composite stay alive through that mapping)."""
        self.views = []
        lib = L.lib()
        for h in self.handles:
            L.check(lib.bdl_chunk_release(h), "bdl_chunk_release")
        self.handles = []


def chunk_geometry(n):
    """(chunks per vector, chunk bytes) for an n-element fp32 vector."""
    per = max(1, math.ceil(4 * n / CHUNK_TARGET))
    cb = math.ceil(4 * n / per / ALIGN) * ALIGN
    return per, cb


def _has_fast_pair(times):
    t = sorted(times)
    return t[0] < FAST_PAIR * t[len(t) // 2]


def candidate_assignments(times, nchunks, names, per, limit=COMPOSITES):
    """Chunk ids per role for the full-size candidates: the allocation order
    first, then up to `limit` greedy assignments — each seeded by one of the
    fastest (theta, mom) chunk pairs of `times` ({(i, j): ms}) and completed
    with the fastest pairs disjoint from it; theta / mom take the pairs' chunks,
    the other roles the remaining chunks in allocation order.  Chunk-pair
    times only rank the seeds (they predict a composite weakly), so every
    candidate is timed at full size afterwards.  No chunk serves two roles."""
    it, im = names.index("theta"), names.index("mom")
    ranked = sorted(times, key=times.get)

    def greedy(first):
        used, th, mo = set(), [], []
        for i, j in [first] + ranked:
            if i in used or j in used:
                continue
            th.append(i)
            mo.append(j)
            used.update((i, j))
            if len(th) == per:
                break
        rest = [k for k in range(nchunks) if k not in used]
        out, r = {}, 0
        for q, nm in enumerate(names):
            if q == it:
                out[nm] = th
            elif q == im:
                out[nm] = mo
            else:
                out[nm] = rest[r * per:(r + 1) * per]
                r += 1
        return out

    cands = [{nm: list(range(q * per, (q + 1) * per)) for q, nm in enumerate(names)}]
    for first in ranked:
        if len(cands) > limit:
            break
        c = greedy(first)
        if c not in cands:
            cands.append(c)
    return cands


def place(n, device, names, launcher, time_launch, budget_bytes, spare=None, search=True,
          with_torch=True):
    """Allocate `names` (fp32, n elements each, zeroed) from physical chunks,
    theta / mom paired fast.  `launcher(roles: {name: tensor}, n)` returns a
    zero-argument launch of the sampler's kernel; `time_launch(launch)` its
    median ms.  search=False: chunks mapped in allocation order, no pair
    timing.  Returns ({name: tensor}, info)."""
    import time
    t_start = time.perf_counter()
    dev_index = torch.device(device).index
    if dev_index is None:
        dev_index = torch.cuda.current_device()
    per, cb = chunk_geometry(n)
    nchunk = cb // 4
    nroles = len(names)
    it, im = names.index("theta"), names.index("mom")
    spare = (2 * per if spare is None else spare) if search else 0
    ch = _Chunks(dev_index, cb)
    try:
        ch.add(nroles * per + spare)

        def roles_for(i, j):
            rest = [k for k in range(len(ch.views)) if k not in (i, j)]
            out, r = {}, 0
            for q, nm in enumerate(names):
                if q == it:
                    out[nm] = ch.views[i]
                elif q == im:
                    out[nm] = ch.views[j]
                else:
                    out[nm] = ch.views[rest[r]]
                    r += 1
            return out

        times, rounds = {}, 0
        while search:
            for i in range(len(ch.views)):
                for j in range(len(ch.views)):
                    if i != j and (i, j) not in times:
                        times[(i, j)] = time_launch(launcher(roles_for(i, j), nchunk))
            if _has_fast_pair(times.values()) or rounds >= SPARE_ROUNDS or \
                    (len(ch.views) + spare) * cb > budget_bytes:
                break
            ch.add(spare)
            rounds += 1

        def composite(assign):
            return {nm: Mapping(dev_index, [ch.handles[k] for k in ids], cb, n).tensor()
                    for nm, ids in assign.items()}

        cands = candidate_assignments(times, len(ch.views), names, per)
        best, best_ms, comp_ms, best_src = None, None, [], None
        for c in cands:
            vec = composite(c)
            for v in vec.values():
                v.zero_()
            ms = time_launch(launcher(vec, n))
            comp_ms.append(round(ms, 4))
            if best_ms is None or ms < best_ms:
                best, best_ms, chosen, best_src = vec, ms, c, "chunks"
            del vec
        ms_d = comp_ms[0]
        # torch's own allocations compete too (on some boxes hipMalloc'd
        # memory pairs faster than any chunk composite): the roles' vectors
        # allocated plainly, with every (theta, mom) pairing among them
        torch_ms = []
        if search and with_torch:
            tv = [torch.zeros(n, dtype=torch.float32, device=device)
                  for _ in range(len(names) + max(0, TORCH_EXTRA))]
            pairs = [(it, im)] + [p for p in itertools.combinations(range(len(tv)), 2)
                                  if set(p) != {it, im}]
            for i, j in pairs[:TORCH_PAIRINGS]:
                rest = [k for k in range(len(tv)) if k not in (i, j)]
                vec, r = {}, 0
                for q, nm in enumerate(names):
                    if q == it:
                        vec[nm] = tv[i]
                    elif q == im:
                        vec[nm] = tv[j]
                    else:
                        vec[nm] = tv[rest[r]]
                        r += 1
                ms = time_launch(launcher(vec, n))
                torch_ms.append(round(ms, 4))
                if ms < best_ms:
                    best, best_ms, best_src = vec, ms, "torch"
                    chosen = {nm: [] for nm in names}
            del tv
        keep = best
        for v in keep.values():
            v.zero_()
        th_ids, mom_ids = chosen[names[it]], chosen[names[im]]
        nk = len(ch.views)
    finally:
        ch.release()
    pair_ms = sorted(times.values()) or [float("nan")]
    info = {"allocator": "torch" if best_src == "torch" else "vmm", "search": bool(search), "chunk_mb": cb >> 20,
            "chunks_per_vector": per, "chunks_allocated": nk,
            "pairs_timed": len(times), "pair_ms_min": round(pair_ms[0], 4),
            "pair_ms_median": round(pair_ms[len(pair_ms) // 2], 4),
            "pair_ms_max": round(pair_ms[-1], 4),
            "seconds": round(time.perf_counter() - t_start, 3),
            "default_ms": ms_d, "chosen_ms": round(best_ms, 4),
            "untuned_torch_ms": torch_ms[0] if torch_ms else None,
            "composites_ms": comp_ms, "torch_ms": torch_ms,
            "kept": best_src if best_src == "torch" else
            ("default" if chosen is cands[0] else "search"),
            "theta_chunks": th_ids, "mom_chunks": mom_ids}
    return keep, info
