"""Physical-chunk placement of a chain's swept vectors (include/bdl_placement.h).

Why: the fused step rewrites two vectors in place — theta and the momentum /
SGD buffer — and on MI355X its HBM rate depends on which physical memory
those two land on: for ViT-L/32 the explore sweep runs ~0.96 ms when the pair
of physical regions is a "fast" pair and ~1.03-1.10 ms otherwise.  The
relation is a property of physical regions of several GB (moving a vector by
256 B ... 1 GB inside its allocation never changes it; interleaving theta and
the momentum in one allocation makes every pair slow, tools/layout_probe.hip),
invisible from user space, and torch's allocator hands out whatever comes
next.

Opt-in (BDL_PLACEMENT=search; the default, for the Runners and bench.py
alike, is torch's allocator: on the Runner path the search bought no
end-to-end time and cost 2.2x the transient HBM).  How — a
bounded search, once per chain state:

  1. create physical chunks (hipMemCreate, <= 1 GiB each, `per` per vector),
     each also mapped alone;
  2. time the method's production kernel with chunk 0 as theta and every
     other chunk as the momentum (chunk-sized sweeps): chunks slow against
     chunk 0 share its physical group, fast ones are in another — growing the
     pool 2 x per chunks at a time until a second group shows, up to
     MAX_CHUNKS chunks or SEARCH_SECONDS;
  3. full-size candidates: the allocation order, up to COMPOSITES assignments
     with theta from chunk 0's group and the momentum from the fast group (and
     swapped), and the roles allocated plainly by torch; each is mapped and
     timed at full size and the fastest kept.  Unchosen chunks go back to the
     driver at once.

Results never depend on placement (the kernels read the same values from any
address).  The mapped ranges are exposed to torch through
__cuda_array_interface__.  Their virtual addresses come from the library's
arena (bdl_vmm_map): one large reservation, bump-allocated, no address handed
out twice — on this stack an address mapped once keeps translating to its
first physical backing after hipMemUnmap (tools/vmm_alias_repro.cpp).

The kept vectors of a placement form a PlacedSet.  A chain state's set is
unmapped when its last tensor dies (the chain's parameters are views into
theta, so that is when the Runner, its network and its sampler are gone).
The autotuner's scratch state (kernels.autotune) is placed with the chain's
roles and its set is PARKED instead — still mapped, up to
BDL_PLACEMENT_POOL_GB (default POOL_GB_DEFAULT) per process — so the chain
state that follows takes it back without a second search.  A search for
another key and `release_pool()` unmap parked sets.

Knobs: BDL_PLACEMENT = 0 (torch's allocator, the default) | search | order
(chunks in allocation order, no timing); BDL_PLACEMENT_POOL_GB."""
from __future__ import annotations

import ctypes as C
import math
import os
import time

import torch

from . import _lib as L

CHUNK_TARGET = 1 << 30   # vectors of up to 1 GiB are one chunk
ALIGN = 2 << 20          # chunk sizes are multiples of 2 MiB (large-page mappings)
MAX_CHUNKS = 16          # the search's chunk pool, at most
SEARCH_SECONDS = 0.3     # no new chunk-pair timing or chunks past this
SPLIT = 0.97             # chunk times show two groups when the fastest is this much below the slowest
COMPOSITES = 4           # full-size group assignments timed besides the allocation order
POOL_GB_DEFAULT = 16

POOL_MAX_BYTES = int(float(os.environ.get("BDL_PLACEMENT_POOL_GB", str(POOL_GB_DEFAULT)))
                     * (1 << 30))
_POOL = {}
_POOL_BYTES = [0]
_pending = []  # (device index, va, total bytes) whose unmap was deferred (graph capture)


def mode():
    m = os.environ.get("BDL_PLACEMENT", "0")
    if m not in ("search", "order", "0"):
        raise ValueError(f"BDL_PLACEMENT must be search, order or 0, got {m!r}")
    return m


def va_reserved_bytes():
    """(address space the library's arena reserved, sub-ranges handed out)."""
    r, m = C.c_uint64(), C.c_uint64()
    L.check(L.lib().bdl_vmm_arena_info(C.byref(r), C.byref(m)), "bdl_vmm_arena_info")
    return int(r.value), int(m.value)


def pooled_bytes():
    return _POOL_BYTES[0]


def _unmap_now(dev_index, va, total):
    with torch.cuda.device(dev_index):
        torch.cuda.synchronize()
    L.check(L.lib().bdl_vmm_unmap(C.c_void_p(va), total), "bdl_vmm_unmap")


def _unmap_or_defer(dev_index, va, total):
    if torch.cuda.is_current_stream_capturing():
        _pending.append((dev_index, va, total))
    else:
        _unmap_now(dev_index, va, total)


def release_pending():
    """Unmap ranges whose last tensor died during a graph capture."""
    if not _pending or torch.cuda.is_current_stream_capturing():
        return
    while _pending:
        _unmap_now(*_pending.pop())


def release_pool(keep_key=None):
    """Unmap every parked set except those of `keep_key` (their physical
    memory returns to the driver)."""
    for key in list(_POOL):
        if key == keep_key:
            continue
        for ps in _POOL.pop(key):
            _POOL_BYTES[0] -= ps.nbytes()
            for va, total in ps.back.values():
                _unmap_or_defer(ps.dev_index, va, total)


class PlacedSet:
    """The kept vectors of one placement (role -> mapped range).  While any of
    them lives, all stay mapped; when the last dies the set is parked in the
    pool (`park`, within the cap) or unmapped."""

    def __init__(self, key, dev_index, info, park=False):
        self.key, self.dev_index, self.info, self.park = key, dev_index, info, park
        self.roles = {}  # role -> (va, total) of the live mappings
        self.back = {}   # role -> (va, total) of the mappings whose tensors died

    def adopt(self, role, mapping):
        mapping.owner, mapping.role = self, role
        self.roles[role] = (mapping.va, mapping.total)

    def nbytes(self):
        return sum(t for _, t in self.roles.values())

    def give_back(self, role, va, total):
        """Called from Mapping.__del__."""
        self.back[role] = (va, total)
        if len(self.back) < len(self.roles):
            return  # others of the set still alive: stay mapped
        nb = self.nbytes()
        if self.park and self.key is not None and _POOL_BYTES[0] + nb <= POOL_MAX_BYTES:
            _POOL.setdefault(self.key, []).append(self)
            _POOL_BYTES[0] += nb
            return
        for v, t in self.back.values():
            _unmap_or_defer(self.dev_index, v, t)


def take_parked(key, n, park=False):
    """A parked set for `key`, re-exposed as fresh tensors over the same
    mappings (no map call; parked again when they die if `park`), or None."""
    sets = _POOL.get(key)
    if not sets:
        return None
    old = sets.pop()
    if not sets:
        del _POOL[key]
    _POOL_BYTES[0] -= old.nbytes()
    with torch.cuda.device(old.dev_index):
        torch.cuda.synchronize()  # work on the dead tensors is finished
    ps = PlacedSet(key, old.dev_index, old.info, park)
    vecs = {}
    for role, (va, total) in old.back.items():
        m = Mapping(old.dev_index, None, None, n, adopt=(va, total))
        ps.adopt(role, m)
        vecs[role] = m.tensor()
    return vecs, ps


class Mapping:
    """One contiguous virtual range mapped from physical chunks (bdl_vmm_map),
    seen by torch as a flat fp32 tensor.  Torch's tensor keeps this object
    alive (it holds the __cuda_array_interface__ owner); when it goes, the
    range is unmapped or its set parked."""

    def __init__(self, dev_index, handles, chunk_bytes, nelem, adopt=None):
        self.owner, self.role = None, None
        self.dev_index = dev_index
        if adopt is None:
            arr = (C.c_uint64 * len(handles))(*handles)
            va = C.c_void_p()
            L.check(L.lib().bdl_vmm_map(dev_index, arr, len(handles), chunk_bytes, C.byref(va)),
                    "bdl_vmm_map")
            self.va = int(va.value)
            self.total = len(handles) * int(chunk_bytes)
        else:  # a parked set's range, still mapped
            self.va, self.total = int(adopt[0]), int(adopt[1])
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
            if self.owner is not None:
                self.owner.give_back(self.role, va, self.total)
                return
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


def split_groups(times0, per):
    """times0 {j: ms of (theta = chunk 0, mom = chunk j)}: (slow, fast) chunk
    lists — slow: above the midpoint of the fastest and slowest time, slowest
    first (chunk 0's own group); fast: the rest, fastest first — or None when
    the times show no two groups (spread under SPLIT) or too few of either
    (slow >= per - 1, fast >= per)."""
    if not times0:
        return None
    lo, hi = min(times0.values()), max(times0.values())
    if not lo < SPLIT * hi:
        return None
    mid = 0.5 * (lo + hi)
    slow = sorted((j for j, t in times0.items() if t > mid), key=lambda j: -times0[j])
    fast = sorted((j for j, t in times0.items() if t <= mid), key=lambda j: times0[j])
    if len(slow) < per - 1 or len(fast) < per:
        return None
    return slow, fast


def assignments(times0, nchunks, names, per, limit=COMPOSITES):
    """Chunk ids per role for the full-size candidates: the allocation order
    first, then up to `limit` assignments with theta = chunk 0 plus the
    per - 1 next-slowest chunks against it (its group) and the momentum = per
    chunks of the fast group — windows sliding along both rankings — and the
    same with theta / momentum swapped; the other roles take the remaining
    chunks in allocation order.  No chunk serves two roles."""
    it, im = names.index("theta"), names.index("mom")

    def assign(th, mo):
        rest = [k for k in range(nchunks) if k not in set(th) | set(mo)]
        out, r = {}, 0
        for q, nm in enumerate(names):
            if q in (it, im):
                out[nm] = list(th if q == it else mo)
            else:
                out[nm] = rest[r * per:(r + 1) * per]
                r += 1
        return out

    cands = [{nm: list(range(q * per, (q + 1) * per)) for q, nm in enumerate(names)}]
    split = split_groups(times0, per)
    if split is None:
        return cands
    slow, fast = split
    for w in range(limit):
        th, mo = [0] + slow[w:w + per - 1], fast[w:w + per]
        if len(th) < per or len(mo) < per:
            break
        for a, b in ((th, mo), (mo, th)):
            c = assign(a, b)
            if len(cands) <= limit and c not in cands and all(len(v) == per for v in c.values()):
                cands.append(c)
    return cands


def place(n, device, names, launcher, time_launch, budget_bytes, search=True, pool_key=None,
          park=False, with_torch=True):
    """Allocate `names` (fp32, n elements each, zeroed) from physical chunks,
    theta / mom paired fast (the module docstring's bounded search).
    `launcher(roles: {name: tensor}, n)` returns a zero-argument launch of the
    sampler's kernel; `time_launch(launch)` its median ms.  search=False:
    chunks mapped in allocation order, no timing.  `pool_key`: a set parked
    under this key is reused instead of a new search, and with `park` the kept
    vectors are parked under it when they die.  with_torch=False: no plain
    torch candidate.  Raises RuntimeError
    when the chunks do not fit `budget_bytes` or chunk mappings are
    unavailable (the caller falls back to torch's allocator).
    Returns ({name: tensor}, info)."""
    t_start = time.perf_counter()
    deadline = t_start + SEARCH_SECONDS
    dev_index = torch.device(device).index
    if dev_index is None:
        dev_index = torch.cuda.current_device()
    key = None if pool_key is None else (dev_index, int(n), tuple(names), search, pool_key)
    got = take_parked(key, n, park) if key is not None else None
    if got is not None:
        vecs, ps = got
        for v in vecs.values():
            v.zero_()
        return vecs, dict(ps.info, reused=True, seconds=round(time.perf_counter() - t_start, 3),
                          search_seconds=ps.info["seconds"])
    release_pool()  # parked sets of other keys: their memory is needed now
    per, cb = chunk_geometry(n)
    nchunk = cb // 4
    need = len(names) * per
    cap = min(MAX_CHUNKS, budget_bytes // cb) if search else need
    if cap < need:
        raise RuntimeError(f"placement: {need} chunks of {cb >> 20} MiB exceed the budget "
                           f"({budget_bytes >> 20} MiB)")
    it, im = names.index("theta"), names.index("mom")
    ch = _Chunks(dev_index, cb)
    times0, peak = {}, 0
    try:
        ch.add(min(cap, need + (2 * per if search else 0)))

        def roles_for(j):
            rest = [k for k in range(len(ch.views)) if k not in (0, j)]
            out, r = {}, 0
            for q, nm in enumerate(names):
                if q in (it, im):
                    out[nm] = ch.views[0 if q == it else j]
                else:
                    out[nm] = ch.views[rest[r]]
                    r += 1
            return out

        if search:
            # every chunk as the momentum against chunk 0 as theta; more chunks
            # while the pool shows one group only
            while True:
                for j in range(1, len(ch.views)):
                    if j not in times0:
                        times0[j] = time_launch(launcher(roles_for(j), nchunk))
                if split_groups(times0, per) is not None or len(ch.views) >= cap or \
                        time.perf_counter() > deadline:
                    break
                ch.add(min(2 * per, cap - len(ch.views)))
        cands = assignments(times0, len(ch.views), names, per)
        best = None  # (ms, source, tensors, mappings, assignment)
        comp_ms, torch_ms = [], None
        for q, c in enumerate(cands):
            if q > 1 and time.perf_counter() > deadline:
                break  # past the budget: the allocation order and the first group pairing only
            maps = {nm: Mapping(dev_index, [ch.handles[k] for k in ids], cb, n)
                    for nm, ids in c.items()}
            vec = {nm: m.tensor().zero_() for nm, m in maps.items()}
            ms = time_launch(launcher(vec, n)) if search else 0.0
            comp_ms.append(round(ms, 4))
            if best is None or ms < best[0]:
                best = (ms, "chunks", vec, maps, c)
            del vec, maps
        peak = len(ch.views) * cb  # composites map the same chunks: no more physical memory
        if search and with_torch and peak + 4 * n * len(names) <= budget_bytes:
            # the roles allocated plainly by torch compete (BDL_PLACEMENT=0's vectors)
            tv = {nm: torch.zeros(n, dtype=torch.float32, device=device) for nm in names}
            torch_ms = round(time_launch(launcher(tv, n)), 4)
            peak += 4 * n * len(names)
            if torch_ms < best[0]:
                best = (torch_ms, "torch", tv, None, {nm: [] for nm in names})
            del tv
        nk = len(ch.views)
    finally:
        ch.release()
    best_ms, src, keep, maps, chosen = best
    for v in keep.values():
        v.zero_()
    split = split_groups(times0, per)
    info = {"allocator": "torch" if src == "torch" else "vmm", "search": bool(search),
            "kept": "torch" if src == "torch" else
            ("default" if chosen == cands[0] else "search"),
            "chunk_mb": cb >> 20, "chunks_per_vector": per, "chunks_allocated": nk,
            "pairs_timed": len(times0), "ref_ms": [round(times0[j], 4) for j in sorted(times0)],
            "groups": None if split is None else {"slow": split[0], "fast": split[1]},
            "default_ms": comp_ms[0] if search else None,
            "chosen_ms": round(best_ms, 4) if search else None,
            "composites_ms": comp_ms if search else [], "untuned_torch_ms": torch_ms,
            "theta_chunks": chosen[names[it]], "mom_chunks": chosen[names[im]],
            "transient_gb": round(peak / 2**30, 2), "reused": False,
            "seconds": round(time.perf_counter() - t_start, 3)}
    if maps is not None and key is not None:
        ps = PlacedSet(key, dev_index, info, park)
        for nm, m in maps.items():
            ps.adopt(nm, m)
    del maps
    return keep, info
