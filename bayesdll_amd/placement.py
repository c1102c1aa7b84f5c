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
  3. if the pair times show no clearly fast pair (the pool sits in one
     physical group), allocate more chunks, `spare` at a time, and time each
     new one against chunk 0 only, until a group FAST_REF faster than chunk
     0's shows or the pool holds MAX_CHUNKS / the budget;
  4. candidate assignments: the allocation order, up to COMPOSITES
     greedy ones (seeded by each of the fastest pairs, completed with the
     fastest disjoint pairs; theta / momentum from the pairs, the other roles
     from the remaining chunks in allocation order) and up to COMPOSITES from
     the times against chunk 0 (its group for one role, the fastest group for
     the other: ref_candidates); each is mapped and timed
     at FULL size — chunk-pair times only rank the seeds; and, competing
     with them, the roles plus TORCH_EXTRA more vectors allocated plainly by
     torch, with up to TORCH_PAIRINGS (theta, mom) pairings among them (on
     some boxes hipMalloc'd memory pairs faster than any chunk composite).
     The fastest is kept; the per-chunk views are unmapped and every handle
     released (unchosen chunks return to the driver at once — nothing is
     parked in torch's cache).

Results never depend on placement (the kernels read the same values from any
address).  The mapped ranges are exposed to torch through
__cuda_array_interface__.

Virtual ranges are never handed to a second set of chunks: on this stack a
virtual address that has once been mapped keeps translating to its FIRST
physical backing after hipMemUnmap, whatever the synchronisation, the unmap
granularity, or whether the range was freed and re-reserved or kept and
re-mapped (tools/vmm_alias_repro.cpp, profiles/round3/vmm/: every scenario
that maps other chunks at a used address writes the OLD chunks; only a
never-used address is correct).  So an unmapped range stays reserved for the
life of the process (bdl_vmm_unmap), and to keep that address space from
growing with every chain state, the kept vectors of a placement are a
PlacedSet: when the last tensor of the set dies the set is PARKED — still
mapped, physical memory kept, like a block in torch's caching allocator — and
the next placement with the same key (device, size, roles, method) takes it
back as is: same chunks, same addresses, already searched.  Parked sets of
other keys are unmapped when a new search starts (their memory is then
needed); `release_pool()` unmaps all of them.  A range that is not part of a
set (candidates that lost, per-chunk views) is unmapped when its last tensor
goes — after a device synchronisation, and never inside a HIP-graph capture
(it is then queued and unmapped at the next release point)."""
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
# when the first pool shows no fast pair, chunks are added `spare` at a time and
# each new one is timed against chunk 0 only, until one group is this much
# faster than chunk 0's own (the best of the three pairing levels, DESIGN.md §4,
# — one process on one box found a single group over all of 62 chunks, 36 GB,
# profiles/round3/aux/placement_escalation/box10.jsonl, so the cap is the
# budget (a quarter of the free memory) more than MAX_CHUNKS —
# not the middle one: at chunk size the best level times 5-7 % below chunk 0's
# group, the middle one ~3.5 %, profiles/round3/aux/chunk_matrix/) or the pool
# holds MAX_CHUNKS / the budget
FAST_REF = 0.95
MAX_CHUNKS = int(os.environ.get("BDL_PLACEMENT_MAX_CHUNKS", "128"))
# > 1: the fastest RETIME candidates (chunk composites or plain pairings) are
# timed twice more, interleaved, and the best mean wins (A/B knob)
RETIME = int(os.environ.get("BDL_PLACEMENT_RETIME", "0"))
COMPOSITES = 6           # full-size candidate assignments timed besides allocation order
# plain torch allocations competing with the chunk composites: TORCH_VECTORS
# of them (the roles + extras; BDL_PLACEMENT_TORCH overrides), every unordered
# pair tried as (theta, mom), up to TORCH_PAIRINGS — consecutive allocations
# often sit in one physical group, and a few more of them reach the next;
# negative: no torch competitors (chunk composites only)
TORCH_EXTRA = int(os.environ.get("BDL_PLACEMENT_TORCH", "2"))
TORCH_PAIRINGS = 10

# parked PlacedSets per key, and the bytes they hold (BDL_PLACEMENT_POOL_GB caps
# them per process; 0 disables parking)
POOL_MAX_BYTES = int(float(os.environ.get("BDL_PLACEMENT_POOL_GB", "64")) * (1 << 30))
_POOL = {}
_POOL_BYTES = [0]
_VA_RESERVED = [0]  # bytes of virtual address space this process reserved for mappings

_pending = []  # (device index, va, total bytes) whose unmap was deferred (graph capture)


def va_reserved_bytes():
    """Virtual address space reserved by this process's mappings so far (never
    returned: see the module docstring)."""
    return _VA_RESERVED[0]


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
    """Unmap every parked set (their physical memory returns to the driver;
    the virtual ranges stay reserved), except those of `keep_key`."""
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
    pool (or unmapped when parking is off / over the cap)."""

    def __init__(self, key, dev_index, info):
        self.key, self.dev_index, self.info = key, dev_index, info
        self.roles = {}  # role -> (va, total) of the live mappings
        self.back = {}   # role -> (va, total) of the mappings whose tensors died

    def adopt(self, role, mapping):
        mapping.owner, mapping.role = self, role
        self.roles[role] = (mapping.va, mapping.total)

    def nbytes(self):
        return sum(t for _, t in self.roles.values())

    def give_back(self, role, va, total):
        """Called from Mapping.__del__; True when the range was taken care of."""
        self.back[role] = (va, total)
        if len(self.back) < len(self.roles):
            return True  # others of the set still alive: stay mapped
        nb = self.nbytes()
        if self.key is not None and _POOL_BYTES[0] + nb <= POOL_MAX_BYTES:
            _POOL.setdefault(self.key, []).append(self)
            _POOL_BYTES[0] += nb
            return True
        for v, t in self.back.values():
            _unmap_or_defer(self.dev_index, v, t)
        return True


def take_parked(key, n):
    """A parked set for `key`, re-exposed as fresh tensors over the same
    mappings (no map call), or None."""
    sets = _POOL.get(key)
    if not sets:
        return None
    old = sets.pop()
    if not sets:
        del _POOL[key]
    _POOL_BYTES[0] -= old.nbytes()
    with torch.cuda.device(old.dev_index):
        torch.cuda.synchronize()  # work on the dead tensors is finished
    ps = PlacedSet(key, old.dev_index, old.info)
    vecs = {}
    for role, (va, total) in old.back.items():
        m = Mapping(old.dev_index, None, None, n, adopt=(va, total))
        ps.adopt(role, m)
        vecs[role] = m.tensor()
    return vecs, ps


class Mapping:
    """One contiguous virtual range mapped from physical chunks (bdl_vmm_map),
    seen by torch as a flat fp32 tensor.  Torch's tensor keeps this object
    alive (from_blob with a reference to it); when it goes, the range is
    unmapped."""

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
            _VA_RESERVED[0] += self.total
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
            owner = self.owner
            if owner is not None and owner.give_back(self.role, va, self.total):
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


def _has_fast_pair(times):
    t = sorted(times)
    return t[0] < FAST_PAIR * t[len(t) // 2]


def _fast_pairs_found(times, per):
    """The first pool's stop rule: `per` DISJOINT (theta, mom) chunk pairs each
    FAST_PAIR below the median pair — what a composite needs.  One fast pair
    is not enough when per > 1: with a single chunk of the other group in the
    pool every fast pair shares it, and the best composite pairs one fast and
    one slow chunk (~1.0 ms where two fast pairs give ~0.96)."""
    if not times:
        return False
    vals = sorted(times.values())
    cut = FAST_PAIR * vals[len(vals) // 2]
    used, got = set(), 0
    for (i, j) in sorted(times, key=times.get):
        if times[(i, j)] >= cut:
            break
        if i in used or j in used:
            continue
        used.update((i, j))
        got += 1
        if got == per:
            return True
    return False


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


# which chunk pairs the search times: "all" ordered pairs (K (K - 1)
# timings), or "ref" — every chunk as mom against chunk 0 as theta (K - 1
# timings), the pairing relation being one of physical groups:
# chunks slow against chunk 0 share its group and go with it, the fastest
# against it take the other role (BDL_PLACEMENT_PAIRS overrides)
PAIRS = os.environ.get("BDL_PLACEMENT_PAIRS", "all")


def _ref_split(times0, per):
    """times0 {j: ms of (theta = chunk 0, mom = chunk j)}: (slow, fast) chunk
    lists — slow: above the midpoint of the fastest and slowest time, slowest
    first (chunk 0's own group); fast: the rest, fastest first — or None when
    the times show no two groups (spread under FAST_PAIR) or too few of
    either (slow >= per - 1, fast >= per)."""
    if not times0:
        return None
    lo, hi = min(times0.values()), max(times0.values())
    if not lo < FAST_PAIR * hi:
        return None
    mid = 0.5 * (lo + hi)
    slow = sorted((j for j, t in times0.items() if t > mid), key=lambda j: -times0[j])
    fast = sorted((j for j, t in times0.items() if t <= mid), key=lambda j: times0[j])
    if len(slow) < per - 1 or len(fast) < per:
        return None
    return slow, fast


def with_grad(assign, rank, names, per, nchunks):
    """`assign` (chunk ids per role) with the gradient on the best-ranked
    `per` chunks of `rank` that theta / mom do not use, the other roles
    re-filled from the remaining chunks in allocation order."""
    used = set(assign["theta"]) | set(assign["mom"])
    grad = [k for k in rank if k not in used][:per]
    rest = [k for k in range(nchunks) if k not in used and k not in grad]
    out, r = {}, 0
    for nm in names:
        if nm in ("theta", "mom"):
            out[nm] = list(assign[nm])
        elif nm == "grad":
            out[nm] = grad
        else:
            out[nm] = rest[r * per:(r + 1) * per]
            r += 1
    return out


def _ref_found(times0, per):
    """The escalation's stop rule: a split (_ref_split) whose `per` fastest
    chunks are all FAST_REF faster than chunk 0's group (the median of its
    slow times; the slowest time when the group is chunk 0 alone)."""
    split = _ref_split(times0, per)
    if split is None:
        return False
    slow, fast = split
    ref = sorted(times0[j] for j in slow)[len(slow) // 2] if slow else max(times0.values())
    # the per-th fastest too: a midpoint split with one truly fast chunk can
    # count a slow-group straggler as the second (seen on a box: 0.4819 and
    # 0.5023 against a group at 0.503-0.524 ms)
    return times0[fast[per - 1]] < FAST_REF * ref


def ref_candidates(times0, nchunks, names, per, limit=COMPOSITES):
    """Chunk ids per role for the full-size candidates of the "ref" search:
    the allocation order first, then up to `limit` assignments with theta =
    chunk 0 plus the per - 1 next-slowest chunks against it (its group) and
    mom = per chunks of the fast group — windows sliding along both rankings —
    and the same with theta / mom swapped; the other roles take the remaining
    chunks in allocation order.  No chunk serves two roles."""
    it, im = names.index("theta"), names.index("mom")

    def assign(th, mo):
        used = set(th) | set(mo)
        rest = [k for k in range(nchunks) if k not in used]
        out, r = {}, 0
        for q, nm in enumerate(names):
            if q == it:
                out[nm] = list(th)
            elif q == im:
                out[nm] = list(mo)
            else:
                out[nm] = rest[r * per:(r + 1) * per]
                r += 1
        return out

    cands = [{nm: list(range(q * per, (q + 1) * per)) for q, nm in enumerate(names)}]
    split = _ref_split(times0, per)
    if split is None:
        return cands
    slow, fast = split
    w = 0
    while len(cands) <= limit:
        th = [0] + slow[w:w + per - 1]
        mo = fast[w:w + per]
        if len(th) < per or len(mo) < per:
            break
        for a, b in ((th, mo), (mo, th)):
            c = assign(a, b)
            if len(cands) <= limit and c not in cands and \
                    all(len(v) == per for v in c.values()):
                cands.append(c)
        w += 1
    return cands


def place(n, device, names, launcher, time_launch, budget_bytes, spare=None, search=True,
          with_torch=True, pool_key=None, pairs=None):
    """Allocate `names` (fp32, n elements each, zeroed) from physical chunks,
    theta / mom paired fast.  `launcher(roles: {name: tensor}, n)` returns a
    zero-argument launch of the sampler's kernel; `time_launch(launch)` its
    median ms.  search=False: chunks mapped in allocation order, no pair
    timing.  `pairs`: "all" or "ref" (PAIRS).  `pool_key`: the kept vectors
    form a PlacedSet parked under this key when they die, and a set parked
    under it is reused instead of a new search.  Returns ({name: tensor}, info)."""
    import time
    t_start = time.perf_counter()
    dev_index = torch.device(device).index
    if dev_index is None:
        dev_index = torch.cuda.current_device()
    key = None if pool_key is None else (dev_index, int(n), tuple(names), search, pool_key)
    got = take_parked(key, n) if key is not None else None
    if got is not None:
        vecs, ps = got
        for v in vecs.values():
            v.zero_()
        info = dict(ps.info, reused=True, seconds=round(time.perf_counter() - t_start, 3),
                    search_seconds=ps.info["seconds"], va_reserved_gb=round(_VA_RESERVED[0] / 2**30, 1))
        return vecs, info
    release_pool()  # parked sets of other keys: their memory is needed now
    per, cb = chunk_geometry(n)
    nchunk = cb // 4
    nroles = len(names)
    it, im = names.index("theta"), names.index("mom")
    if spare is None:
        spare = int(os.environ.get("BDL_PLACEMENT_SPARE", "0")) or 2 * per
    spare = spare if search else 0
    # footprint up front: the chunks and the torch competitors are
    # alive together; drop the competition, then the spares, if over budget
    if TORCH_EXTRA < 0 or (nroles * per + spare) * cb + (nroles + TORCH_EXTRA) * 4 * n > budget_bytes:
        with_torch = False
    if (nroles * per + spare) * cb > budget_bytes:
        spare = 0
    ch = _Chunks(dev_index, cb)
    try:
        ch.add(nroles * per + spare)

        # a placed gradient ("grad" among the roles) is left out of the pair
        # timings (the launcher supplies its own) and chosen after them
        grad_role = "grad" in names

        def roles_for(i, j, g=None):
            rest = [k for k in range(len(ch.views)) if k not in (i, j, g)]
            out, r = {}, 0
            for q, nm in enumerate(names):
                if q == it:
                    out[nm] = ch.views[i]
                elif q == im:
                    out[nm] = ch.views[j]
                elif nm == "grad":
                    if g is not None:
                        out[nm] = ch.views[g]
                else:
                    out[nm] = ch.views[rest[r]]
                    r += 1
            return out

        pairs = pairs or PAIRS
        if pairs not in ("all", "ref"):
            raise ValueError(f"BDL_PLACEMENT_PAIRS must be all or ref, got {pairs!r}")
        times, rounds = {}, 0

        def times0():
            return {j: t for (i, j), t in times.items() if i == 0}
        if search:
            # the first pool: every ordered pair ("all") or every chunk against
            # chunk 0 — among the first 2 x per + spare chunks only (theta /
            # mom's share; the pool's other chunks hold the other roles while
            # pairs are timed: Adam's seven roles would make it 306 pairs)
            p0 = min(len(ch.views), 2 * per + spare)
            for i in range(p0 if pairs == "all" else 1):
                for j in range(p0):
                    if i != j:
                        times[(i, j)] = time_launch(launcher(roles_for(i, j), nchunk))
            found = _fast_pairs_found(times, per) if pairs == "all" else _ref_found(times0(), per)
            # no fast pair yet: the pool's chunks sit in one physical group (on
            # some boxes a group spans more than 16 chunks of 586 MB: a 16-chunk
            # all-pairs search kept 1.03-1.04 ms where 28 chunks reached 0.96,
            # profiles/round3/aux/spare_ab.jsonl) — add chunks and time each new
            # one against chunk 0 only until another group shows
            while not found and spare > 0 and len(ch.views) + spare <= MAX_CHUNKS and \
                    (len(ch.views) + spare) * cb <= budget_bytes:
                k0 = len(ch.views)
                ch.add(spare)
                rounds += 1
                for j in range(k0, len(ch.views)):
                    times[(0, j)] = time_launch(launcher(roles_for(0, j), nchunk))
                found = _ref_found(times0(), per)

        def composite(assign):
            maps = {nm: Mapping(dev_index, [ch.handles[k] for k in ids], cb, n)
                    for nm, ids in assign.items()}
            return maps, {nm: m.tensor() for nm, m in maps.items()}

        cands = candidate_assignments(times, len(ch.views), names, per) if pairs == "all" else []
        for c in ref_candidates(times0(), len(ch.views), names, per):
            if c not in cands:
                cands.append(c)
        grad_ms = {}
        if search and grad_role and times:
            # the gradient's chunks: every other chunk timed as the gradient of
            # the fastest (theta, mom) pair — on some boxes the read-only
            # stream's memory moves the sweep by ~2 % (tools/grad_spread.py)
            bi, bj = min(times, key=times.get)
            for g in range(len(ch.views)):
                if g not in (bi, bj):
                    grad_ms[g] = time_launch(launcher(roles_for(bi, bj, g), nchunk))
            rank = sorted(grad_ms, key=grad_ms.get)
            cands = cands[:1] + [with_grad(c, rank, names, per, len(ch.views)) for c in cands[1:]]
            uniq = []
            for c in cands:
                if c not in uniq:
                    uniq.append(c)
            cands = uniq
        # the fastest RETIME candidates stay alive (mapped) for a second timing
        # round; the others are dropped (unmapped) as soon as they lose
        top = []  # [ms, source, vectors, mappings, chunk ids per role]

        def consider(ms, src, vec, maps, assign):
            top.append([ms, src, vec, maps, assign])
            top.sort(key=lambda e: e[0])
            del top[max(1, RETIME):]

        comp_ms = []
        for c in cands:
            maps, vec = composite(c)
            for v in vec.values():
                v.zero_()
            ms = time_launch(launcher(vec, n))
            comp_ms.append(round(ms, 4))
            consider(ms, "chunks", vec, maps, c)
            del vec, maps
        ms_d = comp_ms[0]
        # torch's own allocations compete too (on some boxes hipMalloc'd
        # memory pairs faster than any chunk composite): the roles' vectors
        # allocated plainly, with every (theta, mom) pairing among them
        torch_ms = []
        if search and with_torch:
            tv = [torch.zeros(n, dtype=torch.float32, device=device)
                  for _ in range(len(names) + max(0, TORCH_EXTRA))]
            tpairs = [(it, im)] + [p for p in itertools.combinations(range(len(tv)), 2)
                                   if set(p) != {it, im}]
            for i, j in tpairs[:TORCH_PAIRINGS]:
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
                consider(ms, "torch", vec, None, {nm: [] for nm in names})
            del tv
        retimed = None
        if RETIME > 1 and len(top) > 1:
            # second round over the finalists, interleaved: the first round's
            # minimum is biased low (the fastest of ~13-23 noisy timings)
            for _ in range(2):
                for e in top:
                    e.append(time_launch(launcher(e[2], n)))
            for e in top:
                e[0] = sum(e[5:] + [e[0]]) / (len(e) - 4)
            retimed = [round(e[0], 4) for e in top]
            top.sort(key=lambda e: e[0])
        best_ms, best_src, best, best_maps, chosen = top[0][:5]
        del top
        keep = best
        for v in keep.values():
            v.zero_()
        th_ids, mom_ids = chosen[names[it]], chosen[names[im]]
        nk = len(ch.views)
    finally:
        ch.release()
    pair_ms = sorted(times.values()) or [float("nan")]
    info = {"allocator": "torch" if best_src == "torch" else "vmm", "search": bool(search), "chunk_mb": cb >> 20,
            "chunks_per_vector": per, "chunks_allocated": nk, "pairs": pairs if search else None,
            "escalation_rounds": rounds, "grad_timed": len(grad_ms),
            "grad_chunks": chosen.get("grad") if grad_role else None,
            "ref_ms": [round(t, 4) for _, t in sorted(times0().items())],
            "pairs_timed": len(times), "pair_ms_min": round(pair_ms[0], 4),
            "pair_ms_median": round(pair_ms[len(pair_ms) // 2], 4),
            "pair_ms_max": round(pair_ms[-1], 4),
            "seconds": round(time.perf_counter() - t_start, 3),
            "default_ms": ms_d, "chosen_ms": round(best_ms, 4), "retimed_ms": retimed,
            "untuned_torch_ms": torch_ms[0] if torch_ms else None,
            "composites_ms": comp_ms, "torch_ms": torch_ms,
            "kept": best_src if best_src == "torch" else
            ("default" if chosen == cands[0] else "search"),
            "theta_chunks": th_ids, "mom_chunks": mom_ids, "reused": False,
            "va_reserved_gb": round(_VA_RESERVED[0] / 2**30, 1)}
    if best_maps is not None and key is not None:
        ps = PlacedSet(key, dev_index, info)
        for nm, m in best_maps.items():
            ps.adopt(nm, m)
    del best_maps
    return keep, info


ONE_COMPOSITES = 3  # full-size composites timed by place_one besides allocation order


def one_candidates(pos_ms, per, limit=ONE_COMPOSITES):
    """Chunk lists for place_one's full-size composites from `pos_ms` (per
    lists: position p's ms for every chunk — position p of the vector is swept
    together with the inputs' p-th slice, so a chunk's time depends on where
    it sits): candidate w takes, position by position, the w-th fastest chunk
    not yet used; then the allocation order; no list twice."""
    nch = len(pos_ms[0])
    ranked = [sorted(range(nch), key=lambda i, p=p: pos_ms[p][i]) for p in range(per)]
    cands = []
    for w in range(limit):
        used, ids = set(), []
        for p in range(per):
            free = [c for c in ranked[p] if c not in used]
            if len(free) <= w:
                break
            ids.append(free[w])
            used.add(free[w])
        if len(ids) == per and ids not in cands:
            cands.append(ids)
    order = list(range(per))
    if order not in cands:
        cands.append(order)
    return cands


def _one_estimate(pos_ms, per):
    """Greedy estimate of the best composite from per-position chunk times
    (position by position, the fastest chunk not yet used)."""
    nch, used, est = len(pos_ms[0]), set(), 0.0
    for p in range(per):
        c = min((c for c in range(nch) if c not in used), key=lambda c: pos_ms[p][c])
        used.add(c)
        est += pos_ms[p][c]
    return est


ONE_SPREAD = 0.98  # place_one: two groups of chunks show as this much spread
# place_one's first pool (the draw's chunk-sized timings are cheap: ~1 ms a
# chunk) and its bar against the caller's best plain allocation: the per
# fastest chunks must sum below ONE_BEAT x beat_ms (a composite times 2-5 %
# above the sum of its chunk-sized sweeps, profiles/round3/final*/bench.log)
ONE_POOL = 16
ONE_BEAT = 0.96


def _one_found(chunk_ms, per):
    """place_one's stop rule: the chunk times split into two groups (fastest
    ONE_SPREAD below the slowest) with at least `per` chunks in the faster
    (at or below the midpoint)."""
    lo, hi = min(chunk_ms), max(chunk_ms)
    if not lo < ONE_SPREAD * hi:
        return False
    mid = 0.5 * (lo + hi)
    return sum(t <= mid for t in chunk_ms) >= per


def place_one(n, device, launcher, time_launch, budget_bytes, spare=None, pool_key=None,
              beat_ms=None):
    """One WRITTEN vector (n fp32 elements) from physical chunks, for a sweep
    whose other streams are fixed (the posterior draw: m1 / m2 given, out
    chosen; DESIGN.md §4 — it runs fastest with out in the physical group
    opposite to its reads, which only timing reveals).  `launcher(buf, off)`
    returns a zero-argument launch of the sweep writing `buf` with its inputs
    from element `off` on (buf.numel() <= n - off elements); `time_launch(launch)`
    its median ms.

      1. allocate max(per + spare, ONE_POOL) chunks (each also mapped alone);
      2. time the sweep into every chunk at every position p of the vector
         (chunk-sized: the reads are the inputs' p-th slices — the sweep's
         speed depends on the output's memory AND the inputs' at the same
         offset); while the times show no second group, or the best
         position-by-position estimate does not promise to beat `beat_ms`,
         allocate `spare` more (up to MAX_CHUNKS / the budget);
      3. map composites (one_candidates: position by position, the w-th
         fastest free chunk) and the allocation order, and time each at FULL
         size.

    The fastest composite is returned if it beats `beat_ms` (the caller's best
    plain allocation), else (None, info): the caller keeps its own buffer.
    `pool_key`: as for place() — the kept vector is parked when it dies, and
    the next call with the key takes it back without a search."""
    import time
    t_start = time.perf_counter()
    dev_index = torch.device(device).index
    if dev_index is None:
        dev_index = torch.cuda.current_device()
    key = None if pool_key is None else (dev_index, int(n), ("out",), True, pool_key)
    got = take_parked(key, n) if key is not None else None
    if got is not None:
        vecs, ps = got
        info = dict(ps.info, reused=True, seconds=round(time.perf_counter() - t_start, 3),
                    search_seconds=ps.info["seconds"], va_reserved_gb=round(_VA_RESERVED[0] / 2**30, 1))
        return vecs["out"], info
    release_pool()
    per, cb = chunk_geometry(n)
    k = min(cb // 4, n)  # elements the chunk-sized sweeps write (a 1-chunk vector's chunk is rounded up)
    spare = (2 * per if spare is None else spare)
    first = max(per + spare, min(ONE_POOL, MAX_CHUNKS))
    while first > per and first * cb > budget_bytes:
        first -= 1
    if first * cb > budget_bytes:
        return None, {"allocator": "torch", "kept": "torch", "skipped": "over budget"}
    ch = _Chunks(dev_index, cb)
    best, best_ms, best_map, comp_ms = None, None, None, []

    def enough(pos_ms):
        if beat_ms is None:
            return _one_found(pos_ms[0], per)
        return _one_estimate(pos_ms, per) < ONE_BEAT * beat_ms

    def time_chunks(views):
        # position p: the chunk-sized sweep over the inputs' p-th slice (the
        # last position's slice may be shorter than a chunk)
        return [[time_launch(launcher(v[:min(k, n - p * k)], p * k)) for v in views]
                for p in range(per)]
    try:
        ch.add(first)
        pos_ms = time_chunks(ch.views)
        # all chunks alike (one physical group), or none promising to beat the
        # plain allocation: add more, within MAX_CHUNKS / the budget
        while not enough(pos_ms) and spare > 0 and \
                len(ch.views) + spare <= MAX_CHUNKS and (len(ch.views) + spare) * cb <= budget_bytes:
            k1 = len(ch.views)
            ch.add(spare)
            for p, more in enumerate(time_chunks(ch.views[k1:])):
                pos_ms[p] += more
        chunk_ms = pos_ms[0]
        for ids in one_candidates(pos_ms, per):
            m = Mapping(dev_index, [ch.handles[i] for i in ids], cb, n)
            t = m.tensor()
            t.zero_()
            ms = time_launch(launcher(t, 0))
            comp_ms.append(round(ms, 4))
            if best_ms is None or ms < best_ms:
                best, best_ms, best_map, chosen = t, ms, m, ids
            del t, m
    finally:
        ch.release()
    won = beat_ms is None or best_ms < beat_ms
    info = {"allocator": "vmm" if won else "torch", "kept": "chunks" if won else "torch",
            "chunk_mb": cb >> 20, "chunks_per_vector": per, "chunks_allocated": len(chunk_ms),
            "chunk_ms": [round(t, 4) for t in chunk_ms],
            "chunk_ms_by_pos": [[round(t, 4) for t in row] for row in pos_ms],
            "composites_ms": comp_ms,
            "chosen_ms": round(best_ms, 4), "chunks": chosen if won else [],
            "beat_ms": None if beat_ms is None else round(beat_ms, 4), "reused": False,
            "seconds": round(time.perf_counter() - t_start, 3),
            "va_reserved_gb": round(_VA_RESERVED[0] / 2**30, 1)}
    if not won:
        return None, info
    if key is not None:
        PlacedSet(key, dev_index, info).adopt("out", best_map)
    del best_map
    return best, info
