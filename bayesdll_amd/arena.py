"""Gradient arena: the backward pass allocates from ONE device reservation.

The reference reads every parameter's gradient where autograd leaves it
(`p.grad`, methods/csghmc.py:741-778), and so does the fused update
("tensor" gradient mode: a per-tensor base-address table, flat.py).  Where
those ~300 tensors (ViT-L/32) sit is torch's caching allocator's choice:
~100 separately hipMalloc'd segments, and the sweep over them ran up to 1.8 %
behind the same sweep over views of one allocation on some boxes
(BENCH_r05.json `explore_tensor_grad`: 1.0561 ms vs `one_allocation`
1.0356 ms).

`GradArena` is a `torch.cuda.MemPool` whose segments are carved from one
reservation by the library's bump allocator (include/bdl_arena.h, through
`torch.cuda.memory.CUDAPluggableAllocator`).  `arena.routing()` sends every
allocation on the device to that pool while it is active — including the
autograd engine's device thread, which is where backward allocates (torch's
`use_mem_pool` routes only the calling thread, so it would miss them).  The
pool's caching allocator keeps the segments it carved; from the second step
on, the step's gradients come back at the same addresses (the gradient-table
cache in flat.py hits) and the arena is not called at all.

Measured (round 6, DESIGN.md §3, profiles/round6/grad_layout/): it does not
close the gap.  Over five same-process comparisons (five box acquisitions)
the explore sweep on arena gradients averaged 1.0526 ms against 1.0501 ms on
torch's default pool (flat gradient 1.034-1.039 ms); the same 296 tensors
copied into ONE fresh allocation at their flat offsets ran 0.993-1.004 of
flat, and other single-allocation layouts 0.998-1.020 — the spread is the
physical placement of each allocation, which no layout chosen from user
space fixes.
So the arena is opt-in: BDL_GRAD_ARENA=1 (values never depend on it).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os

import torch

from . import _lib as L

# first region: the gradients plus this much room for the backward's
# temporaries (activation gradients), which the pool also serves
ARENA_SLACK_BYTES = 256 << 20


def default_grad_arena():
    """BDL_GRAD_ARENA=1 turns the arena on (default: gradients from torch's
    default pool, as autograd leaves them)."""
    return os.environ.get("BDL_GRAD_ARENA", "0") not in ("", "0", "false", "False")


_ALLOCATOR = None


def _allocator():
    """One CUDAPluggableAllocator over the library's arena entry points.  Its
    C++ object must outlive every MemPool built on it (a pool keeps a raw
    pointer to it and calls it when it is destroyed, possibly during
    interpreter shutdown, after module globals are gone): it is created once
    and deliberately never released."""
    global _ALLOCATOR
    if _ALLOCATOR is None:
        L.lib()  # fail loudly (no CPU path) before torch dlopens the library
        a = torch.cuda.memory.CUDAPluggableAllocator(
            L.LIB_PATH, "bdl_arena_alloc", "bdl_arena_free")
        C.pythonapi.Py_IncRef(C.py_object(a))
        C.pythonapi.Py_IncRef(C.py_object(a.allocator()))
        _ALLOCATOR = a
    return _ALLOCATOR


def stats(device):
    """The library's arena statistics for `device` (bdl_arena_stats)."""
    idx = torch.device(device).index
    out = (C.c_int64 * 8)()
    L.check(L.lib().bdl_arena_stats(int(idx), out, 8), "bdl_arena_stats")
    keys = ("regions", "reserved", "carved", "live", "carvings", "grown", "base", "size")
    return dict(zip(keys, (int(v) for v in out)))


def contains(device, t):
    """Does tensor `t`'s storage lie in a live arena region of `device`?"""
    idx = torch.device(device).index
    return bool(L.lib().bdl_arena_contains(int(idx), C.c_void_p(t.data_ptr()),
                                           t.numel() * t.element_size()))


class GradArena:
    """A MemPool on `device` backed by one reservation of `nbytes` (+ slack)."""

    def __init__(self, device, nbytes):
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("bayesdll_amd: the gradient arena needs a HIP device")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.nbytes = int(nbytes) + ARENA_SLACK_BYTES
        L.check(L.lib().bdl_arena_reserve(dev.index, self.nbytes), "bdl_arena_reserve")
        self._allocator = _allocator()
        self.pool = torch.cuda.MemPool(self._allocator.allocator())
        self.active = False

    @contextlib.contextmanager
    def routing(self):
        """Every allocation on the device (any thread, any stream) goes to the
        arena's pool while the context is active: wrap `loss.backward()`."""
        if self.active:  # re-entrant: already routing
            yield
            return
        idx = self.device.index
        torch._C._cuda_beginAllocateToPool(idx, self.pool.id)
        self.active = True
        try:
            yield
        finally:
            self.active = False
            torch._C._cuda_endAllocateToPool(idx, self.pool.id)
            torch._C._cuda_releasePool(idx, self.pool.id)
