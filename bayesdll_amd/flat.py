"""Flat, HBM-resident state of one SG-MCMC chain.

The reference keeps parameters, gradients, momenta and posterior moments as
hundreds of separate tensors (one per named parameter) and walks them in a
Python loop (methods/csghmc.py:747-778).  Here every per-chain quantity is ONE
contiguous fp32 vector in the canonical `parameters_to_vector` order
(methods/csghmc.py:328, methods/sgld.py:98), so the fused kernel sweeps each
of them exactly once per step:

    theta  — the network's parameters; every nn.Parameter's .data is rebound
             to a view into it, so the network computes with it directly.
    grad   — gradients.  Default ("tensor" mode): NOT a flat vector — .grad is
             set to None before backward, autograd's AccumulateGrad steals each
             fresh gradient tensor (as after the reference's net.zero_grad()),
             and the kernel reads every tensor's gradient where autograd left it
             through a per-run base-address table (bdl_step_args.grad_base):
             no zero-fill, no accumulation pass, no copy.  "flat" mode
             (BDL_GRAD_MODE=flat, and the segment-only states of the bench and
             kernel tests): every .grad is a view into one flat vector that
             autograd accumulates into (zeroed before backward).
    mom    — cSGHMC/SGHMC momentum v, or the SGD momentum buffer (sgld/csgld).
    prior  — theta0 = net0's parameters (sgld/sghmc prior mean).
    noise  — only in "torch" noise mode: per-tensor torch normal_ draws.

The segment table (offset, numel, attributes per named parameter) is reduced
once by the library's bdl_build_runs into a handful of runs (maximal ranges
of equal attributes: lr group from `readout_name in pname`, prior on/off from
`'bias' in pname and bias == 'uninformative'`, methods/sgld.py:471-479), kept
on the device for the kernels.
"""
from __future__ import annotations

import contextlib
import ctypes as C

import numpy as np
import torch

from . import _lib as L
from .arena import default_grad_arena


def segment_attrs(names, readout_name, bias, requires_grad):
    attrs = []
    for nm, rg in zip(names, requires_grad):
        a = 0
        if readout_name is not None and readout_name in nm:
            a |= L.ATTR_HEAD
        if not ("bias" in nm and bias == "uninformative"):
            a |= L.ATTR_PRIOR
        if not rg:
            a |= L.ATTR_SKIP
        attrs.append(a)
    return attrs


def build_runs(offsets, numels, attrs, n):
    """Host-side call of bdl_build_runs; returns an int64 [nruns, 2] CPU tensor."""
    nseg = len(offsets)
    segs = (L.Segment * max(nseg, 1))()
    for i, (o, k, a) in enumerate(zip(offsets, numels, attrs)):
        segs[i].offset, segs[i].numel, segs[i].attr, segs[i].pad = int(o), int(k), int(a), 0
    cap = 2 * nseg + 2
    runs = (L.Run * cap)()
    nr = L.lib().bdl_build_runs(segs, nseg, int(n), runs, cap)
    if nr < 0:
        L.check(nr, "bdl_build_runs")
    out = torch.empty(nr, 2, dtype=torch.int64)
    for i in range(nr):
        out[i, 0] = runs[i].end
        out[i, 1] = runs[i].attr
    return out


GRAD_MODES = ("tensor", "flat")
MAX_TENSOR_RUNS = 2730  # 24 B per run in 64 KiB of LDS (bdl_step_args.grad_base)
GRAD_TABLE_CACHE = 8  # device run/base tables kept per state (one per pointer set)


def default_grad_mode():
    import os
    m = os.environ.get("BDL_GRAD_MODE", "tensor")
    if m not in GRAD_MODES:
        raise ValueError(f"BDL_GRAD_MODE must be one of {GRAD_MODES}, got {m!r}")
    return m


class FlatState:
    """Flat buffers for one chain, bound to `net`'s parameters (and, in "flat"
    gradient mode, grads)."""

    def __init__(self, net, net0=None, *, readout_name=None, bias="informative",
                 need_prior=False, need_mom=True, need_noise=False, extra=(), grad_mode=None):
        named = list(net.named_parameters())
        if not named:
            raise ValueError("bayesdll_amd: the network has no parameters")
        self.names = [nm for nm, _ in named]
        self.params = [p for _, p in named]
        self.shapes = [tuple(p.shape) for p in self.params]
        self.numels = [p.numel() for p in self.params]
        self.offsets = np.concatenate([[0], np.cumsum(self.numels)[:-1]]).astype(np.int64).tolist()
        self.n = int(sum(self.numels))
        dev = self.params[0].device
        for nm, p in named:
            L.require_hip(p.data, f"parameter {nm!r}")
            if p.device != dev:
                raise RuntimeError("bayesdll_amd: all parameters must be on one device")
        self.device = dev
        self.readout_name = readout_name if readout_name is not None else getattr(
            net, "readout_name", None)
        self.bias = bias
        self.requires_grad = [p.requires_grad for p in self.params]
        self.grad_mode = grad_mode or default_grad_mode()
        if self.grad_mode not in GRAD_MODES:
            raise ValueError(f"grad_mode must be one of {GRAD_MODES}")
        if self.grad_mode == "tensor" and len(self.params) > MAX_TENSOR_RUNS:
            # one run per tensor would not fit the kernels' LDS run table
            import warnings
            warnings.warn(f"bayesdll_amd: {len(self.params)} parameter tensors > "
                          f"{MAX_TENSOR_RUNS}: using the flat gradient vector")
            self.grad_mode = "flat"

        # the swept vectors, each one allocation from torch's caching allocator
        # (no flat gradient vector in "tensor" mode)
        names_ = ["theta"] + (["grad"] if self.grad_mode == "flat" else []) + \
            (["mom"] if need_mom else []) + (["prior"] if need_prior else []) + list(extra)
        vecs = {nm: torch.zeros(self.n, dtype=torch.float32, device=dev) for nm in names_}
        # further per-element state of the sampler (e.g. Adam's m, v and the
        # SGD buffer), zeroed
        self.extra = {nm: vecs[nm] for nm in extra}
        # theta: copy then rebind every parameter as a view (same storage order
        # as nn.utils.parameters_to_vector)
        self.theta = vecs["theta"]
        with torch.no_grad():
            for p, o, k in zip(self.params, self.offsets, self.numels):
                self.theta[o:o + k].copy_(p.data.reshape(-1))
                p.data = self.theta[o:o + k].view(p.shape)
        self.grad = vecs["grad"].zero_() if self.grad_mode == "flat" else None
        self.gbase = None  # device per-run gradient bases ("tensor" mode)
        self._bind_grads()
        # "tensor" mode with BDL_GRAD_ARENA=1: the backward allocates the
        # gradients from one reservation (arena.GradArena, wrapped around
        # loss.backward() by backward_routing; opt-in)
        self.arena = None
        if self.grad_mode == "tensor" and default_grad_arena():
            from .arena import GradArena
            self.arena = GradArena(dev, 4 * self.n)

        self.mom = vecs["mom"].zero_() if need_mom else None
        self.prior = None
        if need_prior:
            self.prior = vecs["prior"].zero_()
            if net0 is not None:
                p0 = list(net0.parameters())
                if [tuple(q.shape) for q in p0] != self.shapes:
                    raise ValueError("bayesdll_amd: net0 does not match net's parameter shapes")
                with torch.no_grad():
                    for q, o, k in zip(p0, self.offsets, self.numels):
                        self.prior[o:o + k].copy_(q.detach().reshape(-1))
        self.noise = torch.empty(self.n, dtype=torch.float32, device=dev) if need_noise else None
        # divergence flag the step kernels set on a non-finite theta / grad
        self.nonfinite = torch.zeros(1, dtype=torch.int32, device=dev)

        attrs = segment_attrs(self.names, self.readout_name, bias, self.requires_grad)
        self.attrs = attrs
        self.runs = build_runs(self.offsets, self.numels, attrs, self.n).to(dev)
        self.nruns = int(self.runs.shape[0])
        self._base_runs = (self.runs, self.nruns)
        self._skip_tables = {}
        self._grad_tables = {}
        self._untouched = ()
        # which parameters received a gradient in the current backward: the
        # reference skips a parameter whose .grad is None after net.zero_grad()
        # + backward (`if p.grad is not None`, e.g. methods/csghmc.py:749).
        # "tensor" mode sees it directly (.grad stays None); "flat" mode marks
        # it with a post-accumulate hook (its .grad views always exist).
        self._touched = [False] * len(self.params) if self.grad_mode == "flat" else []
        self._hooks = [p.register_post_accumulate_grad_hook(self._mark(i))
                       for i, p in enumerate(self.params) if p.requires_grad] \
            if self.grad_mode == "flat" else []

    def _mark(self, i):
        touched = self._touched

        def hook(_p):
            touched[i] = True
        return hook

    @classmethod
    def from_segments(cls, segments, readout_name, *, bias="informative", device="cuda",
                      need_prior=False, need_mom=True, need_noise=False, init=None, extra=()):
        """Flat chain state for a segment table alone (no nn.Module): the
        benchmark and kernel tests use it with synthetic vectors."""
        self = cls.__new__(cls)
        self.names = [nm for nm, _ in segments]
        self.shapes = [tuple(s) for _, s in segments]
        self.numels = [int(np.prod(s)) for s in self.shapes]
        self.offsets = np.concatenate([[0], np.cumsum(self.numels)[:-1]]).astype(np.int64).tolist()
        self.n = int(sum(self.numels))
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.readout_name = readout_name
        self.bias = bias
        self.requires_grad = [True] * len(self.names)
        self.params = []
        self._grad_ptrs = []
        f32 = dict(dtype=torch.float32, device=self.device)
        names_ = (["theta"] if init is None else []) + ["grad"] + (["mom"] if need_mom else []) \
            + (["prior"] if need_prior else []) + list(extra)
        vecs = {nm: torch.zeros(self.n, **f32) for nm in names_}
        self.extra = {nm: vecs[nm] for nm in extra}
        self.theta = vecs["theta"] if init is None else init
        self.grad_mode = "flat"
        self.gbase = None
        self.arena = None
        self._grad_tables = {}
        self._untouched = ()
        self.grad = vecs["grad"].zero_()
        self.mom = vecs["mom"].zero_() if need_mom else None
        self.prior = vecs["prior"].zero_() if need_prior else None
        self.noise = torch.empty(self.n, **f32) if need_noise else None
        self.nonfinite = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.attrs = segment_attrs(self.names, readout_name, bias, self.requires_grad)
        self.runs = build_runs(self.offsets, self.numels, self.attrs, self.n).to(self.device)
        self.nruns = int(self.runs.shape[0])
        self._base_runs = (self.runs, self.nruns)
        self._skip_tables = {}
        self._touched = []
        self._hooks = []
        return self

    # ---------------------------------------------------------------- grads
    def _bind_grads(self):
        if self.grad_mode == "tensor":
            for p in self.params:
                p.grad = None
            self._grad_ptrs = [0 if rg else None for rg in self.requires_grad]
            return
        self._grad_ptrs = []
        for p, o, k, rg in zip(self.params, self.offsets, self.numels,
                               [p.requires_grad for p in self.params]):
            if rg:
                p.grad = self.grad[o:o + k].view(p.shape)
                self._grad_ptrs.append(p.grad.data_ptr())
            else:
                self._grad_ptrs.append(None)

    def zero_grad(self):
        """Replaces net.zero_grad().  "tensor" mode: .grad = None (torch's
        set_to_none), so backward hands each fresh gradient tensor over without
        an accumulation kernel.  "flat" mode: zero the flat buffer and keep
        every .grad bound to it."""
        if self.grad_mode == "tensor":
            for p in self.params:
                p.grad = None
            return
        self.grad.zero_()
        for i in range(len(self._touched)):
            self._touched[i] = False
        for p, ptr in zip(self.params, self._grad_ptrs):
            if ptr is not None and (p.grad is None or p.grad.data_ptr() != ptr):
                self._bind_grads()
                break

    def backward_routing(self):
        """Context for `loss.backward()`: with a gradient arena, every
        allocation of the backward pass comes from its one reservation."""
        if self.arena is None:
            return contextlib.nullcontext()
        return self.arena.routing()

    def sync_grads(self):
        """After backward: if user code replaced a .grad, copy it into the flat
        buffer; then select the run table of this step — parameters that got no
        gradient (unused in the forward pass, or .grad set to None) are
        skipped, exactly like the reference's `if p.grad is not None`.
        "tensor" mode: select (or build) the run / gradient-base table of the
        gradient tensors autograd produced."""
        if self.grad_mode == "tensor":
            self._sync_tensor_grads()
            return
        rebind = False
        untouched = []
        for i, (p, o, k, ptr) in enumerate(zip(self.params, self.offsets, self.numels,
                                               self._grad_ptrs)):
            if ptr is None:
                continue
            g = p.grad
            if g is None:
                self.grad[o:o + k].zero_()
                untouched.append(i)
                rebind = True
            else:
                if g.data_ptr() != ptr:
                    self.grad[o:o + k].copy_(g.reshape(-1))
                    rebind = True
                if self._touched and not self._touched[i]:
                    untouched.append(i)
        if rebind:
            self._bind_grads()
        self._select_runs(tuple(untouched))

    def _select_runs(self, untouched):
        if not untouched:
            self.runs, self.nruns = self._base_runs
            return
        tab = self._skip_tables.get(untouched)
        if tab is None:
            attrs = list(self.attrs)
            for i in untouched:
                attrs[i] |= L.ATTR_SKIP
            runs = build_runs(self.offsets, self.numels, attrs, self.n).to(self.device)
            tab = self._skip_tables[untouched] = (runs, int(runs.shape[0]))
        self.runs, self.nruns = tab

    def use_tensor_grads(self, grads):
        """Segment-only states (no nn.Module): read the gradient of segment i
        from grads[i] (a contiguous fp32 device tensor, or None = no gradient)
        through the per-run base table, as "tensor" mode does for autograd's
        .grad tensors; the flat gradient vector is dropped."""
        if len(grads) != len(self.numels):
            raise ValueError("use_tensor_grads: one gradient (or None) per segment")
        self.grad_mode, self.grad = "tensor", None
        ptrs, untouched = [], []
        for i, (g, k) in enumerate(zip(grads, self.numels)):
            if g is None:
                ptrs.append(0)
                untouched.append(i)
                continue
            if (g.dtype != torch.float32 or g.device != self.device or not g.is_contiguous()
                    or g.numel() != k):
                raise ValueError(f"use_tensor_grads: gradient {i} must be a contiguous fp32 "
                                 f"tensor of {k} elements on {self.device}")
            ptrs.append(g.data_ptr())
        tab = self._build_grad_table(ptrs)
        self.use_grad_table((tab[0], tab[1], tab[2], tuple(untouched)))

    def _sync_tensor_grads(self):
        ptrs, untouched = [], []
        for i, (p, rg) in enumerate(zip(self.params, self.requires_grad)):
            g = p.grad if rg else None
            if g is None:
                ptrs.append(0)
                if rg:
                    untouched.append(i)
                continue
            if g.dtype != torch.float32 or g.device != self.device or not g.is_contiguous():
                g = g.to(device=self.device, dtype=torch.float32).contiguous()
                p.grad = g
            ptrs.append(g.data_ptr())
        key = tuple(ptrs)
        tab = self._grad_tables.get(key)
        if tab is None:
            tab = self._build_grad_table(ptrs)
            if len(self._grad_tables) >= GRAD_TABLE_CACHE:
                self._grad_tables.pop(next(iter(self._grad_tables)))
            self._grad_tables[key] = tab
        self.use_grad_table((tab[0], tab[1], tab[2], tuple(untouched)))

    def _build_grad_table(self, ptrs):
        """One run per tensor (a run must not span two gradient tensors): end,
        attributes (+SKIP without a gradient, +GUNALIGNED when the tensor's
        base address minus 4*offset is not 16-B aligned), and the base
        address; packed as [runs (2 int64 each) | bases] in one device
        tensor, copied from pinned memory on the current stream."""
        nt = len(self.numels)
        host = torch.empty(3 * nt, dtype=torch.int64).pin_memory()
        h = host.numpy()
        for i, (o, k, a, ptr) in enumerate(zip(self.offsets, self.numels, self.attrs, ptrs)):
            base = ptr - 4 * o if ptr else 0
            at = a | (L.ATTR_SKIP if not ptr else 0)
            if ptr and base % 16:
                at |= L.ATTR_GUNALIGNED
            h[2 * i] = o + k
            h[2 * i + 1] = at
            h[2 * nt + i] = base
        dev = host.to(self.device, non_blocking=True)
        return dev[:2 * nt].view(nt, 2), nt, dev[2 * nt:]

    def diverged(self, reset=True):
        """Did any step since the last reset write a non-finite theta / grad?
        (One device-to-host read: call it at epoch granularity, not per step.)"""
        bad = bool(self.nonfinite.item())
        if bad and reset:
            self.nonfinite.zero_()
        return bad

    # ------------------------------------------------- buckets (overlap)
    def bucket_plan(self, target_elems):
        """Contiguous buckets of whole tensors, each about `target_elems`
        long, cut only at flat offsets that are multiples of 4 (a float4 group
        never spans two buckets): [(start, end, tensor indices), ...]."""
        out, start, cur = [], 0, []
        for i, (o, k) in enumerate(zip(self.offsets, self.numels)):
            cur.append(i)
            end = o + k
            if end - start >= target_elems and end % 4 == 0:
                out.append((start, end, tuple(cur)))
                start, cur = end, []
        if cur:
            out.append((start, self.n, tuple(cur)))
        return out

    def bucket_host_table(self, bucket, ptrs):
        """The run / gradient-base table of one bucket as a CPU int64 tensor of
        3 * (tensors in the bucket) entries, [ends, attributes | bases]: run
        ends relative to the bucket start, gradient bases shifted so local
        element e reads ptrs[j] + 4*(start + e - offset_j); 0 = no gradient
        (SKIP)."""
        start, _, idx = bucket
        nt = len(idx)
        host = torch.empty(3 * nt, dtype=torch.int64)
        h = host.numpy()
        for j, (i, ptr) in enumerate(zip(idx, ptrs)):
            o, k = self.offsets[i], self.numels[i]
            at = self.attrs[i] | (L.ATTR_SKIP if not ptr else 0)
            base = ptr - 4 * o + 4 * start if ptr else 0
            if ptr and base % 16:
                at |= L.ATTR_GUNALIGNED
            h[2 * j], h[2 * j + 1], h[2 * nt + j] = o + k - start, at, base
        return host

    def bucket_state(self, bucket, ptrs, table=None):
        """A launchable view of one bucket: every vector sliced to
        [start, end), with the bucket's per-tensor run / gradient-base table
        (bucket_host_table) on the device; launch it with philox_offset =
        start // 4 for the whole-vector noise.  table: a device int64 tensor
        of 3 * (tensors in the bucket) entries to point the launch at instead
        of a cached copy of the table — left UNFILLED (the graph-mode capture
        allocates it before the capture and fills it once the static
        gradients exist, _base._capture_overlapped)."""
        from types import SimpleNamespace
        start, end, idx = bucket
        nt = len(idx)
        if table is None:
            key = (start, tuple(ptrs))
            tab = self._grad_tables.get(key)
            if tab is None:
                dev = self.bucket_host_table(bucket, ptrs).pin_memory().to(self.device,
                                                                            non_blocking=True)
                tab = (dev[:2 * nt].view(nt, 2), nt, dev[2 * nt:])
                if len(self._grad_tables) >= 4 * GRAD_TABLE_CACHE:
                    self._grad_tables.pop(next(iter(self._grad_tables)))
                self._grad_tables[key] = tab
        else:
            if table.numel() != 3 * nt or table.dtype != torch.int64 or table.device != self.device:
                raise ValueError("bucket_state: table must be 3 x (bucket tensors) int64 on the device")
            tab = (table[:2 * nt].view(nt, 2), nt, table[2 * nt:])
        sl = (lambda v: None if v is None else v[start:end])
        return SimpleNamespace(theta=self.theta[start:end], grad=None, gbase=tab[2], runs=tab[0],
                               nruns=tab[1], mom=sl(self.mom), prior=sl(self.prior), noise=None,
                               n=end - start, device=self.device, nonfinite=self.nonfinite,
                               extra={k: v[start:end] for k, v in self.extra.items()}, timer=None)

    def grad_table(self):
        """The run / gradient-base selection of the current step (to reuse
        when the same gradient tensors are produced again, e.g. graph replay)."""
        return (self.runs, self.nruns, self.gbase, self._untouched)

    def use_grad_table(self, t):
        self.runs, self.nruns, self.gbase, self._untouched = t

    def has_grad(self, i):
        """Did parameter i receive a gradient in the current step?"""
        if not self.requires_grad[i]:
            return False
        if self.grad_mode == "tensor":
            return i not in self._untouched
        return not self._touched or self._touched[i]

    def check_bound(self):
        """Raise if a parameter no longer aliases the flat theta buffer."""
        for nm, p, o in zip(self.names, self.params, self.offsets):
            if p.data.data_ptr() != self.theta.data_ptr() + 4 * o:
                raise RuntimeError(f"bayesdll_amd: parameter {nm!r} was re-allocated outside the "
                                   "sampler; rebuild the sampler state")

    # --------------------------------------------------------------- views
    def views(self, vec):
        return [vec[o:o + k].view(s) for o, k, s in zip(self.offsets, self.numels, self.shapes)]

    def fill_noise_torch(self, generator=None):
        """Per-tensor standard-normal draws in named_parameters order: the same
        generator calls as the reference's torch.randn_like(p) per tensor
        (methods/csghmc.py:766) — used by the "torch" parity noise mode."""
        for i, v in enumerate(self.views(self.noise)):
            if self.has_grad(i):
                v.normal_(generator=generator)
        return self.noise

    def segment_table(self):
        return [(nm, o, k, a) for nm, o, k, a in zip(self.names, self.offsets, self.numels,
                                                       self.attrs)]


def runs_ptr(state):
    return C.c_void_p(state.runs.data_ptr())


def bind_parameters(net, flat=None):
    """Rebind `net`'s parameters as views of ONE flat fp32 buffer (a new one,
    or `flat`; values copied) and drop their grads; returns the buffer.  Used
    for the evaluation copies whose theta the posterior-sample kernel writes
    in one sweep."""
    params = list(net.parameters())
    n = sum(p.numel() for p in params)
    dev = params[0].device
    if flat is None:
        flat = torch.empty(n, dtype=torch.float32, device=dev)
    elif flat.numel() != n or flat.dtype != torch.float32 or flat.device != dev:
        raise ValueError("bind_parameters: flat buffer does not match the network")
    off = 0
    with torch.no_grad():
        for p in params:
            k = p.numel()
            flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = flat[off:off + k].view(p.shape)
            p.grad = None
            off += k
    return flat


MOMENT_PAIR_ALIGN = 64  # elements: m2 starts 256 B after a 256-B boundary
MOMENT_PAIR_MIN_ELEMS = 1 << 24  # smaller pairs: two plain allocations


def moment_pair(n, device):
    """(m1, m2) for one cycle's Welford / running moments (methods/csghmc.py:333-337,
    methods/csgld.py:282-293): the two halves of ONE allocation, m2 starting
    on a 256-B boundary.  Why: the posterior draw (m1 r, m2 r, out w) ran
    0.608-0.616 ms for ViT-L/32 with m1 / m2 in one allocation against
    0.631-0.650 with the two split over separately allocated physical memory
    (profiles/round2/placement/aux_roles/collect_and_sample_by_class.jsonl);
    the collect steps that fill them do not care (1.754-1.762 ms).  A layout,
    not a search.  Pairs below MOMENT_PAIR_MIN_ELEMS: two plain allocations.
    Values never depend on it; torch.save of both halves in one call stores
    the shared storage once."""
    f32 = dict(dtype=torch.float32, device=device)
    if n < MOMENT_PAIR_MIN_ELEMS:
        return torch.empty(n, **f32), torch.empty(n, **f32)
    stride = -(-n // MOMENT_PAIR_ALIGN) * MOMENT_PAIR_ALIGN
    buf = torch.empty(stride + n, **f32)
    return buf[:n], buf[stride:stride + n]


def fill_normal_per_tensor(vec, numels, generator=None):
    """Per-tensor normal_() over consecutive slices of `vec` (the reference's
    per-parameter torch.randn_like(p) stream)."""
    off = 0
    for k in numels:
        vec[off:off + k].normal_(generator=generator)
        off += k
    return vec
