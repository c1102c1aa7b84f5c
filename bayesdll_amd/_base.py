"""Shared machinery of the drop-in sampler Models.

Each method module (csghmc, sghmc, csgld, sgld) keeps the reference's
`Model(nn.Module).forward(x, y, net, net0, criterion, lrs, Ninflate, nd, ...)`
signature and return value `(loss.item(), out.detach())`.  What changes is
what happens after `loss.backward()`: instead of the per-tensor Python loop,
one fused HIP kernel updates the chain's flat state.

Noise modes (`Model.noise_mode`, or env BDL_NOISE_MODE):
  "philox"   — N(0,1) generated inside the kernel by Philox4x32-10 keyed by
               (seed, chain, step, element): no noise buffer, no extra HBM
               traffic (the production mode).
  "torch"    — per-tensor `normal_()` draws from torch's generator into a flat
               noise buffer, in named_parameters order, on every step: the
               exact stream the reference's `torch.randn_like(p)` consumes, so
               a chain matches the reference sampler draw-for-draw on the same
               device and seed.
  "external" — `Model.noise_provider(step, flat_noise)` fills the buffer
               (used by the parity tests to replay captured reference noise).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import gc
import os
import time

import torch
import torch.nn as nn

from . import _lib as L
from .flat import FlatState

NOISE_MODES = ("philox", "torch", "external")

# Captured graphs whose sampler was dropped while a capture was in progress on
# this thread: destroying them then would free their private pools on a
# capturing stream (a process abort), so they are parked here and destroyed at
# the next point outside any capture (release_deferred_graphs).
_DEFERRED_GRAPHS = []


def release_deferred_graphs():
    """Destroy the graphs parked by a sampler dropped during a capture."""
    if _DEFERRED_GRAPHS and not torch.cuda.is_current_stream_capturing():
        torch.cuda.synchronize()
        _DEFERRED_GRAPHS.clear()


def _drop_graphs(graphs):
    """Destroy `graphs` (a list) now, or park them if a capture is running."""
    if not graphs:
        return
    if torch.cuda.is_current_stream_capturing():
        _DEFERRED_GRAPHS.extend(graphs)
    else:
        torch.cuda.synchronize()  # no replay of these graphs still in flight
        graphs.clear()
        release_deferred_graphs()
MAX_GRAPHS = 4  # captured forward/backward graphs per sampler (one per input shape)
# with the update captured: one per (input shape, step kind).  Each holds a
# private pool with its own static gradients and activations (for ViT-L/32 at
# batch 16 about 1.6 GB each), for an opt-in mode that does not pay
MAX_OVERLAP_GRAPHS = 8


@contextlib.contextmanager
def no_gc():
    """Keep Python's cyclic GC from running during a HIP-graph capture: an
    automatic collection triggered by allocations DURING capture can destroy
    an unrelated object that frees device memory (e.g. an old graph's private
    pool) — an operation a capturing stream forbids, which aborts the process.
    (The installed torch.cuda.graph collects garbage before capture only under
    torch.compiler.config.force_cudagraph_gc; the samplers release their own
    graphs explicitly, release_graphs, and collect before capturing.)"""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def default_noise_mode():
    m = os.environ.get("BDL_NOISE_MODE", "philox")
    if m not in NOISE_MODES:
        raise ValueError(f"BDL_NOISE_MODE must be one of {NOISE_MODES}, got {m!r}")
    return m


def default_graph():
    """BDL_GRAPH=1: replay forward + backward from a captured HIP graph."""
    return os.environ.get("BDL_GRAPH", "0") not in ("", "0", "false", "False")


def default_overlap():
    """BDL_OVERLAP=1: launch the fused update per bucket of parameters as
    their gradients complete, on a side stream, overlapping backward."""
    return os.environ.get("BDL_OVERLAP", "0") not in ("", "0", "false", "False")


# elements per overlap bucket (BDL_OVERLAP_BUCKET_MB, default 64 MB of fp32)
OVERLAP_BUCKET_ELEMS = int(float(os.environ.get("BDL_OVERLAP_BUCKET_MB", "64")) * (1 << 18))


def default_chain():
    """Chain id = process rank when torch.distributed is initialised."""
    from . import chains
    return chains.rank()


class FusedModelBase(nn.Module):
    """Holds the chain's FlatState and the noise configuration."""

    need_prior = False
    need_mom = True
    tune_method = "sgld"  # which production kernel autotune_once times for this sampler
    extra_vectors = ()    # further per-element state of the chain (FlatState.extra)

    # set by the bundled Runners: Model.forward returns the loss as a device
    # scalar instead of loss.item(), so a step issues no host synchronisation
    defer_loss = False

    def _result(self, loss, out):
        """(loss.item(), logits) as the reference's Model.forward returns them,
        or (detached device loss, logits) under defer_loss."""
        return (loss.detach() if self.defer_loss else loss.item()), out.detach()

    def __init__(self):
        super().__init__()
        self.noise_mode = default_noise_mode()
        self.noise_provider = None
        self.seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFFFFFF
        self.chain = default_chain()
        self.step_count = 0
        self.div_mode = None
        self.graph = default_graph()
        self._graphs = {}
        self._graph_bound = None  # the graph whose static gradients the params' .grad hold
        self.graph_captures = 0   # captures so far (one per input shape, unless released)
        self.overlap = default_overlap()
        self._ovl = None          # per-backward bucket bookkeeping while overlapping
        self._ovl_plan = None
        self._ovl_hooks = None
        self._side = None
        self.overlap_graph_failed = False  # the update could not be captured: eager overlap
        self.overlap_captures = 0  # capture attempts of the graph-mode overlap
        self.overlap_graph_error = None
        self.overlap_rewrite_s = 0.0  # host time rewriting captured bucket nodes
        self.overlap_replays = 0
        self._state = None
        self._state_net = None

    # -------------------------------------------------------------- state
    def state_for(self, net, net0=None):
        if self._state is None or self._state_net is not net:
            self.release_graphs()  # graphs captured against the old state's buffers
            if self.noise_mode not in NOISE_MODES:
                raise ValueError(f"noise_mode must be one of {NOISE_MODES}")
            from . import kernels as K
            self._state = FlatState(net, net0, readout_name=getattr(net, "readout_name", None),
                                    bias=getattr(self, "bias", "informative"),
                                    need_prior=self.need_prior, need_mom=self.need_mom,
                                    need_noise=self.noise_mode != "philox",
                                    extra=self.extra_vectors)
            self._state_net = net
            steps_timed = int(os.environ.get("BDL_STEP_TIMING", "0") or 0)
            if steps_timed > 0:  # sampled update timing, logged once per epoch
                self._state.timer = K.StepTimer(steps_timed)
            # launch geometry (speed only: results never depend on it), tuned
            # on the chain's OWN vectors at the first launch of each kind
            # (plain step, collect step) with that launch's arguments, the
            # vectors it writes restored after every candidate
            # (kernels.request_state_tuning)
            self._state.launch_cfg = self._state.collect_cfg = self._state.init_cfg = None
            K.request_state_tuning(self._state, self.tune_method)
        return self._state

    @property
    def flat(self):
        return self._state

    # ----------------------------------------------------------- fwd/bwd
    def forward_backward(self, st, net, x, y, criterion):
        if self.graph and x.is_cuda and y.is_cuda and torch.is_grad_enabled():
            got = self._graphed_forward_backward(st, net, x, y, criterion)
            if got is not None:
                return got
        out = net(x)
        loss = criterion(out, y)
        st.zero_grad()          # in place of net.zero_grad() (FlatState.zero_grad)
        with st.backward_routing():  # BDL_GRAD_ARENA=1: one reservation (arena.GradArena)
            loss.backward()
        st.sync_grads()         # which tensors got a gradient, and where they live
        return loss, out

    def can_overlap(self, st):
        return self.overlap and st.grad_mode == "tensor" and self.noise_mode == "philox"

    def forward_backward_overlapped(self, st, net, x, y, criterion, launch, kind=None):
        """Forward + backward with the fused update overlapped: the flat
        vectors are cut into ~64 MB buckets of whole tensors
        (FlatState.bucket_plan); when the last gradient of a bucket has been
        accumulated (post-accumulate hook), `launch(bucket_state, start)`
        enqueues that bucket's update on a side stream behind an event on the
        backward's stream — every kernel that reads those parameters has been
        enqueued before it — so the memory-bound sweep runs beside the
        GEMM-bound backward of the layers below.  Same per-element arithmetic
        and (with philox_offset = start // 4) the same noise as one launch:
        the chain is bit-identical.  Buckets holding a parameter without a
        gradient are launched after backward, with it skipped.  Philox noise
        and "tensor" gradients only (can_overlap).  In graph mode the bucket
        launches are captured with forward and backward, one graph per `kind`
        (the step's kernel selection), _graphed_overlapped."""
        if self.graph and kind is not None and x.is_cuda and y.is_cuda and \
                torch.is_grad_enabled():
            got = self._graphed_overlapped(st, net, x, y, criterion, launch, kind)
            if got is not None:
                return got
        self._ensure_ovl_plan(st)
        _, plan, owner, need = self._ovl_plan
        main = torch.cuda.current_stream(st.device)
        side = self._side

        def fire(bi):
            start, end, idx = plan[bi]
            ptrs = [0 if st.params[i].grad is None else st.params[i].grad.data_ptr() for i in idx]
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                launch(st.bucket_state(plan[bi], ptrs), start)

        out = net(x)
        loss = criterion(out, y)
        st.zero_grad()
        with st.backward_routing():
            self._backward_firing(loss, plan, need, owner, fire)
        main.wait_stream(side)
        st.sync_grads()  # which parameters got a gradient (has_grad / noise bookkeeping)
        return loss, out

    def _backward_firing(self, loss, plan, need, owner, fire):
        """loss.backward() with each bucket's `fire` called from the hook of
        its last gradient; buckets not fired by then are fired after it."""
        self._ovl = {"pending": list(need), "done": [False] * len(plan), "fire": fire,
                     "owner": owner}
        try:
            loss.backward()  # (eager: inside st.backward_routing(), the caller's)
        finally:
            ctx, self._ovl = self._ovl, None
        for bi, d in enumerate(ctx["done"]):
            if not d:
                ctx["done"][bi] = True
                fire(bi)

    def _ensure_ovl_plan(self, st):
        dev = st.device
        if self._ovl_plan is None or self._ovl_plan[0] is not st:
            plan = st.bucket_plan(OVERLAP_BUCKET_ELEMS)
            owner = {}
            for bi, (_, _, idx) in enumerate(plan):
                for i in idx:
                    owner[i] = bi
            need = [sum(1 for i in idx if st.requires_grad[i]) for _, _, idx in plan]
            self._ovl_plan = (st, plan, owner, need)
            if self._ovl_hooks is not None:
                for h in self._ovl_hooks:
                    h.remove()
            self._ovl_hooks = [p.register_post_accumulate_grad_hook(self._ovl_hook(i))
                               for i, p in enumerate(st.params) if st.requires_grad[i]]
            self._side = torch.cuda.Stream(dev)

    def _ovl_hook(self, i):
        def hook(_p):
            ctx = self._ovl
            if ctx is None:
                return
            bi = ctx["owner"][i]
            ctx["pending"][bi] -= 1
            if ctx["pending"][bi] == 0 and not ctx["done"][bi]:
                ctx["done"][bi] = True
                ctx["fire"](bi)
        return hook

    def _graphed_overlapped(self, st, net, x, y, criterion, launch, kind):
        """Graph mode with the update inside the graph, overlapped with the
        backward: the bucket launches of forward_backward_overlapped are
        captured on the side stream (fork / join through events), so the
        memory-bound sweep of a bucket runs beside the GEMM-bound backward of
        the layers below it.  The step's scalars change every step (learning
        rate, noise scale, Philox step, moment vectors, counts): before each
        replay every bucket's kernel node is rewritten in the instantiated
        graph (bdl_graph_redirect, hipGraphExecKernelNodeSetParams) by the
        same `launch` call the eager path makes, so the arguments are formed
        by one code path.  One graph per (input shape, kind), `kind` naming
        the kernel the step selects (noise on / off, collect kind).  Same
        kernels, same arguments, same order per bucket as eager: bit-identical
        chains (tests/test_gpu_graph_overlap.py)."""
        if self.overlap_graph_failed:
            # a capture or a node rewrite failed once: eager overlap from now
            # on, without recapturing every step (each attempt costs two
            # warm-up passes, a capture and a synchronisation)
            return None
        key = (tuple(x.shape), x.dtype, tuple(y.shape), y.dtype, net.training, id(criterion),
               id(net), "overlap", kind)
        g = self._graphs.get(key)
        if g is None:
            if len(self._graphs) >= MAX_OVERLAP_GRAPHS:
                return None
            self.overlap_captures += 1
            g = self._capture_overlapped(st, net, x, y, criterion, launch)
            if g is None:
                self.overlap_graph_failed = True
                return None
            self._graphs[key] = g
        self._bind_graph_grads(st, g)
        h = L.lib()
        ex = g["graph"].raw_cuda_graph_exec()
        t0 = time.perf_counter()
        try:
            for bi, node in enumerate(g["nodes"]):
                L.check(h.bdl_graph_redirect(ex, node), "bdl_graph_redirect")
                launch(g["buckets"][bi], g["plan"][bi][0])
        except RuntimeError as e:  # a node that is not this step's kernel: eager overlap
            del self._graphs[key]
            _drop_graphs([g["graph"]])
            self.overlap_graph_failed, self.overlap_graph_error = True, str(e)
            return None
        finally:
            h.bdl_graph_redirect(None, None)
        # host time spent rewriting the bucket nodes (informational)
        self.overlap_rewrite_s += time.perf_counter() - t0
        self.overlap_replays += 1
        g["x"].copy_(x)
        g["y"].copy_(y)
        g["graph"].replay()
        st.use_grad_table(g["table"])
        if st._touched:
            st._touched[:] = g["touched"]
        return g["loss"], g["out"].detach().clone()

    def _capture_overlapped(self, st, net, x, y, criterion, launch):
        """Capture forward + backward with every bucket's update launched from
        the post-accumulate hook of its last gradient, on the side stream.

        The buckets' run / gradient-base tables are allocated BEFORE the
        capture, from torch's ordinary pool, and filled AFTER it from the
        graph's static gradients.  (Round 4 allocated them inside the capture,
        from the hooks: mid-backward, the graph's private pool hands out
        blocks that earlier nodes of the same graph use for activations, so
        every replay's forward overwrote the table the bucket kernel then read
        — garbage gradient bases, HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION
        on the first replay.)  Before the graph is used, each captured node's
        arguments are read back and checked against the bucket it launches
        (_check_overlap_nodes)."""
        from . import kernels as K
        sx, sy = x.detach().clone(), y.detach().clone()
        self._warm_up(st, net, sx, sy, criterion)
        self._ensure_ovl_plan(st)
        _, plan, owner, need = self._ovl_plan
        if K._ACTIVE[0] is None:
            # pin the geometry the nodes are captured with, so every replay's
            # redirect re-installs it (bs.launch_cfg below) whatever another
            # state installs in between
            K.set_launch_config(*K.LIBRARY_DEFAULT)
        side = self._side
        nodes, buckets, hook_ptrs = [None] * len(plan), [None] * len(plan), [None] * len(plan)
        sizes = [3 * len(idx) for _, _, idx in plan]
        tables = torch.zeros(sum(sizes), dtype=torch.int64, device=st.device)  # outside the graph pool
        views, off = [], 0
        for k in sizes:
            views.append(tables[off:off + k])
            off += k
        h = L.lib()

        def fire(bi):
            start, end, idx = plan[bi]
            ptrs = [0 if st.params[i].grad is None else st.params[i].grad.data_ptr() for i in idx]
            hook_ptrs[bi] = ptrs
            bs = st.bucket_state(plan[bi], ptrs, table=views[bi])
            main = torch.cuda.current_stream(st.device)
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                launch(bs, start)
            bs.launch_cfg = K._ACTIVE[0]  # the kernel (unroll) the node was captured with
            buckets[bi] = bs

        st.zero_grad()
        graph = torch.cuda.CUDAGraph(keep_graph=True)  # node handles stay valid
        with no_gc(), torch.cuda.graph(graph):
            out = net(sx)
            loss = criterion(out, sy)
            self._backward_firing(loss, plan, need, owner, fire)
            torch.cuda.current_stream(st.device).wait_stream(side)
        raw = graph.raw_cuda_graph()
        for bi, bs in enumerate(buckets):  # each bucket's kernel node, by kernel and range
            node = C.c_void_p()
            if bs is not None and h.bdl_graph_find_step_node(
                    raw, bs.theta.data_ptr(), int(bs.n), C.byref(node)) == L.BDL_OK:
                nodes[bi] = node.value
        err = None
        if any(n is None for n in nodes):
            err = "a bucket's kernel node was not found in the captured graph"
        elif any(p.grad is not None and (p.grad.dtype != torch.float32 or
                                         not p.grad.is_contiguous()) for p in st.params):
            err = "a captured gradient is not a contiguous fp32 tensor"
        else:
            # the tables from the graph's static gradients (the hooks saw the same)
            static = [[0 if st.params[i].grad is None else st.params[i].grad.data_ptr()
                       for i in idx] for _, _, idx in plan]
            if static != hook_ptrs:
                err = "the static gradients are not the tensors the hooks saw"
            else:
                host = torch.cat([st.bucket_host_table(b, p) for b, p in zip(plan, static)])
                tables.copy_(host)
                torch.cuda.synchronize(st.device)
                err = self._check_overlap_nodes(st, plan, nodes, buckets, tables, host, static)
        if err is not None:
            self.overlap_graph_error = err
            _drop_graphs([graph])
            return None
        graph.instantiate()
        st.sync_grads()
        out, loss = out.detach(), loss.detach()
        self.graph_captures += 1
        return {"graph": graph, "x": sx, "y": sy, "out": out, "loss": loss,
                "grads": [p.grad for p in st.params], "touched": list(st._touched),
                "table": st.grad_table(), "nodes": nodes, "buckets": buckets, "plan": plan,
                "tables": tables}

    @staticmethod
    def _check_overlap_nodes(st, plan, nodes, buckets, tables, host, static):
        """Before any replay: every captured bucket node's kernel arguments
        (bdl_graph_node_step_args) point at its bucket's vectors and at the
        table allocated outside the graph; the table on the device equals the
        one built on the host; and every gradient base, shifted back by its
        tensor's offset, is the address of that tensor's static gradient.
        Returns None, or what differs."""
        h = L.lib()
        if not torch.equal(tables.cpu(), host):
            return "bucket table read back differs from the host table"
        off = 0
        for bi, ((start, end, idx), node, bs) in enumerate(zip(plan, nodes, buckets)):
            f = (C.c_int64 * 10)()
            if h.bdl_graph_node_step_args(C.c_void_p(node), f, 10) != L.BDL_OK:
                return f"bucket {bi}: node arguments unreadable"
            want = [bs.theta.data_ptr(), 0, bs.mom.data_ptr() if bs.mom is not None else 0,
                    bs.runs.data_ptr(), bs.gbase.data_ptr(), len(idx), int(bs.n)]
            got = [int(v) for v in f[:7]]
            if got != want:
                return f"bucket {bi}: captured arguments {got} != {want}"
            if bs.runs.data_ptr() != tables.data_ptr() + 8 * off:
                return f"bucket {bi}: run table not in the pre-allocated block"
            nt = len(idx)
            for j, (i, ptr) in enumerate(zip(idx, static[bi])):
                base = int(host[off + 2 * nt + j])
                if ptr and base + 4 * (st.offsets[i] - start) != ptr:
                    return f"bucket {bi} tensor {i}: gradient base does not address its .grad"
            off += 3 * nt
        return None

    def _bind_graph_grads(self, st, g):
        if g is not self._graph_bound or any(p.grad is not gt
                                             for p, gt in zip(st.params, g["grads"])):
            for p, gt in zip(st.params, g["grads"]):
                p.grad = gt
        self._graph_bound = g

    def _graphed_forward_backward(self, st, net, x, y, criterion):
        """Forward + loss + backward replayed from a captured HIP graph
        (torch.cuda.CUDAGraph = hipGraph on ROCm): one graph launch instead of
        one host launch per kernel, which is what bounds a small network's step
        (mlp_mnist: tools/e2e_compare.py).  The graph holds exactly the eager
        ops (in "tensor" gradient mode autograd's gradient tensors become
        static graph outputs the kernel reads through the captured base table;
        in "flat" mode the graph zeroes the flat buffer autograd accumulates
        into), so a step is bit-identical to eager mode for networks whose
        forward has no random ops.  Assumes a static network: which parameters
        get a gradient is fixed at capture (the eager path re-checks it every
        step, like the reference's `if p.grad is not None`).  One graph per
        (input shape, dtype, train mode, criterion), at most MAX_GRAPHS;
        beyond that, eager.  A replay binds every .grad to its graph's static
        gradients, so switching between shapes never recaptures."""
        key = (tuple(x.shape), x.dtype, tuple(y.shape), y.dtype, net.training, id(criterion),
               id(net))
        g = self._graphs.get(key)
        if g is None:
            if len(self._graphs) >= MAX_GRAPHS:
                return None
            g = self._capture(st, net, x, y, criterion)
            if g is None:  # not capturable as is: stay eager for this shape
                self.graph = False
                return None
            self._graphs[key] = g
        # another shape's graph (a ragged last batch, then the next epoch's
        # full one), an eager step or user code left other tensors in .grad:
        # point every .grad at this graph's static gradient outputs (the
        # update reads them through the graph's table either way)
        self._bind_graph_grads(st, g)
        g["x"].copy_(x)
        g["y"].copy_(y)
        g["graph"].replay()
        st.use_grad_table(g["table"])
        if st._touched:
            st._touched[:] = g["touched"]
        return g["loss"], g["out"].detach().clone()

    def release_graphs(self):
        """Drop every captured graph (and with it its private memory pool) now,
        deterministically, on the caller's stream — never from a garbage
        collection that might run inside another capture.  Called when the
        sampler state is rebuilt (its buffers are what the graphs captured);
        call it when done with a sampler instead of leaving the graphs to the
        garbage collector."""
        graphs, self._graphs, self._graph_bound = self._graphs, {}, None
        _drop_graphs(list(graphs.values()))

    def __del__(self):
        """A dropped sampler releases its graphs deterministically here (or
        parks them when dropped inside another capture), instead of leaving
        their pools to whichever garbage collection runs next."""
        try:
            if getattr(self, "_graphs", None):
                self.release_graphs()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def _capture(self, st, net, x, y, criterion):
        sx, sy = x.detach().clone(), y.detach().clone()
        self._warm_up(st, net, sx, sy, criterion)
        st.zero_grad()  # "tensor" mode: .grad = None, so the graph's gradients are its own
        graph = torch.cuda.CUDAGraph()
        with no_gc(), torch.cuda.graph(graph):
            if st.grad is not None:  # "flat" mode: the graph zeroes the flat buffer
                st.grad.zero_()
            out = net(sx)
            loss = criterion(out, sy)
            loss.backward()
        if st.grad is None and any(p.grad is not None and (p.grad.dtype != torch.float32 or
                                                           not p.grad.is_contiguous())
                                   for p in st.params):
            return None  # the table would point at eager copies, not the graph's outputs
        st.sync_grads()  # the (static) gradient tensors' table; which parameters got one
        # keep the static outputs, not the captured autograd graph: its
        # AccumulateGrad nodes would otherwise outlive the capture and meet the
        # next capture's warm-up on another stream
        out, loss = out.detach(), loss.detach()
        self.graph_captures += 1
        return {"graph": graph, "x": sx, "y": sy, "out": out, "loss": loss,
                "grads": [p.grad for p in st.params], "touched": list(st._touched),
                "table": st.grad_table()}

    def _warm_up(self, st, net, sx, sy, criterion):
        gc.collect()  # pending garbage (old pools included) goes before the capture, not in it
        release_deferred_graphs()
        # warm-up passes on a side stream (library handles, autotuned kernels)
        # must not move the network's state: keep buffers (BatchNorm running
        # statistics) and the device RNG as they were
        bufs = [b.detach().clone() for b in net.buffers()]
        rng = torch.cuda.get_rng_state(st.device)
        side = torch.cuda.Stream(st.device)
        side.wait_stream(torch.cuda.current_stream(st.device))
        with torch.cuda.stream(side):
            for _ in range(2):
                st.zero_grad()
                criterion(net(sx), sy).backward()
        torch.cuda.current_stream(st.device).wait_stream(side)
        with torch.no_grad():
            for b, c in zip(net.buffers(), bufs):
                b.copy_(c)
        torch.cuda.set_rng_state(rng, st.device)

    # -------------------------------------------------------------- noise
    def draw_noise(self, st):
        """Advance the noise source for this step; return the kernel noise mode
        to use when the noise term is applied."""
        if self.noise_mode == "philox":
            return L.NOISE_PHILOX
        if self.noise_mode == "torch":
            st.fill_noise_torch()
        else:
            if self.noise_provider is None:
                raise RuntimeError("noise_mode='external' needs Model.noise_provider")
            self.noise_provider(self.step_count, st.noise)
        return L.NOISE_BUFFER

    # ------------------------------------------------------ reference API
    @property
    def momentum_buffer(self):
        """name -> momentum view (the reference's dict, methods/csghmc.py:727-730)."""
        st = self._state
        if st is None or st.mom is None:
            return {}
        return dict(zip(st.names, st.views(st.mom)))

    def load_momentum_buffer(self, d, flat=None):
        """Copy a saved name -> tensor dict into the flat buffer (st.mom, or
        `flat`), in place, so the kernel's pointers stay valid."""
        st = self._state
        if st is None:
            raise RuntimeError("load the checkpoint after the first step has bound the state")
        dst = st.mom if flat is None else flat
        with torch.no_grad():
            for nm, v in zip(st.names, st.views(dst)):
                if nm in d:
                    v.copy_(d[nm].reshape(v.shape))
