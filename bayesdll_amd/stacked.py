"""Stacked chains: K independent SG-MCMC chains of one network on one device.

The reference runs one chain per process (methods/csghmc.py:41); its own
recipe for more chains is more processes.  On an MI355X a small network
leaves the device idle between launches, so K chains here share every
launch instead:

  * the K chains' flat vectors are stacked chain-major in one buffer
    (`theta[k]` = parameters_to_vector of chain k, padded to a multiple of 4
    elements so every chain starts on a float4 group);
  * forward and backward run once for all chains, `torch.func.vmap` over
    `functional_call` with the chains' parameters as strided views of the
    stacked theta (the data batch shared, or one batch per chain);
  * ONE fused update launch (`bdl_sgmcmc_step` with `chain_groups`, ABI v6)
    covers all chains, reading each chain's gradient in place from the vmapped
    gradient tensors through the per-run base table (one run per chain and
    tensor), with the Welford collect of methods/csghmc.py:327-345 fused.

Chain k draws the Philox noise of a one-chain sampler with chain id
`chain0 + k` (same seed, same step keys): its update equals the one-chain
update bit for bit given the same gradient (tests/test_gpu_stacked.py).  The
gradients come from batched GEMMs, so a stacked chain agrees with a separately
run chain to rounding, not bitwise.

Scope: StackedCSGHMC (the north-star sampler: cyclical schedule, thinning,
per-cycle Welford moments), StackedSGLD (SGLD + SGD momentum, prior mean
theta0, burn-in, thinned running moments), StackedSGHMC (the same loop with
the SGHMC momentum update) and StackedCSGLD (cyclical SGLD, per-cycle running
moments); the predictive averages
probabilities uniformly over chains and (nst posterior draws of) the collected
components.  Networks with BatchNorm running statistics are refused (vmap cannot
update shared buffers per chain), and every trainable parameter must take part
in the forward pass (torch.func returns zeros, not None, for unused inputs).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch
import torch.nn.functional as F
from torch.func import functional_call, grad_and_value, vmap

from . import _lib as L
from . import kernels as K
from ._base import no_gc
from ._runner import EVAL_STEP_BASE
from .cyclical import CyclicalSGMCMC
from .flat import MAX_TENSOR_RUNS, build_runs, segment_attrs


class StackedState:
    """K chains' flat cSGHMC state of one network, stacked chain-major.

    theta2d / mom2d are [K, stride] (stride = n rounded up to 4); `params`
    maps every parameter name to its [K, *shape] strided view of theta2d.  The
    launchable attributes (theta, grad / gbase, mom, runs, nruns, n,
    chain_groups, nonfinite) are what kernels._step_args reads."""

    def __init__(self, net, K_, *, readout_name=None, bias="informative", init="copy",
                 seed=0, need_mom=True, need_prior=False, net0=None):
        import torch.nn as nn
        if K_ < 1:
            raise ValueError("StackedState: K must be >= 1")
        for m in net.modules():
            if isinstance(m, nn.modules.batchnorm._BatchNorm) and m.track_running_stats:
                raise ValueError("StackedState: BatchNorm running statistics cannot be stacked "
                                 "(use track_running_stats=False or one chain per process)")
        named = list(net.named_parameters())
        if not named:
            raise ValueError("StackedState: the network has no parameters")
        dev = named[0][1].device
        for nm, p in named:
            L.require_hip(p.data, f"parameter {nm!r}")
        self.K = int(K_)
        self.device = dev
        self.names = [nm for nm, _ in named]
        self.shapes = [tuple(p.shape) for _, p in named]
        self.numels = [p.numel() for _, p in named]
        self.offsets = np.concatenate([[0], np.cumsum(self.numels)[:-1]]).astype(np.int64).tolist()
        self.n1 = int(sum(self.numels))
        self.stride = (self.n1 + 3) // 4 * 4
        self.n = self.K * self.stride
        self.chain_groups = self.stride // 4
        if (self.n + 3) // 4 >= 1 << 32:
            raise ValueError("StackedState: K * n too large for stacked Philox keys")
        self.requires_grad = [p.requires_grad for _, p in named]
        self.readout_name = readout_name if readout_name is not None else getattr(
            net, "readout_name", None)
        self.attrs = segment_attrs(self.names, self.readout_name, bias, self.requires_grad)

        f32 = dict(dtype=torch.float32, device=dev)
        self.theta2d = torch.zeros(self.K, self.stride, **f32)
        with torch.no_grad():
            src = torch.cat([p.detach().reshape(-1).float() for _, p in named])
            self.theta2d[:, :self.n1].copy_(src)
            if init == "reinit":
                import copy
                from ._runner import reinit_network
                tmp = copy.deepcopy(net)
                for k in range(self.K):
                    with torch.random.fork_rng(devices=[dev] if dev.type == "cuda" else []):
                        torch.manual_seed(int(seed) + k)
                        reinit_network(tmp)
                    self.theta2d[k, :self.n1].copy_(
                        torch.cat([p.detach().reshape(-1) for p in tmp.parameters()]))
            elif init != "copy":
                raise ValueError("StackedState: init must be 'copy' or 'reinit'")
        self.theta = self.theta2d.view(-1)
        self.mom2d = torch.zeros(self.K, self.stride, **f32) if need_mom else None
        self.mom = None if self.mom2d is None else self.mom2d.view(-1)
        self.noise = None
        # prior mean theta0 (SGLD): net0's parameters (zeros without one) in
        # every chain's slot
        self.prior = None
        if need_prior:
            p2 = torch.zeros(self.K, self.stride, **f32)
            if net0 is not None:
                p0 = [q.detach().reshape(-1).float() for q in net0.parameters()]
                if [q.numel() for q in p0] != self.numels:
                    raise ValueError("StackedState: net0 does not match net's parameter shapes")
                with torch.no_grad():
                    p2[:, :self.n1].copy_(torch.cat(p0).to(dev))
            self.prior = p2.view(-1)
        self.nonfinite = torch.zeros(1, dtype=torch.int32, device=dev)
        self.params = {nm: self.theta2d[:, o:o + k].view(self.K, *s)
                       for nm, o, k, s in zip(self.names, self.offsets, self.numels, self.shapes)}
        # gradient source: per-run bases into the vmapped gradient tensors
        # ("tensor"), or a stacked gradient vector the gradients are copied into
        # ("flat", when K x tensors runs would not fit the LDS run table)
        gap = 1 if self.stride > self.n1 else 0
        self.grad_mode = "tensor" if self.K * (len(self.names) + gap) <= MAX_TENSOR_RUNS else "flat"
        self.grad, self.gbase, self._tables = None, None, {}
        if self.grad_mode == "flat":
            self.grad2d = torch.zeros(self.K, self.stride, **f32)
            self.grad = self.grad2d.view(-1)
            offs, nums, ats = [], [], []
            for k in range(self.K):
                for o, kk, a in zip(self.offsets, self.numels, self.attrs):
                    offs.append(k * self.stride + o)
                    nums.append(kk)
                    ats.append(a)
            self.runs = build_runs(offs, nums, ats, self.n).to(dev)
            self.nruns = int(self.runs.shape[0])
        else:
            self.runs, self.nruns = None, 0
        self.timer = None
        self.extra = {}

    def chain_vector(self, k):
        """parameters_to_vector of chain k (a view)."""
        return self.theta2d[k, :self.n1]

    def load_chain(self, net, k):
        """Copy chain k's parameters into `net` (same architecture)."""
        with torch.no_grad():
            for p, o, n in zip(net.parameters(), self.offsets, self.numels):
                p.copy_(self.theta2d[k, o:o + n].view(p.shape))

    def use_grads(self, grads):
        """Point the next launch at the vmapped gradients {name: [K, *shape]}
        (None or a missing name: that tensor is frozen / has no gradient)."""
        gl = [grads.get(nm) for nm in self.names]
        if self.grad_mode == "flat":
            for g, o, k in zip(gl, self.offsets, self.numels):
                if g is not None:
                    self.grad2d[:, o:o + k].copy_(g.reshape(self.K, k))
            return
        ptrs = []
        for g, k in zip(gl, self.numels):
            if g is None:
                ptrs.append(0)
                continue
            if (g.dtype != torch.float32 or g.device != self.device or not g.is_contiguous()
                    or g.numel() != self.K * k):
                raise ValueError("StackedState: gradients must be contiguous fp32 [K, *shape]")
            ptrs.append(g.data_ptr())
        key = tuple(ptrs)
        tab = self._tables.get(key)
        if tab is None:
            tab = self._build_table(ptrs)
            if len(self._tables) >= 8:
                self._tables.pop(next(iter(self._tables)))
            self._tables[key] = tab
        self.runs, self.nruns, self.gbase = tab

    def _build_table(self, ptrs):
        """One run per (chain, tensor) — a run must not span two gradient
        tensors — plus a SKIP run over each chain's padding; chain k of tensor
        i reads ptrs[i] + 4*(k*numel_i + j), i.e. base = that - 4*(flat index)."""
        rows, bases = [], []
        for k in range(self.K):
            for o, n, a, ptr in zip(self.offsets, self.numels, self.attrs, ptrs):
                start = k * self.stride + o
                base = ptr + 4 * k * n - 4 * start if ptr else 0
                at = a | (0 if ptr else L.ATTR_SKIP)
                if ptr and base % 16:
                    at |= L.ATTR_GUNALIGNED
                rows.append((start + n, at))
                bases.append(base)
            if self.stride > self.n1:
                rows.append(((k + 1) * self.stride, L.ATTR_SKIP))
                bases.append(0)
        nt = len(rows)
        host = torch.empty(3 * nt, dtype=torch.int64).pin_memory()
        h = host.numpy()
        h[:2 * nt] = np.asarray(rows, dtype=np.int64).reshape(-1)
        h[2 * nt:] = np.asarray(bases, dtype=np.int64)
        dev = host.to(self.device, non_blocking=True)
        return dev[:2 * nt].view(nt, 2), nt, dev[2 * nt:]

    def diverged(self, reset=True):
        bad = bool(self.nonfinite.item())
        if bad and reset:
            self.nonfinite.zero_()
        return bad


def st_big(st):
    """Worth tuning the launch geometry for (small sweeps are launch-bound)."""
    return st.device.type == "cuda" and st.n >= 1 << 20


class _StackedSampler:
    """What every stacked sampler shares: K chains' state, the vmapped
    forward/backward (optionally replayed from a HIP graph), the predictive
    over chains and collected posterior components, the epoch driver."""

    need_prior = False
    tune_method = "csghmc"  # the production kernel autotune_once times

    def __init__(self, net, K_, args, *, chain0=None, seed=None, init="copy", criterion=None,
                 per_chain_batches=False, logger=None, graph=None, net0=None):
        from . import chains
        from ._base import default_graph
        self.args, self.logger = args, logger
        # replay the vmapped forward/backward from a captured HIP graph (per
        # input shape): the vmap dispatch costs ~1.2 ms of host time per step
        self.graph = default_graph() if graph is None else bool(graph)
        self._graphs = {}
        hp = args.hparams
        self.net = net.to(args.device)
        self.prior_sig = float(hp["prior_sig"])
        self.Ninflate, self.nd = float(hp["Ninflate"]), float(hp["nd"])
        self.thin, self.nst = int(hp["thin"]), int(hp["nst"])
        self.seed = int(getattr(args, "seed", 0) or 0) if seed is None else int(seed)
        self.chain0 = chains.rank() * K_ if chain0 is None else int(chain0)
        # re-initialisation seeds seed + chain id: distinct across processes too
        self.state = StackedState(self.net, K_, bias=str(hp["bias"]), init=init,
                                  seed=self.seed + self.chain0, need_prior=self.need_prior,
                                  net0=net0)
        self.K = K_
        # launch geometry tuned for the stacked size (speed only)
        if st_big(self.state):
            # (scratch on plain allocations, as the stacked state's own vectors)
            self.state.launch_cfg = K.autotune_once(self.state.n, self.state.device,
                                                    self.tune_method)
            if self.state.launch_cfg is not None:  # the collect steps' own geometry
                self.state.collect_cfg = K.collect_config(self.state.n, self.state.device,
                                                          self.tune_method)
        self.criterion = criterion or torch.nn.CrossEntropyLoss()
        self.step_count = 0
        self.draws = 0
        st = self.state
        self.trainable = [nm for nm, rg in zip(st.names, st.requires_grad) if rg]
        self.buffers = dict(self.net.named_buffers())
        xdim = 0 if per_chain_batches else None

        # the closures hold the module, not the sampler: no reference cycle,
        # so a dropped sampler (and its graphs) is freed at once, never by a
        # later garbage collection
        net_, bufs_, crit_ = self.net, self.buffers, self.criterion

        def loss_fn(tp, fp, x, y):
            out = functional_call(net_, ({**tp, **fp}, bufs_), (x,))
            return crit_(out, y), out

        self._grad = vmap(grad_and_value(loss_fn, has_aux=True),
                          in_dims=(0, 0, xdim, xdim), randomness="different")
        # evaluation: every chain sees the same batch
        self._fwd = vmap(lambda p, x: functional_call(net_, (p, bufs_), (x,)),
                         in_dims=(0, None), randomness="different")

    def _split(self):
        p = self.state.params
        return ({nm: p[nm] for nm in self.trainable},
                {nm: p[nm] for nm in p if nm not in self.trainable})

    # ----------------------------------------------------------------- step
    def gradients(self, x, y):
        """Vmapped forward/backward of all chains: ({name: [K, *shape]},
        loss [K], logits [K, B, C]).  In graph mode these are the graph's
        static outputs, overwritten by the next step."""
        if self.graph:
            return self._graphed_gradients(x, y)
        tp, fp = self._split()
        grads, (loss, out) = self._grad(tp, fp, x, y)
        return grads, loss.detach(), out.detach()

    def _graphed_gradients(self, x, y):
        """Capture once per input shape (after two warm-up runs on a side
        stream), then copy the batch into the static inputs and replay.  The
        graph reads the chains' parameters in place (views of the stacked
        theta), so the fused update between replays is seen by the next one."""
        key = (tuple(x.shape), x.dtype, tuple(y.shape), y.dtype)
        g = self._graphs.get(key)
        if g is None:
            import gc
            gc.collect()  # pending garbage (old graphs' pools) goes before the capture
            tp, fp = self._split()
            sx, sy = x.clone(), y.clone()
            side = torch.cuda.Stream(device=self.state.device)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):
                    self._grad(tp, fp, sx, sy)
            torch.cuda.current_stream().wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with no_gc(), torch.cuda.graph(graph):
                grads, (loss, out) = self._grad(tp, fp, sx, sy)
            g = self._graphs[key] = (graph, sx, sy, grads, loss.detach(), out.detach())
        graph, sx, sy, grads, loss, out = g
        sx.copy_(x)
        sy.copy_(y)
        graph.replay()
        return grads, loss, out

    def release_graphs(self):
        """Drop the captured graphs (and their memory pools) now, after the
        device has finished with them — not whenever a collection happens."""
        graphs, self._graphs = self._graphs, {}
        if graphs:
            torch.cuda.synchronize(self.state.device)
        graphs.clear()

    def step(self, x, y, *a, **kw):
        """One step of all K chains: vmapped forward/backward, then one fused
        launch (`update`).  Returns per-chain (loss [K], logits [K, B, C]) on
        the device, without a host sync."""
        grads, loss, out = self.gradients(x, y)
        self.update(grads, *a, **kw)
        return loss, out

    def _accumulate(self, acc, loss, out, y):
        """Per-chain running (loss sum, error count, examples) on the device."""
        bs = y.shape[-1]
        acc[0] += loss.double() * bs
        acc[1] += out.argmax(-1).ne(y).sum(-1)
        acc[2] += bs

    def _new_acc(self):
        dev = self.args.device
        return [torch.zeros(self.K, dtype=torch.float64, device=dev),
                torch.zeros(self.K, dtype=torch.int64, device=dev), 0]

    @staticmethod
    def _epoch_result(acc):
        nb = max(acc[2], 1)
        return (acc[0] / nb).cpu().numpy(), (acc[1].double() / nb).cpu().numpy()

    # ----------------------------------------------------------- predictive
    def chain_logits(self, x):
        """[K, B, C] logits of every chain at its current theta."""
        with torch.no_grad():
            return self._fwd(self.state.params, x)

    def predictive_logprob(self, x):
        """log of the predictive probability averaged uniformly over the K
        chains x the collected posterior components (`_components`: posterior
        draws or means); the chains' current theta while none is collected.
        With one process per GPU (torch.distributed initialised) the
        processes' stacked predictives are averaged too
        (chains.average_predictive: one all-reduce)."""
        from . import chains
        lp = self._local_logprob(x)
        return chains.average_predictive(lp) if chains.world() > 1 else lp

    def _local_logprob(self, x):
        st = self.state
        with torch.no_grad():
            buf = torch.empty_like(st.theta)
            views = {nm: buf.view(self.K, st.stride)[:, o:o + k].view(self.K, *s)
                     for nm, o, k, s in zip(st.names, st.offsets, st.numels, st.shapes)}
            comps = [F.log_softmax(self._fwd(views, x), dim=-1) for _ in self._components(buf)]
            if not comps:
                comps = [F.log_softmax(self.chain_logits(x), dim=-1)]
            lp = torch.cat(comps, 0)  # [K * components, B, C]
            return lp.logsumexp(0) - math.log(lp.shape[0])

    def _sample(self, out, mean, m2, var_mode, ratio):
        """One posterior draw of every chain into `out` ([K*stride]); chain k
        keyed chain0 + k (= the one-chain PosteriorDraw of that chain id)."""
        K.posterior_sample(out, mean, m2, var_mode=var_mode, ratio=ratio, seed=self.seed,
                           chain=self.chain0, step=EVAL_STEP_BASE + self.draws,
                           chain_groups=self.state.chain_groups)
        self.draws += 1

    def evaluate(self, loader):
        """(NLL, error) of the stacked predictive over a data loader (the
        network in eval mode, as the reference's evaluate)."""
        dev = self.args.device
        loss, err, nb = 0.0, 0, 0
        was = self.net.training
        self.net.eval()
        try:
            for x, y in loader:
                x, y = x.to(dev), y.to(dev)
                lp = self.predictive_logprob(x)
                loss += F.nll_loss(lp, y, reduction="sum").item()
                err += lp.argmax(-1).ne(y).sum().item()
                nb += len(y)
        finally:
            self.net.train(was)
        return loss / nb, err / nb

    # ---------------------------------------------------------- checkpoint
    def state_dict(self):
        """Everything an exact continuation of all K chains needs: the stacked
        theta / momentum / prior, the sampler's step counter (the Philox step
        key), draw counter and the method's moments and counters."""
        st = self.state
        d = {"stacked": type(self).__name__, "K": self.K, "chain0": self.chain0,
             "seed": self.seed, "n": st.n1, "stride": st.stride, "theta": st.theta,
             "mom": st.mom, "prior": st.prior, "step_count": self.step_count,
             "draws": self.draws}
        d.update(self._extra_state())
        return d

    def save_ckpt(self, path):
        torch.save(self.state_dict(), path)
        return path

    def load_ckpt(self, path):
        """Restore a save_ckpt file (weights-only load) into this sampler."""
        d = torch.load(path, map_location=self.state.device, weights_only=True)
        st = self.state
        if (d.get("stacked") != type(self).__name__ or d["K"] != self.K or d["n"] != st.n1
                or d["stride"] != st.stride):
            raise ValueError("load_ckpt: checkpoint of a different stacked sampler / network")
        with torch.no_grad():
            st.theta.copy_(d["theta"])
            for mine, theirs in ((st.mom, d["mom"]), (st.prior, d["prior"])):
                if mine is not None and theirs is not None:
                    mine.copy_(theirs)
        self.chain0, self.seed = d["chain0"], d["seed"]
        self.step_count, self.draws = d["step_count"], d["draws"]
        self._load_extra_state(d)
        return d

    def train(self, train_loader, test_loader=None, start_epoch=0):
        """Run epochs start_epoch .. args.epochs-1 (start_epoch > 0 continues
        after load_ckpt); logs per-chain losses and, after the epochs
        `_evaluate_after` names, the stacked predictive on test_loader."""
        log = self.logger.info if self.logger is not None else (lambda *_: None)
        hist = []
        for ep in range(start_epoch, self.args.epochs):
            tic = time.time()
            lt, et = self.train_one_epoch(train_loader, ep)
            if self.state.diverged():
                log(f"[Epoch {ep}] a chain wrote a non-finite theta")
            rec = {"epoch": ep, "loss": lt.tolist(), "error": et.tolist(),
                   "seconds": time.time() - tic}
            log(f"[Epoch {ep}/{self.args.epochs}] {self.K} chains: loss = {lt.mean():.4f} "
                f"(min {lt.min():.4f}, max {lt.max():.4f}), error = {et.mean():.4f} "
                f"({rec['seconds']:.2f} s)")
            if test_loader is not None and self._evaluate_after(ep, train_loader):
                rec["test"] = self.evaluate(test_loader)
                log(f"(Epoch {ep}) stacked predictive: loss = {rec['test'][0]:.4f}, "
                    f"error = {rec['test'][1]:.4f}")
            hist.append(rec)
        return hist


class StackedCSGHMC(_StackedSampler):
    """K cyclical-SGHMC chains of `net` on one device, stepped together.

    `args` carries the csghmc Runner's fields (lr, lr_head, epochs,
    num_cycles, proportion_exploration, ND, hparams with prior_sig,
    momentum_decay, Ninflate, nd, thin, nst, bias; device).  Chains are
    keyed chain0 + k (default: rank * K, so chains stay distinct across
    processes) with Philox seed `seed`."""

    def __init__(self, net, K_, args, **kw):
        super().__init__(net, K_, args, **kw)
        self.momentum_decay = float(args.hparams["momentum_decay"])
        self.sched = CyclicalSGMCMC(base_lr=args.lr, nbr_of_cycles=getattr(args, "num_cycles", 10),
                                    epochs=args.epochs,
                                    proportion_exploration=getattr(args, "proportion_exploration",
                                                                   0.5))
        self.samples_per_cycle, self.mom1, self.mom2 = {}, {}, {}

    def update(self, grads, lr, should_sample=False, collect=None):
        """The fused launch over all chains for given gradients (step's second
        half): v <- v(1-a) - lr(g + prior_sig theta) [+ noise]; theta += v;
        Welford collect on sample steps."""
        args, st = self.args, self.state
        st.use_grads(grads)
        lrs = (lr, lr * (args.lr_head / args.lr))
        N = args.ND * self.Ninflate
        ns = [self.nd * np.sqrt(2 * self.momentum_decay * v) / N for v in lrs]
        ckind, m1, m2, ca = (L.COLLECT_NONE, None, None, 1.0) if collect is None else collect
        K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns,
                      noise_mode=L.NOISE_PHILOX if should_sample else L.NOISE_NONE,
                      one_minus_alpha=1 - self.momentum_decay, prior_sig=self.prior_sig,
                      collect=ckind, mom1=m1, mom2=m2, collect_a=ca, seed=self.seed,
                      chain=self.chain0, step=self.step_count)
        self.step_count += 1

    def _collect_spec(self, c):
        """Welford bookkeeping of methods/csghmc.py:333-348 (quirk Q2 double
        count), shared by all chains (they sample on the same steps)."""
        st = self.state
        if c not in self.mom1:
            self.mom1[c] = torch.zeros(st.n, dtype=torch.float32, device=st.device)
            self.mom2[c] = torch.zeros(st.n, dtype=torch.float32, device=st.device)
            return (L.COLLECT_WELFORD_INIT, self.mom1[c], self.mom2[c], 1.0), 1
        n = self.samples_per_cycle.get(c, 0) + 1
        return (L.COLLECT_WELFORD, self.mom1[c], self.mom2[c], float(n)), n

    def train_one_epoch(self, loader, epoch):
        """All batches of one epoch under the cyclical schedule
        (methods/csghmc.py:246-384).  Returns per-chain (loss, error) arrays;
        one host sync per epoch."""
        dev, sched = self.args.device, self.sched
        self.net.train()
        sched.current_epoch = epoch
        bpe = len(loader)
        acc = self._new_acc()
        for b, (x, y) in enumerate(loader):
            x, y = x.to(dev, non_blocking=True), y.to(dev, non_blocking=True)
            lr = sched.calculate_lr(epoch=epoch, batch=b, batches_per_epoch=bpe)
            ss = sched.should_sample(epoch=epoch, batch=b, batches_per_epoch=bpe) \
                and b % self.thin == 0
            collect, cnt, c = None, None, None
            if ss:
                c = sched.get_cycle_number(epoch=epoch, batch=b, batches_per_epoch=bpe)
                collect, cnt = self._collect_spec(c)
            loss, out = self.step(x, y, lr, should_sample=ss, collect=collect)
            if ss:  # Q2: the reference bumps the count twice per sample
                self.samples_per_cycle[c] = cnt + 1
            self._accumulate(acc, loss, out, y)
        return self._epoch_result(acc)

    def _components(self, buf):
        """Every collected cycle: nst posterior draws (its Welford mean and
        variance M2/(n-1), 1e-12 for a single sample; methods/csghmc.py:446-468)
        or, with nst = 0, its mean."""
        for c in sorted(self.mom1):
            n = self.samples_per_cycle.get(c, 0)
            for _ in range(max(1, self.nst)):
                if self.nst == 0:
                    buf.copy_(self.mom1[c])
                elif n > 1:
                    self._sample(buf, self.mom1[c], self.mom2[c], L.VAR_WELFORD, float(n - 1))
                else:
                    self._sample(buf, self.mom1[c], None, L.VAR_GIVEN, 1.0)
                yield c

    def _evaluate_after(self, ep, loader):
        return self.sched.last_in_cycle(epoch=ep, batch=len(loader) - 1,
                                        batches_per_epoch=len(loader))

    def _extra_state(self):
        return {"samples_per_cycle": dict(self.samples_per_cycle), "mom1": dict(self.mom1),
                "mom2": dict(self.mom2), "epoch": self.sched.current_epoch}

    def _load_extra_state(self, d):
        self.samples_per_cycle = dict(d["samples_per_cycle"])
        self.mom1, self.mom2 = dict(d["mom1"]), dict(d["mom2"])
        self.sched.current_epoch = d["epoch"]

    def export_chain(self, k, epoch=None):
        """Chain k as a one-chain csghmc checkpoint (the keys of
        methods/csghmc.py:530-549 / bayesdll_amd.csghmc.Runner.save_ckpt, flat
        vectors in parameters_to_vector order): `torch.save` it and a
        Runner's load_ckpt takes it."""
        st, n1 = self.state, self.state.n1
        sl = (lambda v: v.view(self.K, st.stride)[k, :n1].clone())
        return {"last_theta": st.chain_vector(k).clone(),
                "cycle_theta_mom1": {c: sl(v) for c, v in self.mom1.items()},
                "cycle_theta_mom2": {c: sl(v) for c, v in self.mom2.items()},
                "cycle_likelihoods": {}, "cycle_states": {},
                "epoch": self.sched.current_epoch if epoch is None else epoch,
                "current_cycle": max(self.mom1) if self.mom1 else 0,
                "samples_per_cycle": dict(self.samples_per_cycle)}


class StackedSGLD(_StackedSampler):
    """K SGLD chains of `net` on one device (methods/sgld.py:69-250 per chain):
    sampler gradient g + (theta - theta0)/sigma^2/N + nd*sqrt(2/(N lr))*eps,
    then torch.optim.SGD(momentum=args.momentum) — one fused launch for all
    chains — with the running posterior moments (m1, m2) after burn-in every
    `thin` iterations fused into the same sweep.  `args` carries the sgld
    Runner's fields (lr, lr_head, epochs, momentum, ND, hparams with
    prior_sig, Ninflate, nd, burnin, thin, nst, bias; device); `net0` is the
    prior mean (zeros when None)."""

    need_prior = True
    tune_method = "sgld"

    def __init__(self, net, K_, args, **kw):
        super().__init__(net, K_, args, **kw)
        self.burnin = int(args.hparams["burnin"])
        self.mu = float(getattr(args, "momentum", 0.0))
        self.has_buffer = False
        self.bi = 0                      # global iteration count thinning uses
        self.m1 = self.m2 = None
        self.cnt = 0

    def update(self, grads, lrs, collect=None):
        """The fused SGLD + SGD(momentum mu) launch over all chains
        (methods/sgld.py:469-484 + :226), optional running-moment collect."""
        args, st = self.args, self.state
        st.use_grads(grads)
        N = args.ND * self.Ninflate
        ns = [self.nd * np.sqrt(2 / (N * v)) for v in lrs]
        mom = self.mu != 0
        ckind, m1, m2, ca, cb = (L.COLLECT_NONE, None, None, 1.0, 1.0) if collect is None \
            else collect
        K.sgmcmc_step(st, L.SGLD, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                      prior_sig=self.prior_sig, sigma2=self.prior_sig ** 2, n_data=N, mu=self.mu,
                      first_step=mom and not self.has_buffer, momentum=mom, collect=ckind,
                      mom1=m1, mom2=m2, collect_a=ca, collect_b=cb, seed=self.seed,
                      chain=self.chain0, step=self.step_count)
        self.has_buffer = self.has_buffer or mom
        self.step_count += 1

    def seed_moments(self):
        """methods/sgld.py:95-102 at the end of burn-in: m1 = theta,
        m2 = theta^2, count 1 (one stand-alone sweep over all chains)."""
        st = self.state
        self.m1 = torch.empty_like(st.theta)
        self.m2 = torch.empty_like(st.theta) if self.nst > 0 else None
        K.moments_update(st.theta, self.m1, self.m2, L.COLLECT_MEAN_INIT)
        self.cnt = 1

    def train_one_epoch(self, loader, epoch):
        args, dev = self.args, self.args.device
        self.net.train()
        if epoch == self.burnin:
            self.seed_moments()
        collect = epoch >= self.burnin
        lrs = (args.lr, args.lr_head)
        acc = self._new_acc()
        for x, y in loader:
            x, y = x.to(dev, non_blocking=True), y.to(dev, non_blocking=True)
            spec = None
            do_collect = collect and (self.bi + 1) % self.thin == 0
            if do_collect:  # methods/sgld.py:239-246
                spec = (L.COLLECT_MEAN, self.m1, self.m2, float(self.cnt), float(self.cnt + 1))
            loss, out = self.step(x, y, lrs, collect=spec)
            if do_collect:
                self.cnt += 1
            self.bi += 1
            self._accumulate(acc, loss, out, y)
        return self._epoch_result(acc)

    def _components(self, buf):
        """nst posterior draws, var = cnt/(cnt-1) * (m2 - m1^2) (1.0 for one
        sample; methods/sgld.py:324-350), or the posterior mean (nst = 0)."""
        if self.m1 is None:
            return
        for _ in range(max(1, self.nst)):
            if self.nst == 0:
                buf.copy_(self.m1)
            else:
                ratio = self.cnt / (self.cnt - 1) if self.cnt > 1 else 1.0
                self._sample(buf, self.m1, self.m2, L.VAR_RAW_MOMENTS, ratio)
            yield 0

    def _evaluate_after(self, ep, loader):
        freq = int(getattr(self.args, "test_eval_freq", 1) or 1)
        return ep >= self.burnin and ((ep + 1) % freq == 0 or ep + 1 == self.args.epochs)

    def _extra_state(self):
        return {"m1": self.m1, "m2": self.m2, "cnt": self.cnt, "bi": self.bi,
                "has_buffer": self.has_buffer}

    def _load_extra_state(self, d):
        self.m1, self.m2 = d["m1"], d["m2"]
        self.cnt, self.bi, self.has_buffer = d["cnt"], d["bi"], d["has_buffer"]


class StackedCSGLD(StackedSGLD):
    """K cyclical-SGLD chains (methods/csgld.py:195-331 per chain): SGLD + SGD
    momentum under the cyclical step size, per-cycle running moments
    (m1 = theta, m2 = theta^2 at a cycle's first sample, then the running
    mean) on the sample steps.  No burn-in; `args` as the csgld Runner's."""

    def __init__(self, net, K_, args, **kw):
        super().__init__(net, K_, args, **kw)
        self.burnin = -1  # cSGLD collects per cycle, not after a burn-in
        self.sched = CyclicalSGMCMC(base_lr=args.lr, nbr_of_cycles=getattr(args, "num_cycles", 10),
                                    epochs=args.epochs,
                                    proportion_exploration=getattr(args, "proportion_exploration",
                                                                   0.5))
        self.samples_per_cycle, self.mom1, self.mom2 = {}, {}, {}

    def train_one_epoch(self, loader, epoch):
        args, dev, sched = self.args, self.args.device, self.sched
        self.net.train()
        sched.current_epoch = epoch
        bpe = len(loader)
        acc = self._new_acc()
        st = self.state
        for b, (x, y) in enumerate(loader):
            x, y = x.to(dev, non_blocking=True), y.to(dev, non_blocking=True)
            lr = sched.calculate_lr(epoch=epoch, batch=b, batches_per_epoch=bpe)
            ss = sched.should_sample(epoch=epoch, batch=b, batches_per_epoch=bpe) \
                and b % self.thin == 0
            spec, c = None, None
            if ss:  # methods/csgld.py:280-293
                c = sched.get_cycle_number(epoch=epoch, batch=b, batches_per_epoch=bpe)
                if c not in self.mom1:
                    self.mom1[c] = torch.zeros_like(st.theta)
                    self.mom2[c] = torch.zeros_like(st.theta)
                    spec = (L.COLLECT_MEAN_INIT, self.mom1[c], self.mom2[c], 1.0, 1.0)
                else:
                    cc = self.samples_per_cycle.get(c, 0) + 1
                    spec = (L.COLLECT_MEAN, self.mom1[c], self.mom2[c], float(cc - 1), float(cc))
            loss, out = self.step(x, y, (lr, lr * (args.lr_head / args.lr)), collect=spec)
            if ss:
                self.samples_per_cycle[c] = self.samples_per_cycle.get(c, 0) + 1
            self._accumulate(acc, loss, out, y)
        return self._epoch_result(acc)

    def _components(self, buf):
        """Every collected cycle: nst draws with var = spc/(spc-1) * (m2 - m1^2)
        (ratio 1 for a one-sample cycle; methods/csgld.py:394-400), or its mean."""
        for c in sorted(self.mom1):
            spc = self.samples_per_cycle.get(c, 0)
            for _ in range(max(1, self.nst)):
                if self.nst == 0:
                    buf.copy_(self.mom1[c])
                else:
                    self._sample(buf, self.mom1[c], self.mom2[c], L.VAR_RAW_MOMENTS,
                                 spc / (spc - 1) if spc > 1 else 1.0)
                yield c

    def _evaluate_after(self, ep, loader):
        return self.sched.last_in_cycle(epoch=ep, batch=len(loader) - 1,
                                        batches_per_epoch=len(loader))

    def _extra_state(self):
        return {"samples_per_cycle": dict(self.samples_per_cycle), "mom1": dict(self.mom1),
                "mom2": dict(self.mom2), "has_buffer": self.has_buffer,
                "epoch": self.sched.current_epoch}

    def _load_extra_state(self, d):
        self.samples_per_cycle = dict(d["samples_per_cycle"])
        self.mom1, self.mom2 = dict(d["mom1"]), dict(d["mom2"])
        self.has_buffer, self.sched.current_epoch = d["has_buffer"], d["epoch"]


class StackedSGHMC(StackedSGLD):
    """K SGHMC chains (methods/sghmc.py:16-512 per chain): momentum
    v' = v(1-a) + lr-scaled sampler gradient with the prior pull and
    nd*sqrt(2a/(N lr)) noise, then SGD(momentum 0) on g + v' — one fused
    launch for all chains — and the SGLD Runner's burn-in / thinned running
    moments.  `args` as the sghmc Runner's (hparams with momentum_decay)."""

    def __init__(self, net, K_, args, **kw):
        super().__init__(net, K_, args, **kw)
        self.momentum_decay = float(args.hparams["momentum_decay"])
        self.mu = 0.0

    def update(self, grads, lrs, collect=None):
        args, st = self.args, self.state
        st.use_grads(grads)
        N = args.ND * self.Ninflate
        ns = [self.nd * np.sqrt(2 * self.momentum_decay / (N * v)) for v in lrs]
        ckind, m1, m2, ca, cb = (L.COLLECT_NONE, None, None, 1.0, 1.0) if collect is None \
            else collect
        K.sgmcmc_step(st, L.SGHMC, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                      one_minus_alpha=1 - self.momentum_decay, prior_sig=self.prior_sig,
                      sigma2=self.prior_sig ** 2, n_data=N, collect=ckind, mom1=m1, mom2=m2,
                      collect_a=ca, collect_b=cb, seed=self.seed, chain=self.chain0,
                      step=self.step_count)
        self.step_count += 1
