"""Runner pieces shared by the four drop-in samplers (host-side, off the hot path).

Mirrors the reference Runners' evaluation / bookkeeping API
(methods/csghmc.py:211-244, :387-670; methods/sgld.py:253-398) on top of the
flat device buffers:

  * posterior draws go through ONE fused kernel per draw (bdl_posterior_sample:
    theta_s = mean + sqrt(clamp(var)) * eps over the whole flat vector) written
    straight into the flat parameter buffer of an evaluation copy of the net,
    instead of nst x tensors-many torch ops (methods/sgld.py:292-296);
  * with several chains (torch.distributed initialised, one chain per GPU),
    the posterior-predictive average is one all_reduce(SUM) of per-chain
    predictive probabilities over RCCL — the only collective in the design.
"""
from __future__ import annotations

import copy
import os
import pickle

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib as L
from . import chains
from . import kernels as K
from .flat import bind_parameters, fill_normal_per_tensor

EVAL_STEP_BASE = 1 << 62  # Philox step keys for evaluation draws (never used by training)


class PosteriorDraw:
    """An evaluation copy of `net` whose flat theta the sample kernel fills."""

    def __init__(self, net, noise_mode, seed, chain, provider=None):
        self.net = copy.deepcopy(net)
        for p in self.net.parameters():
            p.grad = None
        self.theta = bind_parameters(self.net)
        self.numels = [p.numel() for p in self.net.parameters()]
        self.noise_mode = noise_mode
        self.seed = seed
        self.chain = chain
        self.count = 0
        self.noise = None if noise_mode == "philox" else torch.empty_like(self.theta)
        self.provider = provider
        if noise_mode == "external" and provider is None:
            raise RuntimeError("noise_mode='external' needs Model.noise_provider")

    def load_mean(self, mean):
        self.theta.copy_(mean)

    def draw(self, mean, m2, var_mode, ratio):
        """theta = mean + sqrt(clamp(var, 1e-12)) * eps; m2=None -> var = 1e-12."""
        noise = None
        if self.noise_mode == "torch":
            noise = fill_normal_per_tensor(self.noise, self.numels)
        elif self.noise_mode == "external":
            self.provider(-1 - self.count, self.noise)
            noise = self.noise
        K.posterior_sample(self.theta, mean, m2, var_mode=var_mode, ratio=ratio, noise=noise,
                           seed=self.seed, chain=self.chain, step=EVAL_STEP_BASE + self.count)
        self.count += 1


def defer_loss(runner):
    """Let the Runner's Model return device losses (no per-step host sync);
    BDL_SYNC_LOSS=1 restores the reference's per-step loss.item()."""
    runner.model.defer_loss = os.environ.get("BDL_SYNC_LOSS", "0") != "1"


def add_loss(acc, loss_, n):
    """acc + loss_ * n, the reference's float64 running sum (`loss += loss_ *
    len(y)`), kept on the device when loss_ is a device scalar: the same
    float64 operations in the same order, so float(acc) is the same number."""
    return acc + (loss_.double() if torch.is_tensor(loss_) else loss_) * n


def chain_world():
    return chains.world()


def check_divergence(runner, ep):
    """Once per epoch: did the sampler write a non-finite theta (or gradient)?
    The step kernels raise a device flag (bdl_step_args.nonfinite) instead of
    the host checking every step; the reference has no such guard and runs on
    with NaNs.  Logs a warning and records the epoch in runner.diverged_epochs."""
    st = runner.model.flat
    if st is not None and st.diverged():
        runner.diverged_epochs.append(ep)
        runner.logger.warning(f"[Epoch {ep}] the sampler wrote non-finite parameters: the chain "
                              "diverged (step size too large for the gradient scale?)")


def log_calibration(runner, targets_test, logits_test, targets_val=None, logits_val=None):
    """After a new best evaluation, as the reference Runners do
    (methods/csghmc.py:170-196, methods/sgld.py:160-186): ECE / MCE / NLL at
    T = 1 and at the temperature fitted on the validation set, with the
    reliability plots.  args.calibration = False skips it."""
    if not getattr(runner.args, "calibration", True):
        return None
    from .calibration import log_calibration as _log
    return _log(runner.args, runner.logger, targets_test, logits_test, targets_val, logits_val)


def log_update_stats(runner, ep):
    """BDL_STEP_TIMING=k: one log line per epoch with the fused update's
    launch count, sampled mean duration and algorithmic HBM GB/s."""
    st = runner.model.flat
    t = getattr(st, "timer", None) if st is not None else None
    if t is None:
        return None
    s = t.summary()
    if s.get("timed"):
        runner.logger.info(f"[Epoch {ep}] fused update: {s['launches']} launches, "
                           f"{s['avg_ms']:.4f} ms mean over {s['timed']} sampled, "
                           f"{s['gbs']:.1f} GB/s algorithmic ({100 * s['gbs'] / 8000.0:.1f} % of "
                           "8 TB/s HBM3E)")
    return s


def bind_chain_log_dir(args):
    """With several chains (one per rank) sharing a log_dir, every chain writes
    its checkpoints / logits / snapshots under <log_dir>/chain<rank> (the
    reference is single-chain, so its file names would collide).  One chain:
    unchanged."""
    if chains.world() > 1 and getattr(args, "log_dir", None) is not None \
            and not getattr(args, "_chain_dir_bound", False):
        args.log_dir = os.path.join(args.log_dir, f"chain{chains.rank()}")
        os.makedirs(args.log_dir, exist_ok=True)
        args._chain_dir_bound = True
    return args


def chain_average_logprob(logp):
    """Across-chain posterior-predictive average (bayesdll_amd.chains)."""
    return chains.average_predictive(logp)


def evaluate_point_estimate(runner, data_loader, net_to_evaluate):
    """methods/csghmc.py:211-244."""
    args = runner.args
    net_to_evaluate.eval()
    loss, error, nb = 0.0, 0, 0
    with torch.no_grad():
        for x, y in data_loader:
            x, y = x.to(args.device), y.to(args.device)
            out = net_to_evaluate(x)
            lb = runner.criterion(out, y)
            pred = out.data.max(dim=1)[1]
            loss += lb.item() * len(y)
            error += pred.ne(y.data).sum().item()
            nb += len(y)
    if nb == 0:
        return 0.0, 0.0
    return loss / nb, error / nb


def save_logits(args, targets, logits, logits_all, suffix=None):
    suffix = "" if suffix is None else f"_{suffix}"
    fname = os.path.join(args.log_dir, f"logits{suffix}.pkl")
    with open(fname, "wb") as ff:
        pickle.dump({"targets": targets, "logits": logits, "logits_all": logits_all}, ff,
                    protocol=pickle.HIGHEST_PROTOCOL)
    return fname


def load_checkpoint(path, device):
    """torch.load with weights_only=True plus the numpy types the reference's
    checkpoints contain (cycle_likelihoods are np.ndarray, methods/csghmc.py:377):
    nothing from the file is executed."""
    import numpy as _np
    from torch.serialization import safe_globals
    allowed = [_np.ndarray, _np.dtype, _np._core.multiarray._reconstruct]
    allowed += [getattr(_np.dtypes, n) for n in ("Float64DType", "Float32DType", "Int64DType")
                if hasattr(_np.dtypes, n)]
    with safe_globals(allowed):
        return torch.load(path, map_location=device, weights_only=True)


def _sampler_indices(loader):
    """The sample indices one pass of `loader` scores, as a sorted list —
    defined only for samplers that visit a fixed set of samples once each:
    SequentialSampler, RandomSampler without replacement over the whole data
    set, SubsetRandomSampler (its subset).  Any other sampler (weighted, with
    replacement, num_samples != len) draws a rank-dependent multiset, which
    shards cannot partition: ValueError."""
    from torch.utils.data import RandomSampler, SequentialSampler, SubsetRandomSampler
    s, n = loader.sampler, len(loader.dataset)
    if isinstance(s, SequentialSampler):
        return list(range(n))
    if isinstance(s, RandomSampler):
        if s.replacement or s.num_samples != n:
            raise ValueError("a sharded likelihood pass needs a RandomSampler without replacement "
                             "over the whole data set (num_samples == len(dataset))")
        return list(range(n))
    if isinstance(s, SubsetRandomSampler):
        return sorted(int(i) for i in s.indices)
    raise ValueError(f"a sharded likelihood pass cannot partition a {type(s).__name__}: "
                     "use a sequential, random (no replacement) or subset-random sampler")


def shard_loader(loader, r, k):
    """Shard r of k of a training loader for a data-parallel likelihood pass,
    split by SAMPLE index so that the k shards partition the samples the
    loader visits whatever order each rank's loader would draw (the
    reference's train loader shuffles, datasets.py:45-46, and every chain
    seeds its own generator):
      * a torch DataLoader over a map-style data set: a DataLoader over every
        k-th sample (from r) of the sorted index list its sampler visits
        (_sampler_indices: the whole set, or a SubsetRandomSampler's subset),
        with the loader's batch size, collate_fn, workers and their settings,
        pinning and timeout; no shuffling — the loss sum does not depend on
        the order;
      * a list / tuple of batches (identical on every rank): the batches whose
        index is r mod k;
    anything else (an iterable data set, a custom batch sampler, a sampler
    with replacement or weights, drop_last — which drops samples that depend
    on the shuffle) is refused."""
    if k == 1:
        return loader
    from torch.utils.data import DataLoader, IterableDataset, Subset
    if isinstance(loader, DataLoader):
        ds = loader.dataset
        if isinstance(ds, IterableDataset) or not hasattr(ds, "__len__"):
            raise ValueError("a sharded likelihood pass needs a map-style data set")
        if loader.batch_size is None:
            raise ValueError("a sharded likelihood pass needs a DataLoader with a batch_size "
                             "(not a custom batch_sampler)")
        if loader.drop_last:
            raise ValueError("a sharded likelihood pass cannot reproduce drop_last (which samples "
                             "are dropped depends on each rank's shuffle)")
        idx = _sampler_indices(loader)[r::k]
        kw = dict(batch_size=loader.batch_size, shuffle=False, num_workers=loader.num_workers,
                  collate_fn=loader.collate_fn, pin_memory=loader.pin_memory,
                  timeout=loader.timeout, worker_init_fn=loader.worker_init_fn)
        if loader.num_workers > 0:
            kw.update(persistent_workers=loader.persistent_workers,
                      prefetch_factor=loader.prefetch_factor,
                      multiprocessing_context=loader.multiprocessing_context)
        return DataLoader(Subset(ds, idx), **kw)
    if isinstance(loader, (list, tuple)):
        return [b for i, b in enumerate(loader) if i % k == r]
    raise ValueError(f"a sharded likelihood pass needs a DataLoader or a list of batches, "
                     f"got {type(loader).__name__}")


def loss_sums(net, loader, criterion, device, shard=(0, 1)):
    """Sum of per-batch mean loss x batch size over `loader` (the reference's
    `loss += loss_.item() * len(y)`, methods/csghmc.py:620-627), accumulated
    on the device in float64 — the same float64 operations in the same order,
    without a host synchronisation per batch.  shard=(r, k): only shard r of
    k of the loader is scored (shard_loader).  Returns (device float64 sum,
    count)."""
    r, k = shard
    acc = torch.zeros((), dtype=torch.float64, device=device)
    nb = 0
    for x, y in shard_loader(loader, r, k):
        x, y = x.to(device), y.to(device)
        acc = add_loss(acc, criterion(net(x), y), len(y))
        nb += len(y)
    return acc, nb


def _group_rank_size(group):
    import torch.distributed as dist
    return dist.get_rank(group), dist.get_world_size(group)


def _check_same_posterior(group, device, *vecs):
    """Sharded scoring needs the same Gaussian on every rank of the group:
    compare float64 checksums (all_reduce MIN and MAX); raise if they differ."""
    cs = torch.stack([v.double().sum() if v is not None else torch.zeros((), dtype=torch.float64,
                                                                         device=device)
                      for v in vecs]).reshape(-1)
    lo, hi = _reduce_in(cs.clone(), "min", group), _reduce_in(cs.clone(), "max", group)
    if not torch.equal(lo, hi):
        raise ValueError("full_batch_likelihoods(group=...): the ranks of the group hold different "
                         "posterior moments; a sharded pass needs the same mean / variance on every "
                         "rank (replicas of one chain, or chains.pool_moments)")


def _reduce_in(t, op, group):
    import torch.distributed as dist
    o = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op]
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=o, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=o, group=group)
    return t


def full_batch_likelihoods(runner, train_loader, mean, m2, var_mode, ratio, theta, group=None):
    """methods/csghmc.py:568-638 (csgld.py:508-594, adam_csghmc.py:629-...):
    max(1, nst) posterior draws theta_s = mean + sqrt(var) * eps (one fused
    kernel each; nst = 0: the current theta), each scored on the full
    training set; returns [exp(-average loss)] per draw.

    group (a torch.distributed process group, or dist.group.WORLD): a
    data-parallel pass — every rank of the group draws the SAME samples (the
    group's first rank's Philox key; the moments — with nst = 0 the current
    theta — must agree, checked) and scores only its shard of the training
    set, split by sample index (shard_loader); ONE all_reduce of the
    [draws, 2] float64 (loss sum, count) table combines them.  The loss sums
    equal the single-process ones up to the float64 summation order (and the
    per-batch float32 means, whose batches differ)."""
    import torch.distributed as dist
    device = runner.args.device
    model = runner.model
    seed, chain = model.seed, model.chain
    shard = (0, 1)
    if group is not None:
        if model.noise_mode != "philox":
            raise ValueError("a sharded likelihood pass needs noise_mode='philox' (the draws must "
                             "be a function of the group's common key)")
        shard = _group_rank_size(group)
        # nst = 0 scores the current theta: it must be the same on every rank too
        _check_same_posterior(group, mean.device, mean, m2, theta if runner.nst == 0 else None)
        key = torch.tensor([seed & ((1 << 63) - 1), chain], dtype=torch.int64,
                           device=mean.device)
        src = dist.get_global_rank(group, 0) if group is not dist.group.WORLD else 0
        if key.is_cuda and dist.get_backend(group) == "gloo":
            h = key.cpu()
            dist.broadcast(h, src=src, group=group)
            key.copy_(h)
        else:
            dist.broadcast(key, src=src, group=group)
        seed, chain = int(key[0]), int(key[1])
    draw = PosteriorDraw(runner.net, model.noise_mode, seed, chain, model.noise_provider)
    ndraw = max(1, runner.nst)
    table = torch.zeros(ndraw, 2, dtype=torch.float64, device=mean.device)
    draw.net.eval()
    with torch.no_grad():
        for s in range(ndraw):
            if runner.nst > 0:
                draw.draw(mean, m2, var_mode, ratio)
            else:
                draw.theta.copy_(theta)
            acc, nb = loss_sums(draw.net, train_loader, runner.criterion, device, shard)
            table[s, 0] = acc
            table[s, 1] = nb
    if group is not None:
        _reduce_in(table, "sum", group)
    out = []
    for s, (tot, nb) in enumerate(table.tolist()):
        avg = tot / nb
        out.append(np.exp(-avg))
        runner.logger.info(f"Sample {s + 1} - Full batch average loss: {avg:.6f}, "
                           f"likelihood: {np.exp(-avg):.6e}")
    return out


def gmm_weights(cycle_likelihoods):
    """methods/csghmc.py:641-670: w_c = 1 / mean(1/lik), normalised."""
    if not cycle_likelihoods:
        return {0: 1.0}
    w = {c: 1.0 / np.mean([1.0 / lk for lk in liks]) for c, liks in cycle_likelihoods.items()}
    tot = sum(w.values())
    if tot > 0:
        return {c: v / tot for c, v in w.items()}
    return {c: 1.0 / len(w) for c in w}


def mixture_evaluate(runner, test_loader, var_of_cycle):
    """Cyclical methods' GMM predictive (methods/csghmc.py:387-514,
    methods/csgld.py:337-452).  var_of_cycle(c) -> (m2, var_mode, ratio)."""
    args = runner.args
    chain_w = None
    if chain_world() > 1 and getattr(runner, "gmm_over_chains", False):
        # the ensemble's components are every chain's cycles, weighted jointly
        weights, chain_w, joint = chains.chain_gmm_weights(runner.cycle_likelihoods)
        runner.logger.info(f"GMM component weights over chains: {joint}")
    else:
        weights = runner.calculate_gmm_weights()
        runner.logger.info(f"GMM component weights: {weights}")
    model = runner.model
    draw = PosteriorDraw(runner.net, model.noise_mode, model.seed, model.chain,
                         model.noise_provider)
    loss, error, nb = 0.0, 0, 0
    targets, logits, logits_all = [], [], []
    draw.net.eval()
    with torch.no_grad():
        for x, y in test_loader:
            x, y = x.to(args.device), y.to(args.device)
            comp_all, batch_logits = [], None
            for cycle in runner.cycle_theta_mom1.keys():
                weight = weights.get(cycle, 0.0)
                if weight < 1e-10:
                    continue
                mean = runner.cycle_theta_mom1[cycle]
                outs = []
                if runner.nst == 0:
                    draw.load_mean(mean)
                    outs.append(draw.net(x))
                else:
                    m2, var_mode, ratio = var_of_cycle(cycle)
                    for _ in range(runner.nst):
                        draw.draw(mean, m2, var_mode, ratio)
                        outs.append(draw.net(x))
                comp = torch.stack(outs, dim=2)
                if runner.nst == 0:
                    comp_out = comp.squeeze(2)
                else:
                    comp_out = F.log_softmax(comp, dim=1).logsumexp(-1) - np.log(runner.nst)
                comp_all.append(comp)
                batch_logits = weight * comp_out if batch_logits is None else \
                    batch_logits + weight * comp_out
            comp_all = torch.stack(comp_all, dim=3) if comp_all else torch.zeros(
                (x.size(0), args.num_classes, 1, 1), device=x.device)
            if batch_logits is None:  # no cycle collected yet
                batch_logits = draw.net(x)
            if chain_world() > 1:
                batch_logits = chains.average_predictive(batch_logits, chain_w)
            lb = runner.criterion(batch_logits, y)
            pred = batch_logits.data.max(dim=1)[1]
            targets.append(y.cpu().numpy())
            logits.append(batch_logits.cpu().numpy())
            logits_all.append(comp_all.cpu().numpy())
            loss += lb.item() * len(y)
            error += pred.ne(y.data).sum().item()
            nb += len(y)
    return (loss / nb, error / nb, np.concatenate(targets, 0), np.concatenate(logits, 0),
            np.concatenate(logits_all, 0))


def sample_average_evaluate(runner, test_loader, mean, m2, var_mode, ratio):
    """sgld/sghmc predictive: average over nst posterior draws
    (methods/sgld.py:253-321), across chains via chain_average_logprob."""
    args = runner.args
    model = runner.model
    draw = PosteriorDraw(runner.net, model.noise_mode, model.seed, model.chain,
                         model.noise_provider)
    draw.net.eval()
    loss, error, nb = 0.0, 0, 0
    targets, logits, logits_all = [], [], []
    with torch.no_grad():
        for x, y in test_loader:
            x, y = x.to(args.device), y.to(args.device)
            outs = []
            if runner.nst == 0:
                draw.load_mean(mean)
                outs.append(draw.net(x))
                la = torch.stack(outs, 2)
                lg = F.log_softmax(la, 1).logsumexp(-1)
            else:
                for _ in range(runner.nst):
                    draw.draw(mean, m2, var_mode, ratio)
                    outs.append(draw.net(x))
                la = torch.stack(outs, 2)
                lg = F.log_softmax(la, 1).logsumexp(-1) - np.log(runner.nst)
            if chain_world() > 1:
                lg = chain_average_logprob(lg)
            lb = runner.criterion(lg, y)
            pred = lg.data.max(dim=1)[1]
            targets.append(y.cpu().numpy())
            logits.append(lg.cpu().numpy())
            logits_all.append(la.cpu().numpy())
            loss += lb.item() * len(y)
            error += pred.ne(y.data).sum().item()
            nb += len(y)
    return (loss / nb, error / nb, np.concatenate(targets, 0), np.concatenate(logits, 0),
            np.concatenate(logits_all, 0))


__all__ = ["PosteriorDraw", "chain_average_logprob", "evaluate_point_estimate", "save_logits",
           "gmm_weights", "mixture_evaluate", "sample_average_evaluate", "L"]


def reinit_network(net):
    """Cold restart (methods/adam_csghmc.py:102-117, methods/csghmc_fs.py:93-117):
    fresh random weights per layer type — Xavier-uniform Linear, Kaiming-uniform
    (fan_in, ReLU) Conv2d, zero biases, unit/zero BatchNorm affine, else the
    module's own reset_parameters().  In place, so parameters that are views
    into a sampler's flat theta stay bound to it."""
    import torch.nn as nn

    def init(m):
        if isinstance(m, nn.Linear):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Conv2d):
            nn.init.kaiming_uniform_(m.weight, mode="fan_in", nonlinearity="relu")
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, (nn.BatchNorm2d, nn.BatchNorm1d)):
            if m.weight is not None:
                nn.init.ones_(m.weight)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif hasattr(m, "reset_parameters"):
            m.reset_parameters()

    with torch.no_grad():
        net.apply(init)


def resume_state(model, st, sgd=None, **counters):
    """What an exact continuation of a chain needs beyond the reference's
    checkpoint keys: the momentum / SGD buffer, further per-element sampler
    state (Adam m / v, its SGD buffer), the sampler's step counter (the Philox
    noise key) and Adam's t, host counters, and the torch RNG states (the
    "torch" noise mode draws from them)."""
    out = {"mom": None if st.mom is None else st.mom.detach().clone(),
           "extra": {k: v.detach().clone() for k, v in getattr(st, "extra", {}).items()},
           "step_count": int(model.step_count), "seed": int(model.seed),
           "chain": int(model.chain), "t": getattr(model, "t", None),
           "sgd_has_buffer": None if sgd is None else bool(sgd.has_buffer),
           "rng_cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        out["rng_cuda"] = torch.cuda.get_rng_state(st.device)
    out.update(counters)
    return out


def restore_resume_state(model, st, ckpt, sgd=None):
    """Inverse of resume_state (plus theta from the checkpoint's last_theta —
    a flat vector for the cyclical methods, a state_dict for sgld / sghmc),
    in place so the parameter and gradient views stay bound."""
    rs = ckpt.get("resume")
    if rs is None:
        raise RuntimeError("checkpoint has no resume state (save it with args.resume_state=True)")
    last = ckpt["last_theta"]
    if isinstance(last, dict):
        last = torch.cat([last[nm].reshape(-1).to(st.theta.device) for nm in st.names])
    with torch.no_grad():
        st.theta.copy_(last.reshape(-1).to(st.theta.device))
        if rs.get("mom") is not None and st.mom is not None:
            st.mom.copy_(rs["mom"].to(st.mom.device))
        for k, v in rs.get("extra", {}).items():
            st.extra[k].copy_(v.to(st.extra[k].device))
    model.step_count = int(rs["step_count"])
    model.seed = int(rs["seed"])
    model.chain = int(rs["chain"])
    if rs.get("t") is not None:
        model.t = int(rs["t"])
    if sgd is not None and rs.get("sgd_has_buffer") is not None:
        sgd.has_buffer = bool(rs["sgd_has_buffer"])
    torch.set_rng_state(rs["rng_cpu"].cpu())
    if "rng_cuda" in rs and torch.cuda.is_available():
        torch.cuda.set_rng_state(rs["rng_cuda"].cpu(), st.device)
    skip = ("mom", "extra", "step_count", "seed", "chain", "t", "sgd_has_buffer", "rng_cpu",
            "rng_cuda")
    return {k: v for k, v in rs.items() if k not in skip}
