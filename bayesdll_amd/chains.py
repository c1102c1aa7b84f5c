"""Independent-chain ensemble across GPUs (one chain per process / GPU).

The reference runs a single chain on a single device (methods/csghmc.py:41).
Chains are independent Markov chains, so sampling shards with NO
communication: each rank owns a full chain (theta, v, moments resident in its
own HBM) keyed by its rank (Philox chain id; seed = base + rank).

The only exchange is at evaluation: the posterior-predictive average over
chains.  Per batch, each rank holds its chain's predictive scores ([B, C]: the
log-mean-exp over its own nst draws, methods/sgld.py:300, or the csghmc
mixture's weighted scores, methods/csghmc.py:470-480, which the reference
feeds to the loss as logits); the ensemble predictive is
log((1/K) sum_k softmax(s_k)), computed stably as a log-mean-exp over ranks:
all_reduce(MAX) of log_softmax(s_k) for the shift, then all_reduce(SUM) of
exp(log_softmax(s_k) - max) over RCCL (backend "nccl" on ROCm; "gloo" on CPU
for tests).  Messages are B x C fp32 (512 KB at B=128, C=1000): latency-bound,
far below one xGMI link, so no bucketing is needed.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def is_distributed():
    return dist.is_available() and dist.is_initialized()


def world():
    return dist.get_world_size() if is_distributed() else 1


def rank():
    return dist.get_rank() if is_distributed() else 0


def init_chains(backend=None):
    """Initialise one chain per process from torchrun's env (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT).  Returns (rank, world, device)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if ws > 1 and not is_distributed():
        backend = backend or ("nccl" if device.type == "cuda" else "gloo")
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return rank(), world(), device


def _all_reduce(t, op=dist.ReduceOp.SUM):
    """all_reduce in place.  gloo (CPU tests, ranks sharing one GPU) is fed a
    host copy of a device tensor; RCCL ("nccl") reduces on the device."""
    if t.is_cuda and dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)
    return t


def _all_reduce_sum(t):
    return _all_reduce(t, dist.ReduceOp.SUM)


def chain_seed(base_seed):
    """Per-chain seed: base + rank (each chain its own Philox key)."""
    return int(base_seed) + rank()


def average_predictive(scores, weight=None):
    """Ensemble predictive over the K chains: log(sum_k w_k softmax(s_k)), per
    class, with w_k = 1/K (weight=None) or this chain's weight (weights summing
    to 1 over the chains, e.g. chain_gmm_weights).  Each chain's scores are
    normalised first (log_softmax: the csghmc mixture's weighted logits are
    not log-probabilities, and chains may differ in logit scale), then a
    max-shifted log-sum-exp over ranks — no overflow for large logits, no -inf
    for classes every chain finds unlikely.  One process: the scores are
    returned unchanged (the reference's single-chain evaluation)."""
    k = world()
    if k == 1:
        return scores
    lp = torch.log_softmax(scores.float(), dim=1)
    if weight is not None:
        if weight <= 0:  # this chain contributes nothing; exp(-inf) = 0 below
            lp = torch.full_like(lp, float("-inf"))
        else:
            lp = lp + float(np.log(weight))
    shift = _all_reduce(lp.clone(), dist.ReduceOp.MAX)
    s = _all_reduce_sum((lp - shift).exp())
    return shift + (s if weight is not None else s / k).log()


def gather_objects(obj):
    """all_gather of a small picklable host object (one per rank, rank order)."""
    if world() == 1:
        return [obj]
    out = [None] * world()
    dist.all_gather_object(out, obj)
    return out


def chain_gmm_weights(cycle_likelihoods):
    """calculate_gmm_weights over chains: the reference's
    per-cycle weight w_c = 1 / mean(1 / lik) (methods/csghmc.py:641-670),
    computed for every (chain, cycle) component of the ensemble and
    normalised jointly — a chain whose cycles explain the training data better
    weighs more in the ensemble predictive.  One all_gather of the chains'
    likelihood lists (a few floats each).  Returns (within, chain_w, joint):
    this chain's cycle weights normalised within the chain (what its own
    mixture uses), this chain's total weight W_k (sum over its cycles, the
    weight for average_predictive), and {(rank, cycle): w} for all chains."""
    mine = {int(c): [float(v) for v in np.atleast_1d(lk)] for c, lk in cycle_likelihoods.items()}
    every = gather_objects(mine)
    raw = {(r, c): 1.0 / np.mean([1.0 / v for v in liks])
           for r, d in enumerate(every) for c, liks in d.items()}
    tot = sum(raw.values())
    if not raw or not tot > 0:  # no cycle scored anywhere: uniform over chains
        joint = {k: 1.0 / len(raw) for k in raw} if raw else {}
        return ({c: 1.0 / len(mine) for c in mine} if mine else {0: 1.0}), 1.0 / world(), joint
    joint = {k: v / tot for k, v in raw.items()}
    r = rank()
    chain_w = sum(v for (rr, _), v in joint.items() if rr == r)
    within = {c: (joint[(r, c)] / chain_w if chain_w > 0 else 1.0 / len(mine)) for c in mine} \
        if mine else {0: 1.0}
    return within, chain_w, joint


def gather_logits(logits_all):
    """All-gather per-chain sample logits [B, C, S] into [B, C, S*K] (the
    reference's logits_all layout with every chain's samples, rank-major)."""
    k = world()
    if k == 1:
        return logits_all
    src = logits_all.contiguous()
    host = src.is_cuda and dist.get_backend() == "gloo"
    if host:
        src = src.cpu()
    parts = [torch.empty_like(src) for _ in range(k)]
    dist.all_gather(parts, src)
    out = torch.cat(parts, dim=2)
    return out.to(logits_all.device) if host else out


def pool_moments(mom1, mom2=None, count=1.0):
    """Pool the chains' posterior moments into one Gaussian (the
    optional cross-chain posterior average).  Each chain contributes its
    running mean m1 and raw second moment m2 (or Welford-free moments of any
    kind that average linearly) weighted by its sample count:

        m = sum_k c_k m_k / sum_k c_k

    One all_reduce(SUM) of c_k * m_k per vector over RCCL / xGMI (a ViT-L/32
    mean is 1.2 GB: bandwidth-bound, ring-chunked by RCCL) plus one scalar
    all_reduce for the counts.  Returns new tensors; inputs are unchanged."""
    k = world()
    c = float(count)
    if k == 1:
        return mom1.clone(), (None if mom2 is None else mom2.clone())
    tot = torch.tensor([c], dtype=torch.float64, device=mom1.device)
    _all_reduce_sum(tot)
    scale = c / float(tot.item())
    out = []
    for m in (mom1, mom2):
        if m is None:
            out.append(None)
            continue
        w = _all_reduce_sum(m * scale)
        out.append(w)
    return out[0], out[1]
