"""Cycle-end likelihood pass and GMM weights over chains on
CPU with torch.distributed gloo, world_size 2 and 3 — host logic only (the
posterior draws themselves are HIP kernels; tests/test_gpu_chains.py runs the
Runner path on the device).

  * _runner.loss_sums: the reference's `loss += loss_.item() * len(y)`
    (methods/csghmc.py:620-627) accumulated in float64 without a sync per
    batch — bit-identical to the per-batch .item() loop in one process;
    sharded over ranks by batch index and all-reduced, equal to it up to the
    float64 summation order (rtol 1e-12), ragged last batch included;
  * chains.chain_gmm_weights: w = 1 / mean(1 / lik) per (chain, cycle)
    (methods/csghmc.py:641-670), normalised over every chain's cycles;
  * chains.average_predictive(weight=W_k): log(sum_k W_k softmax(s_k)).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _net():
    torch.manual_seed(3)
    return nn.Sequential(nn.Flatten(), nn.Linear(20, 16), nn.ReLU(), nn.Linear(16, 5))


def _loader():
    g = torch.Generator().manual_seed(9)
    x = torch.randn(103, 20, generator=g)
    y = torch.randint(0, 5, (103,), generator=g)
    return [(x[i:i + 16], y[i:i + 16]) for i in range(0, 103, 16)]  # 7 batches, last of 7


def _shuffled_loader(r):
    """The reference's training loader shape (datasets.py:45-46: shuffle=True),
    with a RANK-DEPENDENT shuffle, as chains seeded per rank would draw it."""
    g = torch.Generator().manual_seed(9)
    x = torch.randn(103, 20, generator=g)
    y = torch.randint(0, 5, (103,), generator=g)
    return torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, y), batch_size=16,
                                       shuffle=True,
                                       generator=torch.Generator().manual_seed(1000 + r))


def _likelihoods(r):
    # rank-dependent cycle likelihoods (chain r has r + 1 cycles)
    return {c: np.array([0.2 + 0.1 * r + 0.05 * c, 0.3 + 0.02 * c]) for c in range(1, r + 2)}


def _worker(r, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    from bayesdll_amd import _runner as R
    from bayesdll_amd import chains
    dist.init_process_group("gloo", rank=r, world_size=world)
    try:
        net, crit = _net(), nn.CrossEntropyLoss()
        with torch.no_grad():
            acc, nb = R.loss_sums(net, _loader(), crit, "cpu", shard=(r, world))
            acc2, nb2 = R.loss_sums(net, _shuffled_loader(r), crit, "cpu", shard=(r, world))
        t = torch.tensor([float(acc), float(nb), float(acc2), float(nb2)], dtype=torch.float64)
        dist.all_reduce(t)
        within, chain_w, joint = chains.chain_gmm_weights(_likelihoods(r))
        g = torch.Generator().manual_seed(50 + r)
        scores = torch.randn(6, 5, generator=g) * 4.0
        avg = chains.average_predictive(scores, chain_w)
        q.put((r, t.tolist(), within, chain_w, {f"{k[0]},{k[1]}": v for k, v in joint.items()},
               scores.numpy().copy(), avg.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_loss_sums_and_gmm_weights_over_chains(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=120)
        res[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    # single process, the reference's loop: loss += loss_.item() * len(y)
    net, crit = _net(), nn.CrossEntropyLoss()
    ref, nb = 0.0, 0
    with torch.no_grad():
        for x, y in _loader():
            ref += crit(net(x), y).item() * len(y)
            nb += len(y)
    from bayesdll_amd import _runner as R
    with torch.no_grad():
        acc, n1 = R.loss_sums(net, _loader(), crit, "cpu")
    assert float(acc) == ref and n1 == nb == 103  # same float64 ops, same order
    # per-sample losses, for the shuffled loaders whose batches differ by rank
    with torch.no_grad():
        x = torch.cat([b[0] for b in _loader()])
        y = torch.cat([b[1] for b in _loader()])
        per_sample = nn.CrossEntropyLoss(reduction="sum")(net(x).double(), y).item()
    for r in range(world):
        tot, cnt, tot2, cnt2 = res[r][0]
        assert cnt == 103 and cnt2 == 103  # every sample scored exactly once
        np.testing.assert_allclose(tot, ref, rtol=1e-12)
        np.testing.assert_allclose(tot2, per_sample, rtol=1e-6)  # fp32 batch means

    # joint GMM weights over every chain's cycles
    raw = {(r, c): 1.0 / np.mean(1.0 / lk) for r in range(world)
           for c, lk in _likelihoods(r).items()}
    tot = sum(raw.values())
    for r in range(world):
        within, chain_w, joint = res[r][1], res[r][2], res[r][3]
        assert set(joint) == {f"{a},{c}" for a, c in raw}
        for (a, c), v in raw.items():
            np.testing.assert_allclose(joint[f"{a},{c}"], v / tot, rtol=1e-12)
        np.testing.assert_allclose(sum(joint.values()), 1.0, rtol=1e-12)
        want_w = sum(v for (a, _), v in raw.items() if a == r) / tot
        np.testing.assert_allclose(chain_w, want_w, rtol=1e-12)
        np.testing.assert_allclose(sum(within.values()), 1.0, rtol=1e-12)
        for c, v in within.items():
            np.testing.assert_allclose(v, raw[(r, int(c))] / tot / want_w, rtol=1e-12)

    # weighted ensemble predictive: log(sum_k W_k softmax(s_k))
    mix = sum(res[r][2] * torch.softmax(torch.from_numpy(res[r][4]).double(), 1)
              for r in range(world))
    for r in range(world):
        np.testing.assert_allclose(res[r][5], torch.log(mix).numpy(), rtol=1e-5, atol=1e-6)


def test_single_chain_gmm_weights_match_the_reference_formula():
    from bayesdll_amd import _runner as R
    from bayesdll_amd import chains
    lik = _likelihoods(1)
    within, chain_w, joint = chains.chain_gmm_weights(lik)
    ref = R.gmm_weights(lik)
    assert chain_w == pytest.approx(1.0)
    for c in lik:
        assert within[c] == pytest.approx(ref[c], rel=1e-12)
        assert joint[(0, c)] == pytest.approx(ref[c], rel=1e-12)


def test_shard_loader_partitions_samples_and_refuses_what_it_cannot_split():
    from bayesdll_amd._runner import shard_loader
    dl = _shuffled_loader(0)
    seen = []
    for r in range(3):
        for x, _ in shard_loader(dl, r, 3):
            seen.extend(x[:, 0].tolist())
    allx = torch.cat([b[0] for b in _loader()])[:, 0].tolist()
    assert sorted(seen) == sorted(allx)
    assert shard_loader(dl, 0, 1) is dl
    assert len(shard_loader(_loader(), 1, 3)) == 2  # batches 1, 4 of 7
    ds = dl.dataset
    with pytest.raises(ValueError, match="drop_last"):
        shard_loader(torch.utils.data.DataLoader(ds, batch_size=16, drop_last=True), 0, 2)
    with pytest.raises(ValueError, match="DataLoader or a list"):
        shard_loader(iter(_loader()), 0, 2)


def test_shard_loader_follows_the_loaders_sampler():
    """A SubsetRandomSampler's shards partition ITS subset (not the whole data
    set); samplers that draw a multiset (with replacement, weighted) are
    refused; worker settings carry over."""
    from torch.utils.data import (DataLoader, RandomSampler, SubsetRandomSampler,
                                  WeightedRandomSampler)

    from bayesdll_amd._runner import shard_loader
    ds = _shuffled_loader(0).dataset
    subset = list(range(5, len(ds), 3))
    dl = DataLoader(ds, batch_size=8, sampler=SubsetRandomSampler(subset),
                    worker_init_fn=print, timeout=0)
    seen = []
    for r in range(2):
        sh = shard_loader(dl, r, 2)
        assert sh.worker_init_fn is print
        for x, _ in sh:
            seen.extend(x[:, 0].tolist())
    want = [float(ds[i][0][0]) for i in subset]
    assert sorted(seen) == sorted(want)
    with pytest.raises(ValueError, match="without replacement"):
        shard_loader(DataLoader(ds, batch_size=8, sampler=RandomSampler(ds, replacement=True)),
                     0, 2)
    with pytest.raises(ValueError, match="num_samples"):
        shard_loader(DataLoader(ds, batch_size=8, sampler=RandomSampler(ds, num_samples=10)),
                     0, 2)
    with pytest.raises(ValueError, match="WeightedRandomSampler"):
        shard_loader(DataLoader(ds, batch_size=8,
                                sampler=WeightedRandomSampler([1.0] * len(ds), len(ds))), 0, 2)
