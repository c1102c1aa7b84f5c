"""Multi-chain logic on CPU with torch.distributed gloo, world_size 2, 4 and 8
(stands in for RCCL over xGMI: the same all_reduce / all_gather calls; 8 = config
5's chain count)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(r, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    from bayesdll_amd import chains
    from bayesdll_amd._base import default_chain
    dist.init_process_group("gloo", rank=r, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + r)
        logits = torch.randn(8, 5, generator=g)
        logp = torch.log_softmax(logits, 1)
        avg = chains.average_predictive(logp)
        la = torch.randn(8, 5, 3, generator=g)
        gathered = chains.gather_logits(la)
        m1, m2 = torch.randn(1000, generator=g), torch.rand(1000, generator=g)
        p1, p2 = chains.pool_moments(m1, m2, count=r + 1)
        # nst = 0 mixture scores: weighted raw logits of a large scale (exp overflows
        # fp32 above ~88; every chain puts a class below exp's underflow)
        big = torch.randn(8, 5, generator=g) * 300.0
        big[:, 4] = -5000.0
        avg_big = chains.average_predictive(big)
        # plain numpy over the queue: a torch tensor would travel as a shared-memory
        # fd the parent may open only after this worker has exited
        np_ = lambda t: t.numpy().copy()
        q.put((r, np_(logp), np_(avg), np_(la), np_(gathered), default_chain(),
               chains.chain_seed(42), tuple(np_(t) for t in (m1, m2, p1, p2)),
               (np_(big), np_(avg_big))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_average_predictive_and_gather_chains(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, logp, avg, la, gathered, chain, seed, mom, big = q.get(timeout=120)
        t = torch.from_numpy
        res[r] = (t(logp), t(avg), t(la), t(gathered), chain, seed, tuple(t(m) for m in mom),
                  (t(big[0]), t(big[1])))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = torch.log(sum(res[r][0].exp() for r in range(world)) / world)
    for r in range(world):
        torch.testing.assert_close(res[r][1], want)
        torch.testing.assert_close(res[r][3], torch.cat([res[k][2] for k in range(world)], dim=2))
        assert res[r][4] == r            # Philox chain id = rank
        assert res[r][5] == 42 + r       # per-chain seed
    # pooled moments: count-weighted average of the chains' moments
    cnt = [r + 1 for r in range(world)]
    want1 = sum(c * res[r][6][0].double() for r, c in enumerate(cnt)) / sum(cnt)
    want2 = sum(c * res[r][6][1].double() for r, c in enumerate(cnt)) / sum(cnt)
    for r in range(world):
        torch.testing.assert_close(res[r][6][2].double(), want1, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(res[r][6][3].double(), want2, rtol=1e-6, atol=1e-6)
    # the averaged predictive is a proper distribution
    torch.testing.assert_close(want.exp().sum(1), torch.ones(8))
    # large / very negative scores: finite, and equal to the float64 log-mean of softmaxes
    want_big = torch.logsumexp(torch.stack(
        [torch.log_softmax(res[r][7][0].double(), 1) for r in range(world)]), 0) - np.log(world)
    for r in range(world):
        got = res[r][7][1]
        assert torch.isfinite(got).all()
        torch.testing.assert_close(got.double(), want_big, rtol=1e-5, atol=1e-4)


def test_single_process_is_identity():
    from bayesdll_amd import chains
    x = torch.log_softmax(torch.randn(4, 3), 1)
    assert chains.world() == 1 and chains.average_predictive(x) is x
