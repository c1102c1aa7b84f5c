"""Multi-chain logic on CPU with torch.distributed gloo, world_size 2 and 4
(stands in for RCCL over xGMI: the same all_reduce / all_gather calls)."""
import os
import socket

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
        q.put((r, logp, avg, la, gathered, default_chain(), chains.chain_seed(42)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_average_predictive_and_gather_chains(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, logp, avg, la, gathered, chain, seed = q.get(timeout=120)
        res[r] = (logp, avg, la, gathered, chain, seed)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = torch.log(sum(res[r][0].exp() for r in range(world)) / world)
    for r in range(world):
        torch.testing.assert_close(res[r][1], want)
        torch.testing.assert_close(res[r][3], torch.cat([res[k][2] for k in range(world)], dim=2))
        assert res[r][4] == r            # Philox chain id = rank
        assert res[r][5] == 42 + r       # per-chain seed
    # the averaged predictive is a proper distribution
    torch.testing.assert_close(want.exp().sum(1), torch.ones(8))


def test_single_process_is_identity():
    from bayesdll_amd import chains
    x = torch.log_softmax(torch.randn(4, 3), 1)
    assert chains.world() == 1 and chains.average_predictive(x) is x
