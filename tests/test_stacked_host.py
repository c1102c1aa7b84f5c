"""Host logic of bayesdll_amd.stacked on the CPU (no launches): the stacked
layout, the per-(chain, tensor) run / gradient-base table, the flat fallback,
and the vmapped gradients against per-chain autograd.  The launches themselves
are tested on the GPU (tests/test_gpu_stacked.py)."""
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.nn as nn


class Net(nn.Module):
    readout_name = "head"

    def __init__(self):
        super().__init__()
        self.body = nn.Linear(13, 7)   # 91 + 7
        self.head = nn.Linear(7, 5)    # 35 + 5  -> n = 138, stride 140

    def forward(self, x):
        return self.head(torch.tanh(self.body(x)))


def _args():
    return SimpleNamespace(lr=5e-2, lr_head=1e-1, epochs=2, num_cycles=2,
                           proportion_exploration=0.5, ND=64, device="cpu", seed=7,
                           hparams={"prior_sig": 1.0, "momentum_decay": 0.1, "Ninflate": 1.0,
                                    "nd": 1.0, "thin": 1, "nst": 0, "bias": "informative"})


@pytest.fixture
def host_only(monkeypatch):
    """Let the state live on the CPU and record launches instead of making them."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    calls = []
    monkeypatch.setattr(L, "require_hip", lambda *a, **k: None)
    monkeypatch.setattr(torch.Tensor, "pin_memory", lambda self: self)
    monkeypatch.setattr(K, "sgmcmc_step", lambda st, m, **kw: calls.append((st, m, kw)))
    return calls


def test_stacked_layout_and_grad_table(host_only):
    from bayesdll_amd import _lib as L
    from bayesdll_amd import stacked
    torch.manual_seed(0)
    S = stacked.StackedCSGHMC(Net(), 3, _args(), chain0=4, init="reinit", seed=1)
    st = S.state
    assert (st.n1, st.stride, st.n, st.chain_groups) == (138, 140, 420, 35)
    # chains start from different re-initialisations; padding is zero
    assert not torch.equal(st.theta2d[0], st.theta2d[1])
    assert torch.count_nonzero(st.theta2d[:, 138:]) == 0
    # parameter views alias the stacked theta
    assert st.params["head.bias"].data_ptr() == st.theta2d.data_ptr() + 4 * (91 + 7 + 35)
    x, y = torch.randn(16, 13), torch.randint(0, 5, (16,))
    grads, loss, out = S.gradients(x, y)
    assert loss.shape == (3,) and out.shape == (3, 16, 5)
    S.update(grads, 0.05, should_sample=True)
    (sst, method, kw), = host_only
    assert method == L.CSGHMC and kw["chain"] == 4 and kw["noise_mode"] == L.NOISE_PHILOX
    runs = st.runs.numpy()
    assert st.nruns == 3 * 5 and runs.shape == (15, 2)
    ends = runs[:, 0].tolist()
    assert ends == [91, 98, 133, 138, 140, 231, 238, 273, 278, 280, 371, 378, 413, 418, 420]
    attrs = runs[:, 1] & 0x7
    assert attrs.tolist() == [2, 2, 3, 3, 4] * 3          # PRIOR, +HEAD, SKIP padding
    bases = st.gbase.numpy()
    names = st.names
    for k in range(3):
        for i, nm in enumerate(names):
            r = 5 * k + i
            start = k * 140 + st.offsets[i]
            want = grads[nm].data_ptr() + 4 * k * st.numels[i] - 4 * start
            assert bases[r] == want
            assert bool(runs[r, 1] & L.ATTR_GUNALIGNED) == bool(want % 16)
        assert bases[5 * k + 4] == 0
    # same gradient tensors again -> the cached table
    S.update(grads, 0.05)
    assert host_only[-1][0].runs is sst.runs


def test_stacked_flat_fallback_copies_gradients(host_only, monkeypatch):
    from bayesdll_amd import stacked
    monkeypatch.setattr(stacked, "MAX_TENSOR_RUNS", 4)
    S = stacked.StackedCSGHMC(Net(), 2, _args())
    st = S.state
    assert st.grad_mode == "flat" and st.gbase is None
    grads, _, _ = S.gradients(torch.randn(8, 13), torch.randint(0, 5, (8,)))
    S.update(grads, 0.01)
    for k in range(2):
        for nm, o, n in zip(st.names, st.offsets, st.numels):
            assert torch.equal(st.grad2d[k, o:o + n], grads[nm][k].reshape(-1))
    # merged runs per chain; padding skipped
    ends = st.runs[:, 0].tolist()
    assert ends[-1] == 280 and 140 in ends and 138 in ends


def test_stacked_gradients_equal_per_chain_autograd_on_cpu(host_only):
    from bayesdll_amd import stacked
    torch.manual_seed(2)
    S = stacked.StackedCSGHMC(Net(), 4, _args(), init="reinit", seed=3)
    x, y = torch.randn(32, 13), torch.randint(0, 5, (32,))
    grads, loss, _ = S.gradients(x, y)
    net = Net()
    for k in range(4):
        S.state.load_chain(net, k)
        net.zero_grad()
        lk = nn.CrossEntropyLoss()(net(x), y)
        lk.backward()
        assert abs(lk.item() - loss[k].item()) < 1e-5
        for nm, p in net.named_parameters():
            np.testing.assert_allclose(grads[nm][k].numpy(), p.grad.numpy(), rtol=1e-5, atol=1e-6)


def test_stacked_per_chain_batches(host_only):
    """per_chain_batches: chain k trains on batch k ([K, B, ...]) and is
    evaluated on the shared batch."""
    from bayesdll_amd import stacked
    torch.manual_seed(4)
    S = stacked.StackedCSGHMC(Net(), 3, _args(), init="reinit", seed=1, per_chain_batches=True)
    x, y = torch.randn(3, 8, 13), torch.randint(0, 5, (3, 8))
    grads, loss, out = S.gradients(x, y)
    assert out.shape == (3, 8, 5)
    net = Net()
    for k in range(3):
        S.state.load_chain(net, k)
        net.zero_grad()
        lk = nn.CrossEntropyLoss()(net(x[k]), y[k])
        lk.backward()
        assert abs(lk.item() - loss[k].item()) < 1e-5
        np.testing.assert_allclose(grads["head.weight"][k].numpy(), net.head.weight.grad.numpy(),
                                   rtol=1e-5, atol=1e-6)
    assert S.chain_logits(x[0]).shape == (3, 8, 5)
    assert S.predictive_logprob(x[0]).shape == (8, 5)


def test_stacked_frozen_parameter_is_skipped(host_only):
    from bayesdll_amd import _lib as L
    from bayesdll_amd import stacked
    net = Net()
    net.body.bias.requires_grad_(False)
    S = stacked.StackedCSGHMC(net, 2, _args())
    grads, _, _ = S.gradients(torch.randn(8, 13), torch.randint(0, 5, (8,)))
    assert "body.bias" not in grads
    S.update(grads, 0.01)
    runs = S.state.runs.numpy()
    assert runs[1, 1] & L.ATTR_SKIP and runs[6, 1] & L.ATTR_SKIP
    assert S.state.gbase.numpy()[1] == 0


def test_stacked_refuses_what_it_cannot_stack(host_only):
    from bayesdll_amd import stacked
    with pytest.raises(ValueError, match="BatchNorm"):
        stacked.StackedState(nn.Sequential(nn.Linear(4, 4), nn.BatchNorm1d(4)), 2)
    with pytest.raises(ValueError, match="K must be"):
        stacked.StackedState(Net(), 0)
    with pytest.raises(ValueError, match="init"):
        stacked.StackedState(Net(), 2, init="zeros")


def _stacked_worker(r, world, port, q):
    import torch.distributed as dist
    from bayesdll_amd import _lib as L
    from bayesdll_amd import stacked
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    L.require_hip = lambda *a, **k: None
    dist.init_process_group("gloo", rank=r, world_size=world)
    try:
        torch.manual_seed(0)
        S = stacked.StackedCSGHMC(Net(), 2, _args(), init="reinit", seed=10 + 2 * r)
        x = torch.randn(6, 13, generator=torch.Generator().manual_seed(5))
        # numpy copies, not tensors: a tensor put on a torch.multiprocessing queue
        # travels as a shared-memory handle that the receiver can only open while
        # this process is alive, and it exits right after (a flaky receive)
        q.put((r, S.chain0, S.chain_logits(x).detach().numpy().copy(),
               S.predictive_logprob(x).detach().numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_stacked_predictive_averages_over_processes():
    """Two processes x two stacked chains (gloo): chain ids rank*K + k, and
    every process returns the predictive averaged over all four chains."""
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_stacked_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, c0, logits, lp = q.get(timeout=300)
        res[r] = (c0, torch.from_numpy(logits), torch.from_numpy(lp))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == 0 and res[1][0] == 2
    probs = torch.cat([res[r][1] for r in range(2)]).softmax(-1)  # [4, B, C]
    want = probs.mean(0).log()
    for r in range(2):
        torch.testing.assert_close(res[r][2], want, rtol=1e-5, atol=1e-6)


def test_no_gc_disables_and_restores_the_collector():
    import gc

    from bayesdll_amd._base import no_gc
    assert gc.isenabled()
    with no_gc():
        assert not gc.isenabled()
    assert gc.isenabled()
    gc.disable()
    try:
        with no_gc():
            pass
        assert not gc.isenabled()  # left as the caller had it
    finally:
        gc.enable()
    with pytest.raises(RuntimeError):
        with no_gc():
            raise RuntimeError("capture failed")
    assert gc.isenabled()
