"""Stacked chains (bayesdll_amd.stacked, ABI v6 chain_groups) on the GPU.

The fused launch over K stacked chains must equal K one-chain launches with
chain ids chain0 + k bit for bit, given the same gradients (noise, update,
Welford collect, posterior draws); the vmapped gradients agree with per-chain
autograd to fp32 rounding (1e-5, the north-star tolerance).
"""
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


class Net(nn.Module):
    readout_name = "head"

    def __init__(self, d_in=13, hidden=7, classes=5):  # 13*7+7+7*5+5 = 138: n % 4 != 0
        super().__init__()
        self.body = nn.Linear(d_in, hidden)
        self.head = nn.Linear(hidden, classes)

    def forward(self, x):
        return self.head(torch.tanh(self.body(x)))


def _args(epochs=2, nst=2):
    return SimpleNamespace(
        lr=5e-2, lr_head=1e-1, epochs=epochs, num_cycles=2, proportion_exploration=0.5,
        ND=64, device="cuda", seed=7,
        hparams={"prior_sig": 1.0, "momentum_decay": 0.1, "Ninflate": 1.0, "nd": 1.0,
                 "thin": 1, "nst": nst, "bias": "informative", "burnin": 0})


def _single_states(S, K_):
    from bayesdll_amd.flat import FlatState
    segs = [(nm, s) for nm, s in zip(S.state.names, S.state.shapes)]
    out = []
    for k in range(K_):
        st = FlatState.from_segments(segs, "head", device="cuda", need_mom=True,
                                     init=S.state.chain_vector(k).clone())
        st.mom.copy_(S.state.mom2d[k, :S.state.n1])
        out.append(st)
    return out


def _single_update(S, st, grads_k, lr, ss, collect, k):
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    args = S.args
    st.use_tensor_grads([grads_k[nm].contiguous().view(-1) for nm in S.state.names])
    lrs = (lr, lr * (args.lr_head / args.lr))
    N = args.ND * S.Ninflate
    ns = [S.nd * np.sqrt(2 * S.momentum_decay * v) / N for v in lrs]
    ckind, m1, m2, ca = (L.COLLECT_NONE, None, None, 1.0) if collect is None else collect
    K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns,
                  noise_mode=L.NOISE_PHILOX if ss else L.NOISE_NONE,
                  one_minus_alpha=1 - S.momentum_decay, prior_sig=S.prior_sig, collect=ckind,
                  mom1=m1, mom2=m2, collect_a=ca, seed=S.seed, chain=S.chain0 + k,
                  step=S.step_count - 1)


@pytest.mark.parametrize("grad_mode", ["tensor", "flat"])
def test_stacked_launch_equals_one_chain_launches(grad_mode, monkeypatch):
    from bayesdll_amd import _lib as L
    from bayesdll_amd import stacked
    if grad_mode == "flat":  # force the stacked-gradient-vector fallback
        monkeypatch.setattr(stacked, "MAX_TENSOR_RUNS", 2)
    torch.manual_seed(0)
    K_ = 3
    S = stacked.StackedCSGHMC(Net().cuda(), K_, _args(), chain0=5, init="reinit")
    assert S.state.grad_mode == grad_mode and S.state.stride == 140
    singles = _single_states(S, K_)
    m1s = [torch.zeros(S.state.n1, device="cuda") for _ in range(K_)]
    m2s = [torch.zeros(S.state.n1, device="cuda") for _ in range(K_)]
    x = torch.randn(16, 13, device="cuda")
    y = torch.randint(0, 5, (16,), device="cuda")
    m1 = torch.zeros(S.state.n, device="cuda")
    m2 = torch.zeros(S.state.n, device="cuda")
    plan = [(0.05, False, None), (0.04, True, (L.COLLECT_WELFORD_INIT, 1.0)),
            (0.03, True, (L.COLLECT_WELFORD, 2.0)), (0.02, False, None),
            (0.01, True, (L.COLLECT_WELFORD, 3.0))]
    for lr, ss, col in plan:
        grads, _, _ = S.gradients(x, y)
        S.update(grads, lr, ss, None if col is None else (col[0], m1, m2, col[1]))
        for k in range(K_):
            _single_update(S, singles[k], {nm: g[k] for nm, g in grads.items()}, lr, ss,
                           None if col is None else (col[0], m1s[k], m2s[k], col[1]), k)
    torch.cuda.synchronize()
    n1 = S.state.n1
    for k in range(K_):
        assert torch.equal(S.state.theta2d[k, :n1], singles[k].theta), k
        assert torch.equal(S.state.mom2d[k, :n1], singles[k].mom), k
        assert torch.equal(m1.view(K_, -1)[k, :n1], m1s[k]), k
        assert torch.equal(m2.view(K_, -1)[k, :n1], m2s[k]), k
    # the padding of each chain's slot is never written
    assert torch.count_nonzero(S.state.theta2d[:, n1:]) == 0
    assert not S.state.diverged()
    # chains are distinct (own Philox keys, own init)
    assert not torch.equal(S.state.theta2d[0], S.state.theta2d[1])


def test_stacked_posterior_draws_equal_one_chain_draws():
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd._runner import EVAL_STEP_BASE
    torch.manual_seed(1)
    n1, K_ = 1001, 4
    stride = (n1 + 3) // 4 * 4
    mean = torch.randn(K_, stride, device="cuda")
    m2 = torch.rand(K_, stride, device="cuda")
    out = torch.empty(K_ * stride, device="cuda")
    K.posterior_sample(out, mean.view(-1), m2.view(-1), var_mode=L.VAR_WELFORD, ratio=3.0,
                       seed=11, chain=2, step=EVAL_STEP_BASE + 4, chain_groups=stride // 4)
    for k in range(K_):
        one = torch.empty(n1, device="cuda")
        K.posterior_sample(one, mean[k, :n1].contiguous(), m2[k, :n1].contiguous(),
                           var_mode=L.VAR_WELFORD, ratio=3.0, seed=11, chain=2 + k,
                           step=EVAL_STEP_BASE + 4)
        assert torch.equal(out.view(K_, stride)[k, :n1], one), k


def test_stacked_gradients_match_per_chain_autograd():
    """vmap(functional_call) gradients vs a separate autograd pass per chain:
    equal to fp32 rounding (batched vs single GEMMs)."""
    from bayesdll_amd import stacked
    torch.manual_seed(2)
    K_ = 4
    S = stacked.StackedCSGHMC(Net().cuda(), K_, _args(), init="reinit", seed=3)
    x = torch.randn(32, 13, device="cuda")
    y = torch.randint(0, 5, (32,), device="cuda")
    grads, loss, out = S.gradients(x, y)
    net = Net().cuda()
    for k in range(K_):
        S.state.load_chain(net, k)
        net.zero_grad()
        o = net(x)
        lk = nn.CrossEntropyLoss()(o, y)
        lk.backward()
        assert abs(lk.item() - loss[k].item()) <= 1e-5 * max(1.0, abs(lk.item()))
        torch.testing.assert_close(out[k], o.detach(), rtol=1e-5, atol=1e-5)
        for nm, p in net.named_parameters():
            torch.testing.assert_close(grads[nm][k], p.grad, rtol=1e-5, atol=1e-6)


def test_stacked_training_learns_and_evaluates():
    """Four epochs (two cycles) of 8 stacked chains on a separable
    synthetic problem: every chain's training error falls, moments are
    collected, the stacked predictive beats chance by far."""
    from bayesdll_amd import stacked
    torch.manual_seed(3)
    w = torch.randn(13, 5)
    xs = torch.randn(512, 13)
    ys = (xs @ w).argmax(1)
    loader = [(xs[i:i + 32], ys[i:i + 32]) for i in range(0, 512, 32)]
    args = _args(epochs=4, nst=2)
    args.lr, args.lr_head, args.ND = 0.1, 0.1, 512
    args.hparams["prior_sig"] = 1e-3
    S = stacked.StackedCSGHMC(Net().cuda(), 8, args, init="reinit", seed=5)
    hist = S.train(loader, test_loader=loader)
    first, last = np.array(hist[0]["error"]), np.array(hist[-1]["error"])
    # (a torch emulation of the same update on the CPU: 0.58 -> 0.11, max 0.12)
    assert last.mean() < 0.5 * first.mean() and last.max() < 0.3
    assert sorted(S.mom1) == [1, 2] and all(v >= 2 for v in S.samples_per_cycle.values())
    nll, err = S.evaluate(loader)
    assert np.isfinite(nll) and err < 0.3  # chance: 0.8
    assert "test" in hist[1] and "test" in hist[3]
    assert not S.state.diverged()


def test_stacked_graph_replay_is_bit_identical_to_eager():
    """HIP-graph replay of the vmapped forward/backward: same chains, same
    batches, same theta / momentum bit for bit after mixed steps."""
    from bayesdll_amd import stacked
    runs = []
    for graph in (False, True):
        torch.manual_seed(4)
        S = stacked.StackedCSGHMC(Net().cuda(), 5, _args(), init="reinit", seed=2, graph=graph)
        g = torch.Generator().manual_seed(9)
        for k in range(6):
            x = torch.randn(24, 13, generator=g).cuda()
            y = torch.randint(0, 5, (24,), generator=g).cuda()
            loss, out = S.step(x, y, 0.05 / (k + 1), should_sample=k % 2 == 1)
        torch.cuda.synchronize()
        runs.append((S.state.theta.clone(), S.state.mom.clone(), loss.clone(), len(S._graphs)))
    assert runs[0][3] == 0 and runs[1][3] == 1
    for a, b in zip(runs[0][:3], runs[1][:3]):
        assert torch.equal(a, b)


def test_stacked_sgld_equals_one_chain_launches():
    """StackedSGLD (SGLD + SGD momentum, prior theta0 from net0, burn-in
    seeding, running moments): every chain equals a one-chain SGLD launch
    sequence with chain id chain0 + k, bit for bit, given the same gradients."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd import stacked
    from bayesdll_amd.flat import FlatState
    torch.manual_seed(5)
    K_ = 3
    args = _args()
    args.momentum = 0.5
    args.hparams.update({"Ninflate": 10.0, "burnin": 0, "thin": 2, "nst": 2})
    net0 = Net().cuda()
    S = stacked.StackedSGLD(Net().cuda(), K_, args, chain0=2, init="reinit", net0=net0)
    st = S.state
    segs = [(nm, sh) for nm, sh in zip(st.names, st.shapes)]
    singles = []
    for k in range(K_):
        one = FlatState.from_segments(segs, "head", device="cuda", need_mom=True, need_prior=True,
                                      init=st.chain_vector(k).clone())
        one.prior.copy_(st.prior.view(K_, -1)[k, :st.n1])
        singles.append(one)
    S.seed_moments()
    m1s = [S.m1.view(K_, -1)[k, :st.n1].clone() for k in range(K_)]
    m2s = [S.m2.view(K_, -1)[k, :st.n1].clone() for k in range(K_)]
    x = torch.randn(16, 13, device="cuda")
    y = torch.randint(0, 5, (16,), device="cuda")
    lrs = (args.lr, args.lr_head)
    N = args.ND * 10.0
    for t in range(5):
        grads, _, _ = S.gradients(x, y)
        collect = t % 2 == 1
        spec = (L.COLLECT_MEAN, S.m1, S.m2, float(S.cnt), float(S.cnt + 1)) if collect else None
        cnt = S.cnt
        S.update(grads, lrs, collect=spec)
        if collect:
            S.cnt += 1
        for k, one in enumerate(singles):
            one.use_tensor_grads([grads[nm][k].contiguous().view(-1) for nm in st.names])
            K.sgmcmc_step(one, L.SGLD, lrs=lrs, noise_scale=[np.sqrt(2 / (N * v)) for v in lrs],
                          noise_mode=L.NOISE_PHILOX, prior_sig=1.0, sigma2=1.0, n_data=N, mu=0.5,
                          first_step=t == 0, momentum=True,
                          collect=L.COLLECT_MEAN if collect else L.COLLECT_NONE,
                          mom1=m1s[k] if collect else None, mom2=m2s[k] if collect else None,
                          collect_a=float(cnt), collect_b=float(cnt + 1), seed=S.seed,
                          chain=2 + k, step=t)
    torch.cuda.synchronize()
    for k, one in enumerate(singles):
        assert torch.equal(st.theta2d[k, :st.n1], one.theta), k
        assert torch.equal(st.mom2d[k, :st.n1], one.mom), k
        assert torch.equal(S.m1.view(K_, -1)[k, :st.n1], m1s[k]), k
        assert torch.equal(S.m2.view(K_, -1)[k, :st.n1], m2s[k]), k
    # the prior is net0 in every chain's slot
    p0 = torch.cat([q.detach().reshape(-1) for q in net0.parameters()])
    assert all(torch.equal(st.prior.view(K_, -1)[k, :st.n1], p0) for k in range(K_))


def test_stacked_sgld_trains_and_evaluates():
    from bayesdll_amd import stacked
    torch.manual_seed(6)
    w = torch.randn(13, 5)
    xs = torch.randn(512, 13)
    ys = (xs @ w).argmax(1)
    loader = [(xs[i:i + 32], ys[i:i + 32]) for i in range(0, 512, 32)]
    args = _args(epochs=4, nst=3)
    args.lr, args.lr_head, args.ND, args.momentum = 0.2, 0.2, 512, 0.5  # CPU emulation: 0.55 -> 0.12
    args.hparams.update({"prior_sig": 1.0, "Ninflate": 1e3, "nd": 1.0, "burnin": 2, "thin": 2})
    S = stacked.StackedSGLD(Net().cuda(), 6, args, init="reinit", seed=2, graph=True)
    hist = S.train(loader, test_loader=loader)
    first, last = np.array(hist[0]["error"]), np.array(hist[-1]["error"])
    assert last.mean() < 0.5 * first.mean() and last.max() < 0.3
    assert S.cnt == 1 + (2 * 16) // 2 and "test" not in hist[1] and "test" in hist[3]
    nll, err = S.evaluate(loader)
    assert np.isfinite(nll) and err < 0.3
    assert not S.state.diverged()


@pytest.mark.parametrize("cls", ["StackedCSGHMC", "StackedSGLD", "StackedCSGLD",
                                 "StackedSGHMC"])
def test_stacked_checkpoint_resume_is_exact(cls, tmp_path):
    """Two epochs, save_ckpt, two more epochs == a fresh sampler that loads the
    checkpoint and runs the last two epochs (theta, momentum, moments, bit for
    bit: the step counter is the Philox step key)."""
    from bayesdll_amd import stacked
    g = torch.Generator().manual_seed(8)
    xs, ys = torch.randn(256, 13, generator=g), torch.randint(0, 5, (256,), generator=g)
    loader = [(xs[i:i + 32].cuda(), ys[i:i + 32].cuda()) for i in range(0, 256, 32)]
    args = _args(epochs=4, nst=2)
    args.momentum = 0.5
    args.hparams.update({"burnin": 1, "thin": 2})  # (momentum_decay: sghmc)

    def make():
        torch.manual_seed(11)
        return getattr(stacked, cls)(Net().cuda(), 3, args, init="reinit", seed=4, chain0=0)

    A = make()
    for ep in range(2):
        A.train_one_epoch(loader, ep)
    path = A.save_ckpt(str(tmp_path / "stacked.pt"))
    for ep in range(2, 4):
        A.train_one_epoch(loader, ep)
    B = make()
    B.load_ckpt(path)
    B.train(loader, start_epoch=2)
    torch.cuda.synchronize()
    assert torch.equal(A.state.theta, B.state.theta)
    assert torch.equal(A.state.mom, B.state.mom)
    if cls == "StackedCSGHMC":
        assert sorted(A.mom1) == sorted(B.mom1) == [1, 2]
        for c in A.mom1:
            assert torch.equal(A.mom1[c], B.mom1[c]) and torch.equal(A.mom2[c], B.mom2[c])
        assert A.samples_per_cycle == B.samples_per_cycle
        # chain 1 as a one-chain csghmc checkpoint the Runner loads
        from bayesdll_amd import csghmc
        ck = A.export_chain(1)
        torch.save(ck, tmp_path / "chain1.pt")
        args.pretrained = None
        R = csghmc.Runner(Net().cuda(), None, args, __import__("logging").getLogger("t"))
        R.load_ckpt(str(tmp_path / "chain1.pt"))
        n1 = A.state.n1
        assert torch.equal(ck["last_theta"], A.state.theta2d[1, :n1])
        for c in A.mom1:
            assert torch.equal(R.cycle_theta_mom1[c], A.mom1[c].view(3, -1)[1, :n1])
        assert R.samples_per_cycle == A.samples_per_cycle
    elif cls == "StackedCSGLD":
        assert sorted(A.mom1) == sorted(B.mom1) == [1, 2]
        for c in A.mom1:
            assert torch.equal(A.mom1[c], B.mom1[c]) and torch.equal(A.mom2[c], B.mom2[c])
        assert A.samples_per_cycle == B.samples_per_cycle
    else:
        assert A.cnt == B.cnt and torch.equal(A.m1, B.m1) and torch.equal(A.m2, B.m2)
    with pytest.raises(ValueError, match="different"):
        getattr(stacked, cls)(Net().cuda(), 2, args).load_ckpt(path)


def test_stacked_csgld_trains_and_evaluates():
    """Cyclical SGLD: per-cycle running moments on the sample steps of each
    cycle (16 per cycle here), predictive over chains x cycle draws."""
    from bayesdll_amd import stacked
    torch.manual_seed(7)
    w = torch.randn(13, 5)
    xs = torch.randn(512, 13)
    ys = (xs @ w).argmax(1)
    loader = [(xs[i:i + 32], ys[i:i + 32]) for i in range(0, 512, 32)]
    args = _args(epochs=4, nst=2)
    args.lr, args.lr_head, args.ND, args.momentum = 0.2, 0.2, 512, 0.5
    args.hparams.update({"prior_sig": 1.0, "Ninflate": 1e3, "nd": 1.0, "thin": 1})
    S = stacked.StackedCSGLD(Net().cuda(), 4, args, init="reinit", seed=3)
    hist = S.train(loader, test_loader=loader)
    assert S.samples_per_cycle == {1: 16, 2: 16} and sorted(S.mom1) == [1, 2]
    assert "test" in hist[1] and "test" in hist[3] and "test" not in hist[0]
    first, last = np.array(hist[0]["error"]), np.array(hist[-1]["error"])
    assert last.mean() < first.mean()
    nll, err = S.evaluate(loader)
    assert np.isfinite(nll) and err < 0.5
    assert not S.state.diverged()


def test_stacked_sghmc_equals_one_chain_launches():
    """StackedSGHMC: every chain equals one-chain BDL_SGHMC launches with chain
    id chain0 + k (momentum v, prior theta0, running moments), bit for bit."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd import stacked
    from bayesdll_amd.flat import FlatState
    torch.manual_seed(9)
    K_ = 2
    args = _args()
    args.hparams.update({"Ninflate": 10.0, "burnin": 0, "thin": 1, "nst": 2})
    S = stacked.StackedSGHMC(Net().cuda(), K_, args, chain0=6, init="reinit", net0=Net().cuda())
    st = S.state
    segs = [(nm, sh) for nm, sh in zip(st.names, st.shapes)]
    ones = []
    for k in range(K_):
        one = FlatState.from_segments(segs, "head", device="cuda", need_mom=True, need_prior=True,
                                      init=st.chain_vector(k).clone())
        one.prior.copy_(st.prior.view(K_, -1)[k, :st.n1])
        ones.append(one)
    x = torch.randn(16, 13, device="cuda")
    y = torch.randint(0, 5, (16,), device="cuda")
    lrs = (args.lr, args.lr_head)
    N = args.ND * 10.0
    for t in range(4):
        grads, _, _ = S.gradients(x, y)
        S.update(grads, lrs)
        for k, one in enumerate(ones):
            one.use_tensor_grads([grads[nm][k].contiguous().view(-1) for nm in st.names])
            K.sgmcmc_step(one, L.SGHMC, lrs=lrs,
                          noise_scale=[np.sqrt(2 * 0.1 / (N * v)) for v in lrs],
                          noise_mode=L.NOISE_PHILOX, one_minus_alpha=1 - 0.1, prior_sig=1.0,
                          sigma2=1.0, n_data=N, seed=S.seed, chain=6 + k, step=t)
    torch.cuda.synchronize()
    for k, one in enumerate(ones):
        assert torch.equal(st.theta2d[k, :st.n1], one.theta), k
        assert torch.equal(st.mom2d[k, :st.n1], one.mom), k


def test_graph_capture_with_pending_garbage():
    """A dropped sampler that owns captured graphs must not be collected in
    the middle of another capture (freeing a graph's pool on a capturing
    stream aborts the process).  The invariant itself is checked: a gc
    callback fails the test if a collection ever starts while the current
    stream is capturing, with an unreachable graph-owning cycle created just
    before each capture and the collector at its most eager threshold.
    Samplers hold no reference cycle; capture collects pending garbage first
    and keeps the cyclic GC off until the capture ends; release_graphs()
    frees graphs deterministically."""
    import gc
    import weakref
    import bayesdll_amd.csghmc as csghmc
    from bayesdll_amd import stacked
    x = torch.randn(8, 13, device="cuda")
    y = torch.randint(0, 5, (8,), device="cuda")
    old = stacked.StackedCSGHMC(Net().cuda(), 2, _args(), graph=True)
    old.step(x, y, 0.01)
    ref = weakref.ref(old)
    del old
    assert ref() is None  # freed by reference counting, not left to the GC
    during_capture = []

    def watch(phase, info):
        if phase == "start" and torch.cuda.is_current_stream_capturing():
            during_capture.append(info)

    def garbage_cycle():
        holder = {"s": stacked.StackedCSGHMC(Net().cuda(), 2, _args(), graph=True)}
        holder["s"].step(x, y, 0.01)
        holder["self"] = holder  # unreachable cycle owning a captured graph
    th = gc.get_threshold()
    gc.callbacks.append(watch)
    gc.set_threshold(1)  # collect at every opportunity
    try:
        garbage_cycle()
        S = stacked.StackedCSGHMC(Net().cuda(), 3, _args(), graph=True)
        loss, _ = S.step(x, y, 0.01)
        # the Model path: two input shapes, a cycle created before each capture
        net = Net().cuda()
        model = csghmc.Model(100.0, prior_sig=1.0, momentum_decay=0.1)
        model.graph = True
        for xb, yb in ((x, y), (x[:5], y[:5])):
            garbage_cycle()
            model(xb, yb, net, None, torch.nn.CrossEntropyLoss(), [1e-3, 1e-3], 1.0, 1.0)
        assert model.graph_captures == 2
        model.release_graphs()
        S.release_graphs()
        assert not model._graphs and not S._graphs
        torch.cuda.synchronize()
        assert torch.isfinite(loss).all()
    finally:
        gc.callbacks.remove(watch)
        gc.set_threshold(*th)
        gc.collect()
    assert not during_capture, during_capture


def test_sampler_dropped_inside_a_capture_parks_its_graphs():
    """A graph-mode sampler whose last reference goes while ANOTHER capture is
    running (user code capturing its own graph) must not destroy its graphs
    there (their pools would be freed on a capturing stream): Model.__del__
    parks them (_base._DEFERRED_GRAPHS) and they are destroyed at the next
    point outside any capture."""
    import weakref
    import bayesdll_amd.csghmc as csghmc
    from bayesdll_amd import _base
    x = torch.randn(8, 13, device="cuda")
    y = torch.randint(0, 5, (8,), device="cuda")
    net = Net().cuda()
    model = csghmc.Model(100.0, prior_sig=1.0, momentum_decay=0.1)
    model.graph = True
    model(x, y, net, None, torch.nn.CrossEntropyLoss(), [1e-3, 1e-3], 1.0, 1.0)
    assert model.graph_captures == 1 and len(model._graphs) == 1
    gref = weakref.ref(next(iter(model._graphs.values()))["graph"])
    z = torch.zeros(4, device="cuda")
    user = torch.cuda.CUDAGraph()
    with torch.cuda.graph(user):
        z.add_(1.0)
        del model  # the sampler goes mid-capture
        assert len(_base._DEFERRED_GRAPHS) == 1 and gref() is not None
    user.replay()
    _base.release_deferred_graphs()
    assert not _base._DEFERRED_GRAPHS and gref() is None
    torch.cuda.synchronize()
    assert z.tolist() == [1.0] * 4


def test_stacked_refuses_batchnorm_statistics():
    from bayesdll_amd import stacked
    net = nn.Sequential(nn.Linear(4, 4), nn.BatchNorm1d(4)).cuda()
    with pytest.raises(ValueError, match="BatchNorm"):
        stacked.StackedState(net, 2)
