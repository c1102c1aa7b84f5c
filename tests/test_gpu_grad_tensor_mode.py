"""Per-tensor gradient mode (bdl_step_args.grad_base): the kernels read each
parameter's gradient where autograd left it, through a per-run base table,
instead of from one flat gradient vector.  Every method must give bit for bit
what the flat-vector path gives on the same values — including gradients whose
base is not 16-B addressable (odd offsets, a storage offset: element-wise
path), a parameter without a gradient (SKIP), the *_GRAD methods writing the
gradient tensors back in place, Adam, and clipped SGLD's norm pass.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

# sizes chosen so that some tensors start at flat offsets that are not
# multiples of 4 (their bases are misaligned even for aligned allocations) and
# some are long enough for the unrolled fast path
SEGMENTS = [
    ("a.weight", (300, 257)),        # 77100
    ("a.bias", (257,)),              # odd size: everything after is offset by 1 mod 4
    ("b.weight", (1000, 130)),       # 130000
    ("b.bias", (130,)),
    ("unused.weight", (64,)),        # no gradient in the step
    ("c.weight", (4096, 8)),         # 32768
    ("classifier.weight", (10, 130)),
    ("classifier.bias", (10,)),
]
UNUSED = 4


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _net():
    from fakenet import FakeNet
    return FakeNet(segments=SEGMENTS, readout_name="classifier").to(DEV)


def _states(seed, need_prior, extra=()):
    """(tensor-mode state, flat-mode state) over identical values; the
    tensor-mode gradients are separate tensors, one of them at a 4-B storage
    offset."""
    from bayesdll_amd.flat import FlatState
    kw = dict(readout_name="classifier", need_prior=need_prior, need_mom=True, extra=extra)
    st_t = FlatState(_net(), grad_mode="tensor", **kw)
    st_f = FlatState(_net(), grad_mode="flat", **kw)
    g = torch.Generator(device=DEV).manual_seed(seed)
    st_t.theta.normal_(0.0, 0.02, generator=g)
    st_t.mom.normal_(0.0, 1e-4, generator=g)
    if need_prior:
        st_t.prior.normal_(0.0, 0.02, generator=g)
        st_f.prior.copy_(st_t.prior)
    for nm in extra:
        st_t.extra[nm].uniform_(0.0, 1e-6, generator=g)
        st_f.extra[nm].copy_(st_t.extra[nm])
    st_f.theta.copy_(st_t.theta)
    st_f.mom.copy_(st_t.mom)
    grads = [torch.randn(k, device=DEV, generator=g) * 1e-3 for k in st_t.numels]
    # tensor mode: autograd-like separate gradient tensors (+ one at an offset)
    st_t.zero_grad()
    for i, (p, gr) in enumerate(zip(st_t.params, grads)):
        if i == UNUSED:
            continue
        if i in (1, 2):
            # a storage offset of one float: a.bias (flat offset 77100) gets a
            # misaligned base; b.weight (flat offset 77357, odd) gets an aligned
            # one — the fast path then runs over a tensor at an odd flat offset
            holder = torch.empty(gr.numel() + 1, device=DEV)
            holder[1:].copy_(gr)
            p.grad = holder[1:].view(p.shape)
        else:
            p.grad = gr.clone().view(p.shape)
    st_t.sync_grads()
    # flat mode: the same values in the flat buffer; parameter UNUSED untouched
    st_f.zero_grad()
    for i, (p, gr) in enumerate(zip(st_f.params, grads)):
        if i != UNUSED:
            p.grad.copy_(gr.view(p.shape))
    st_f._touched[:] = [i != UNUSED for i in range(len(st_f.params))]
    st_f.sync_grads()
    return st_t, st_f


def _check_table(st_t):
    from bayesdll_amd import _lib as L
    runs = st_t.runs.cpu().numpy()
    assert st_t.gbase is not None and st_t.nruns == len(SEGMENTS)
    assert runs[UNUSED, 1] & L.ATTR_SKIP
    assert not runs[0, 1] & L.ATTR_GUNALIGNED     # aligned tensor at offset 0
    assert runs[1, 1] & L.ATTR_GUNALIGNED         # storage offset of 4 B
    assert not runs[2, 1] & L.ATTR_GUNALIGNED     # odd flat offset + 4 B storage offset
    assert runs[3, 1] & L.ATTR_GUNALIGNED         # flat offset 207357: odd


def _grads_t(st):
    return torch.cat([torch.zeros(k, device=DEV) if p.grad is None else p.grad.reshape(-1)
                      for p, k in zip(st.params, st.numels)])


@pytest.mark.parametrize("case", ["csghmc_collect", "sghmc", "sgld_first", "sgld",
                                  "sghmc_grad", "sgld_grad", "sgld_clipped",
                                  "adam", "adam_grad"])
def test_tensor_mode_equals_flat_mode(case):
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    need_prior = case != "csghmc_collect"
    adam = case.startswith("adam")
    st_t, st_f = _states(11, need_prior, extra=("adam_m", "adam_v", "sgd_buf") if adam else ())
    _check_table(st_t)
    n = st_t.n
    m1 = {s: torch.randn(n, device=DEV) * 0.02 for s in ("t", "f")}
    m2 = {s: torch.rand(n, device=DEV) * 1e-4 for s in ("t", "f")}
    m1["f"].copy_(m1["t"])
    m2["f"].copy_(m2["t"])
    common = dict(lrs=(1e-3, 3e-3), seed=5, chain=1, step=17, div_mode="recip")
    for tag, st in (("t", st_t), ("f", st_f)):
        if case == "csghmc_collect":
            K.sgmcmc_step(st, L.CSGHMC, noise_scale=(1e-3, 2e-3), noise_mode=L.NOISE_PHILOX,
                          one_minus_alpha=0.82, prior_sig=1.0, collect=L.COLLECT_WELFORD,
                          mom1=m1[tag], mom2=m2[tag], collect_a=3.0, **common)
        elif case in ("sghmc", "sghmc_grad"):
            K.sgmcmc_step(st, L.SGHMC if case == "sghmc" else L.SGHMC_GRAD,
                          noise_scale=(1e-3, 2e-3), noise_mode=L.NOISE_PHILOX,
                          one_minus_alpha=0.9, sigma2=1.0, n_data=1e4, **common)
        elif case in ("sgld_first", "sgld"):
            K.sgmcmc_step(st, L.SGLD, noise_scale=(1e-3, 2e-3), noise_mode=L.NOISE_PHILOX,
                          sigma2=1.0, n_data=1e4, mu=0.5, momentum=True,
                          first_step=case == "sgld_first", collect=L.COLLECT_MEAN,
                          mom1=m1[tag], mom2=m2[tag], collect_a=2.0, collect_b=3.0, **common)
        elif case == "sgld_grad":
            K.sgmcmc_step(st, L.SGLD_GRAD, noise_scale=(1e-3, 2e-3), noise_mode=L.NOISE_PHILOX,
                          sigma2=1.0, n_data=1e4, **common)
        elif case == "sgld_clipped":
            ws = K.sgld_step_clipped(st, 1e-3, noise_scale=(1e-3, 2e-3),
                                     noise_mode=L.NOISE_PHILOX, sigma2=1.0, n_data=1e4, mu=0.5,
                                     momentum=True, **common)
            (m1 if tag == "t" else m2)["clip_" + tag] = ws[:2].clone()
        else:
            K.adam_step(st, L.ADAM_SGHMC if case == "adam" else L.ADAM_SGHMC_GRAD,
                        adam_m=st.extra["adam_m"], adam_v=st.extra["adam_v"],
                        sgd_buf=st.extra["sgd_buf"] if case == "adam" else None, beta1=0.9,
                        beta2=0.999, eps=1e-8, t=3, momentum_decay=0.1, nd=0.01,
                        noise_mode=L.NOISE_PHILOX, sigma2=1.0, n_data=1e4, mu=0.5,
                        momentum=case == "adam", **common)
    torch.cuda.synchronize()
    assert torch.equal(st_t.theta, st_f.theta)
    assert torch.equal(st_t.mom, st_f.mom)
    assert torch.equal(_grads_t(st_t), st_f.grad)  # *_GRAD: written back in place
    assert torch.equal(m1["t"], m1["f"]) and torch.equal(m2["t"], m2["f"])
    for nm in st_t.extra:
        assert torch.equal(st_t.extra[nm], st_f.extra[nm])
    if case == "sgld_clipped":
        assert torch.equal(m1["clip_t"], m2["clip_f"])
    # the parameter without a gradient still has none
    assert st_t.params[UNUSED].grad is None


def test_model_steps_leave_grads_as_autograd_tensors():
    """Through Model.forward on a real MLP: .grad are autograd's own tensors
    after the step (no flat buffer, no accumulation), the table is cached while
    the allocator hands out the same gradient blocks, and the chain equals the
    flat-mode chain bit for bit."""
    import os
    import bayesdll_amd.csghmc as csghmc
    from fakenet import MLP, init_vector, synthetic_mnist
    n = 2797010
    init = torch.tensor(init_vector(41, n, 0.03))
    data = synthetic_mnist(42, 256, 64, device=DEV)
    crit = torch.nn.CrossEntropyLoss()

    def run(mode):
        os.environ["BDL_GRAD_MODE"] = mode
        try:
            net = MLP()
            with torch.no_grad():
                torch.nn.utils.vector_to_parameters(init.clone(), net.parameters())
            net = net.to(DEV)
            model = csghmc.Model(30000.0, prior_sig=1.0, momentum_decay=0.18)
            model.noise_mode, model.seed = "philox", 3
            for ep in range(2):
                for k, (x, y) in enumerate(data):
                    model(x, y, net, None, crit, [1e-2, 2e-2], 1.0, 0.5, should_sample=k % 2 == 0)
            torch.cuda.synchronize()
            return model, net
        finally:
            os.environ.pop("BDL_GRAD_MODE", None)

    m_t, net_t = run("tensor")
    m_f, _ = run("flat")
    st = m_t.flat
    assert st.grad_mode == "tensor" and st.grad is None and st.gbase is not None
    assert m_f.flat.grad_mode == "flat" and m_f.flat.gbase is None
    assert 1 <= len(st._grad_tables) <= 8
    for p in net_t.parameters():
        assert p.grad is not None and p.grad.data_ptr() != 0
    assert torch.equal(m_t.flat.theta, m_f.flat.theta)
    np.testing.assert_array_equal(m_t.flat.mom.cpu().numpy(), m_f.flat.mom.cpu().numpy())


@pytest.mark.parametrize("method", ["sgld", "adam_sghmc"])
def test_frozen_parameters_tensor_vs_flat(method):
    """requires_grad=False parameters (a frozen first layer) are SKIP runs in
    both gradient modes: untouched, no noise, no SGD step; the rest of the
    chain is bit-identical between the modes."""
    import os
    import importlib
    from bayesdll_amd.sgld import FusedSGD
    from fakenet import MLP, init_vector, synthetic_mnist
    mod = importlib.import_module(f"bayesdll_amd.{method}")
    n = 2797010
    init = torch.tensor(init_vector(51, n, 0.03))
    prior = torch.tensor(init_vector(52, n, 0.03))
    data = synthetic_mnist(53, 192, 64, device=DEV)
    crit = torch.nn.CrossEntropyLoss()

    def run(mode):
        os.environ["BDL_GRAD_MODE"] = mode
        try:
            net, net0 = MLP(), MLP()
            with torch.no_grad():
                torch.nn.utils.vector_to_parameters(init.clone(), net.parameters())
                torch.nn.utils.vector_to_parameters(prior.clone(), net0.parameters())
            net, net0 = net.to(DEV), net0.to(DEV)
            for p in net.layers[0].parameters():
                p.requires_grad_(False)
            if method == "sgld":
                model = mod.Model(30000.0, prior_sig=1.0)
            else:
                model = mod.Model(30000.0, prior_sig=1.0, momentum_decay=0.1)
            model.noise_mode, model.seed = "philox", 9
            opt = torch.optim.SGD(net.parameters(), lr=1e-2, momentum=0.5)
            fsgd = FusedSGD(opt, 0.5)
            w0 = net.layers[0].weight.detach().clone()
            for x, y in data:
                model(x, y, net, net0, crit, [1e-2, 1e-2], 1.0, 0.5, sgd=fsgd)
            torch.cuda.synchronize()
            assert torch.equal(net.layers[0].weight.detach(), w0)
            return model.flat.theta.clone()
        finally:
            os.environ.pop("BDL_GRAD_MODE", None)

    assert torch.equal(run("tensor"), run("flat"))


@pytest.mark.parametrize("where", ["fast", "tail"])
@pytest.mark.parametrize("method", ["csghmc", "sgld", "sgld_grad", "adam"])
def test_divergence_flag(method, where):
    """bdl_step_args.nonfinite: a step that writes a NaN / Inf theta (or
    gradient, *_GRAD) raises the device flag — from the unrolled fast path and
    from the guarded tail; a healthy step leaves it 0."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.flat import FlatState
    segs = [("w", (70001,)), ("classifier.weight", (10, 30))]  # n = 70301: a ragged tail
    st = FlatState.from_segments(segs, "classifier", device=DEV, need_prior=True,
                                 extra=("adam_m", "adam_v") if method == "adam" else ())
    g = torch.Generator(device=DEV).manual_seed(3)
    st.theta.normal_(0, 0.02, generator=g)
    st.grad.normal_(0, 1e-3, generator=g)

    def step():
        kw = dict(lrs=(1e-3, 1e-3), noise_mode=L.NOISE_PHILOX, seed=1, step=0)
        if method == "csghmc":
            K.sgmcmc_step(st, L.CSGHMC, noise_scale=(1e-3, 1e-3), one_minus_alpha=0.9,
                          prior_sig=1.0, **kw)
        elif method in ("sgld", "sgld_grad"):
            K.sgmcmc_step(st, L.SGLD if method == "sgld" else L.SGLD_GRAD,
                          noise_scale=(1e-3, 1e-3), sigma2=1.0, n_data=1e3, **kw)
        else:
            K.adam_step(st, L.ADAM_SGHMC, adam_m=st.extra["adam_m"], adam_v=st.extra["adam_v"],
                        beta1=0.9, beta2=0.999, eps=1e-8, t=1, momentum_decay=0.1, nd=0.01,
                        sigma2=1.0, n_data=1e3, **kw)
        torch.cuda.synchronize()

    step()
    assert not st.diverged()
    idx = 1000 if where == "fast" else st.n - 2
    st.grad[idx] = float("nan") if method != "adam" else float("inf")
    step()
    assert st.diverged()          # reads and resets
    assert not st.diverged()
    st.grad.normal_(0, 1e-3, generator=g)
    st.theta.normal_(0, 0.02, generator=g)
    if method == "adam":
        st.extra["adam_m"].zero_()
        st.extra["adam_v"].zero_()
    st.mom.zero_()
    step()
    assert not st.diverged()


def test_runner_reports_divergence():
    """A cSGHMC chain with an absurd step size blows up; the Runner notices at
    the epoch boundary (one flag read per epoch) and records the epoch."""
    import logging
    import tempfile
    from types import SimpleNamespace
    import bayesdll_amd.csghmc as csghmc
    from fakenet import MLP, synthetic_mnist
    train = synthetic_mnist(61, 128, 64, device=DEV)
    test = synthetic_mnist(62, 64, 64, device=DEV)

    def run(lr):
        torch.manual_seed(0)
        args = SimpleNamespace(device=DEV, ND=128, pretrained=None, lr=lr, lr_head=lr,
                               momentum=0.0, epochs=2, num_cycles=1, proportion_exploration=0.5,
                               full_sample=False, test_eval_freq=100, ece_num_bins=15,
                               log_dir=tempfile.mkdtemp(), num_classes=10,
                               hparams={"prior_sig": "1.0", "bias": "informative",
                                        "momentum_decay": "0.1", "Ninflate": "1.0",
                                        "nd": "0.0", "burnin": "0", "thin": "100", "nst": "0"})
        r = csghmc.Runner(MLP().to(DEV), None, args, logging.getLogger("div"))
        r.train(train, None, test)
        return r.diverged_epochs

    assert run(1e-3) == []
    assert run(1e38) != []


def test_step_timing_log(caplog):
    """BDL_STEP_TIMING=k: sampled HIP-event timing of the fused update and one
    log line per epoch with launches, mean ms and algorithmic GB/s."""
    import logging
    import os
    import tempfile
    from types import SimpleNamespace
    import bayesdll_amd.csghmc as csghmc
    from fakenet import MLP, synthetic_mnist
    train = synthetic_mnist(71, 256, 64, device=DEV)
    os.environ["BDL_STEP_TIMING"] = "2"
    try:
        args = SimpleNamespace(device=DEV, ND=256, pretrained=None, lr=1e-3, lr_head=1e-3,
                               momentum=0.0, epochs=2, num_cycles=2, proportion_exploration=0.5,
                               full_sample=False, test_eval_freq=100, ece_num_bins=15,
                               log_dir=tempfile.mkdtemp(), num_classes=10,
                               hparams={"prior_sig": "1.0", "bias": "informative",
                                        "momentum_decay": "0.1", "Ninflate": "1.0",
                                        "nd": "0.01", "burnin": "0", "thin": "2", "nst": "0"})
        torch.manual_seed(0)
        log = logging.getLogger("timing")
        with caplog.at_level(logging.INFO, logger="timing"):
            r = csghmc.Runner(MLP().to(DEV), None, args, log)
            r.train(train, None, synthetic_mnist(72, 64, 64, device=DEV))
    finally:
        os.environ.pop("BDL_STEP_TIMING", None)
    lines = [m for m in caplog.messages if "fused update:" in m]
    assert len(lines) == 2 and "4 launches" in lines[0] and "GB/s algorithmic" in lines[0]


def test_philox_offset_subrange_launches_equal_one_launch():
    """bdl_step_args.philox_offset: launching the cSGHMC step bucket by bucket
    over sub-ranges (FlatState.bucket_state, offsets multiples of 4) gives,
    bit for bit, the whole-vector launch — Philox noise and Welford collection
    included."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.flat import FlatState
    from bayesdll_amd.shapes import segments
    segs, readout = segments("resnet101", 37)
    sts = []
    for _ in range(2):
        st = FlatState.from_segments(segs, readout, device=DEV)
        g = torch.Generator(device=DEV).manual_seed(7)
        st.theta.normal_(0, 0.02, generator=g)
        st.grad.normal_(0, 1e-3, generator=g)
        st.mom.normal_(0, 1e-4, generator=g)
        st.flatg = st.grad  # keep the storage the per-tensor views read
        st.use_tensor_grads([st.grad[o:o + k] for o, k in zip(st.offsets, st.numels)])
        sts.append(st)
    m1 = [torch.full((sts[0].n,), 0.01, device=DEV) for _ in range(2)]
    m2 = [torch.full((sts[0].n,), 1e-4, device=DEV) for _ in range(2)]
    kw = dict(lrs=(1e-4, 1e-2), noise_scale=(1e-3, 2e-3), noise_mode=L.NOISE_PHILOX,
              one_minus_alpha=0.82, prior_sig=1.0, collect=L.COLLECT_WELFORD, collect_a=3.0,
              seed=5, chain=2, step=11)
    K.sgmcmc_step(sts[0], L.CSGHMC, mom1=m1[0], mom2=m2[0], **kw)
    st = sts[1]
    plan = st.bucket_plan(1 << 20)
    assert len(plan) > 10 and all(b[0] % 4 == 0 for b in plan)
    grads = [st.flatg[o:o + k] for o, k in zip(st.offsets, st.numels)]
    for b in plan:
        sub = st.bucket_state(b, [grads[i].data_ptr() for i in b[2]])
        K.sgmcmc_step(sub, L.CSGHMC, mom1=m1[1][b[0]:b[1]], mom2=m2[1][b[0]:b[1]],
                      philox_offset=b[0] // 4, **kw)
    torch.cuda.synchronize()
    assert torch.equal(sts[0].theta, sts[1].theta) and torch.equal(sts[0].mom, sts[1].mom)
    assert torch.equal(m1[0], m1[1]) and torch.equal(m2[0], m2[1])


def test_overlapped_update_equals_one_launch(monkeypatch):
    """BDL_OVERLAP / Model.overlap: the cSGHMC update launched per bucket from
    post-accumulate hooks on a side stream, overlapping backward, gives the
    sequential chain bit for bit (explore and sample steps, Welford collects,
    a parameter without a gradient in one step)."""
    import bayesdll_amd._base as B
    import bayesdll_amd.csghmc as csghmc
    from fakenet import MLP, init_vector, synthetic_mnist
    monkeypatch.setattr(B, "OVERLAP_BUCKET_ELEMS", 1 << 18)  # several buckets on an MLP
    n = 2797010
    init = torch.tensor(init_vector(91, n, 0.03))
    data = synthetic_mnist(92, 256, 64, device=DEV)
    crit = torch.nn.CrossEntropyLoss()

    class Net(MLP):
        def __init__(self):
            super().__init__()
            self.extra = torch.nn.Linear(4, 4)   # used on some steps only
            self.use_extra = True

        def forward(self, x):
            out = super().forward(x)
            if self.use_extra:
                out = out + 0.0 * self.extra(torch.ones(1, 4, device=x.device)).sum()
            return out

    def run(overlap):
        torch.manual_seed(0)
        net = Net()
        with torch.no_grad():
            torch.nn.utils.vector_to_parameters(
                torch.cat([init, torch.zeros(20)]), net.parameters())
        net = net.to(DEV)
        model = csghmc.Model(30000.0, prior_sig=1.0, momentum_decay=0.18)
        model.noise_mode, model.seed, model.overlap = "philox", 3, overlap
        st = None
        m1 = m2 = None
        for ep in range(2):
            for k, (x, y) in enumerate(data):
                net.use_extra = k != 2
                coll = None
                if k == 1:
                    st = model.flat
                    if m1 is None:
                        m1 = torch.empty(st.n, device=DEV)
                        m2 = torch.empty(st.n, device=DEV)
                        coll = (1, m1, m2, 1.0)        # COLLECT_WELFORD_INIT
                    else:
                        coll = (2, m1, m2, 2.0)        # COLLECT_WELFORD
                model(x, y, net, None, crit, [1e-2, 2e-2], 1.0, 0.5, should_sample=k % 2 == 1,
                      collect=coll)
        torch.cuda.synchronize()
        return model, m1, m2

    mo, m1o, m2o = run(True)
    ms, m1s, m2s = run(False)
    assert mo._ovl_plan is not None and len(mo._ovl_plan[1]) >= 4
    assert torch.equal(mo.flat.theta, ms.flat.theta)
    assert torch.equal(mo.flat.mom, ms.flat.mom)
    assert torch.equal(m1o, m1s) and torch.equal(m2o, m2s)
