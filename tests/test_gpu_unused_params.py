"""Parameters that receive no gradient in a step are skipped, as in the
reference (`net.zero_grad()` leaves their .grad None and every Model loop
tests `if p.grad is not None`, e.g. methods/csghmc.py:749, methods/sgld.py:471):
no update, no noise draw, no SGD step — while the per-step run table still
lets the fused kernel sweep the whole flat vector."""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


class Net(nn.Module):
    """fc1 -> (branch A or branch B) -> classifier; the branch not taken in a
    step gets no gradient."""

    readout_name = "classifier"

    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(20, 32)
        self.branch_a = nn.Linear(32, 32)
        self.branch_b = nn.Linear(32, 32)
        self.classifier = nn.Linear(32, 5)
        self.use_a = True

    def forward(self, x):
        h = torch.relu(self.fc1(x))
        h = torch.relu(self.branch_a(h) if self.use_a else self.branch_b(h))
        return self.classifier(h)


@pytest.mark.parametrize("method", ["csghmc", "sgld"])
def test_unused_branch_is_skipped_like_the_reference(method):
    import importlib
    from oracle import sgmcmc_oracle as O
    mod = importlib.import_module(f"bayesdll_amd.{method}")
    from bayesdll_amd.sgld import FusedSGD
    dev = "cuda"
    torch.manual_seed(0)
    base = Net().to(dev)
    prior = Net().to(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    data = [(torch.randn(16, 20, device=dev, generator=g),
             torch.randint(0, 5, (16,), device=dev, generator=g)) for _ in range(6)]
    lrs, N, nd, psig, alpha, mu = [1e-2, 2e-2], 100.0, 0.5, 1.0, 0.2, 0.5
    crit = nn.CrossEntropyLoss()

    def clone(net):
        c = Net().to(dev)
        c.load_state_dict(net.state_dict())
        return c

    # reference: zero_grad (to None) + backward; update only p.grad is not None
    ref = clone(base)
    names = [nm for nm, _ in ref.named_parameters()]
    opt = torch.optim.SGD([{"params": [p for nm, p in ref.named_parameters() if "classifier" not in nm], "lr": lrs[0]},
                           {"params": [p for nm, p in ref.named_parameters() if "classifier" in nm], "lr": lrs[1]}],
                          momentum=mu if method == "sgld" else 0.0)
    moms = {nm: torch.zeros_like(p) for nm, p in ref.named_parameters()}
    torch.manual_seed(7)
    for k, (x, y) in enumerate(data):
        ref.use_a = k % 3 != 2
        loss = crit(ref(x), y)
        ref.zero_grad()
        loss.backward()
        live = [(nm, p, p0) for (nm, p), p0 in zip(ref.named_parameters(), prior.parameters())
                if p.grad is not None]
        with torch.no_grad():
            eps = [torch.randn_like(p) for _, p, _ in live]
            ps = [p for _, p, _ in live]
            nms = [nm for nm, _, _ in live]
            if method == "csghmc":
                new = O.csghmc_update(ps, [p.grad for p in ps], [moms[nm] for nm in nms], nms,
                                      "classifier", lrs, psig, alpha, N, nd, True, eps)
                moms.update(zip(nms, new))
                continue
            g2 = O.sgld_model(ps, [p0 for _, _, p0 in live], [p.grad for p in ps], nms,
                              "classifier", lrs, psig, "informative", N, nd, eps)
            for p, gg in zip(ps, g2):
                p.grad = gg
        opt.step()
    ref_vec = torch.nn.utils.parameters_to_vector(ref.parameters()).detach()

    # product
    net = clone(base)
    if method == "csghmc":
        model = mod.Model(N, prior_sig=psig, momentum_decay=alpha)
    else:
        model = mod.Model(N, prior_sig=psig)
    model.noise_mode, model.div_mode = "torch", "recip"
    opt = torch.optim.SGD([{"params": [p for nm, p in net.named_parameters() if "classifier" not in nm], "lr": lrs[0]},
                           {"params": [p for nm, p in net.named_parameters() if "classifier" in nm], "lr": lrs[1]}],
                          momentum=mu if method == "sgld" else 0.0)
    fsgd = FusedSGD(opt, mu if method == "sgld" else 0.0)
    torch.manual_seed(7)
    b_before = None
    for k, (x, y) in enumerate(data):
        net.use_a = k % 3 != 2
        if k == 2:
            b_before = net.branch_a.weight.detach().clone()
        if method == "csghmc":
            model(x, y, net, prior, crit, lrs, 1.0, nd, should_sample=True)
        else:
            model(x, y, net, prior, crit, lrs, 1.0, nd, sgd=fsgd)
        if k == 2:  # branch_a unused in this step: untouched, and a skip run in the table
            assert torch.equal(net.branch_a.weight.detach(), b_before)
            names = [nm for nm, _ in net.named_parameters()]
            assert not model.flat.has_grad(names.index("branch_a.weight"))
            assert model.flat.has_grad(names.index("classifier.weight"))
    torch.cuda.synchronize()
    got = model.flat.theta
    rel = ((got - ref_vec).abs().max() / ref_vec.abs().max()).item()
    assert rel <= 1e-5, rel
    np.testing.assert_allclose(got.cpu().numpy(), ref_vec.cpu().numpy(), rtol=1e-5, atol=1e-7)
