"""The posterior-draw output buffer choice (flat.draw_buffer, used by
_runner.PosteriorDraw before its first Philox draw) changes where the draw is
written, never what: the drawn parameters, and the network's outputs with
them, equal those of an unplaced draw bit for bit, and the network's
parameters are views of the buffer the kernel writes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _net():
    torch.manual_seed(3)
    # 4097 x 4100 + 4097 = 16,801,797 parameters: above PLACEMENT_MIN_ELEMS
    return torch.nn.Sequential(torch.nn.Linear(4100, 4097)).cuda()


def _draws(monkeypatch, placement):
    from bayesdll_amd import _lib as L
    from bayesdll_amd._runner import PosteriorDraw
    if placement:
        monkeypatch.setenv("BDL_PLACEMENT", "search")  # opt-in
    else:
        monkeypatch.setenv("BDL_PLACEMENT", "0")
    net = _net()
    n = sum(p.numel() for p in net.parameters())
    g = torch.Generator(device="cuda").manual_seed(1)
    mean = torch.randn(n, device="cuda", generator=g) * 0.02
    m2 = torch.rand(n, device="cuda", generator=g) * 1e-4
    d = PosteriorDraw(net, "philox", seed=11, chain=2)
    x = torch.randn(8, 4100, device="cuda", generator=g)
    outs, thetas = [], []
    for _ in range(3):
        d.draw(mean, m2, L.VAR_WELFORD, 4.0)
        with torch.no_grad():
            outs.append(d.net(x).clone())
        thetas.append(d.theta.clone())
    torch.cuda.synchronize()
    return d, outs, thetas


def test_draw_buffer_choice_changes_nothing_but_the_buffer(monkeypatch):
    d0, outs0, th0 = _draws(monkeypatch, placement=False)
    d1, outs1, th1 = _draws(monkeypatch, placement=True)
    assert d0.placement == {}                      # BDL_PLACEMENT=0: plain allocation kept
    assert len(d1.placement["torch_ms"]) == 3      # three plain candidates timed
    assert d1.placement["torch_ms"][d1.placement["kept"]] == min(d1.placement["torch_ms"])
    for a, b in zip(th0, th1):
        assert torch.equal(a, b)
    for a, b in zip(outs0, outs1):
        assert torch.equal(a, b)
    # the network computes with the buffer the kernel writes
    lo, hi = d1.theta.data_ptr(), d1.theta.data_ptr() + 4 * d1.theta.numel()
    assert all(lo <= p.data_ptr() < hi for p in d1.net.parameters())
