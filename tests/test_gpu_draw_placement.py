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
        monkeypatch.delenv("BDL_PLACEMENT", raising=False)
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
    ch = d1.placement["chunks"]                    # and a chunk-built vector competed
    assert ch is not None and "error" not in ch, ch
    assert d1.placement["kept"] in ("torch", "chunks")
    if d1.placement["kept"] == "chunks":
        # kept only when faster (info values are rounded to 0.1 us: a tie can show)
        assert ch["chosen_ms"] <= min(d1.placement["torch_ms"])
    for a, b in zip(th0, th1):
        assert torch.equal(a, b)
    for a, b in zip(outs0, outs1):
        assert torch.equal(a, b)
    # the network computes with the buffer the kernel writes
    lo, hi = d1.theta.data_ptr(), d1.theta.data_ptr() + 4 * d1.theta.numel()
    assert all(lo <= p.data_ptr() < hi for p in d1.net.parameters())


def test_place_one_vector_is_parked_and_reused(monkeypatch):
    """placement.place_one (the draw's chunk-built output, forced to win with
    beat_ms=None): the draw into it equals the draw into a plain allocation bit
    for bit; when it dies it is parked, and the next call with the same key
    takes back the same mapping (no search, no new address space)."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd import placement as P
    from bayesdll_amd.flat import PLACEMENT_MIN_ELEMS, _time_launch
    n = PLACEMENT_MIN_ELEMS + 1000   # one chunk, rounded up past n
    g = torch.Generator(device="cuda").manual_seed(5)
    mean = torch.randn(n, device="cuda", generator=g) * 0.02
    m2 = torch.rand(n, device="cuda", generator=g) * 1e-4

    def launcher(b, off=0):
        m = b.numel()
        return lambda: K.posterior_sample(b, mean[off:off + m], m2[off:off + m],
                                          var_mode=L.VAR_WELFORD, ratio=4.0, seed=3, chain=1,
                                          step=2)
    key = ("draw_test", n)
    buf, info = P.place_one(n, "cuda", launcher, lambda f: _time_launch(f, "cuda", 3),
                            budget_bytes=1 << 34, pool_key=key)
    assert buf is not None and buf.numel() == n and not info["reused"], info
    assert len(info["chunk_ms"]) == info["chunks_allocated"] and info["chunks_per_vector"] == 1
    launcher(buf)()
    ref = torch.empty(n, device="cuda")
    launcher(ref)()
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    ptr, va = buf.data_ptr(), P.va_reserved_bytes()
    del buf
    buf2, info2 = P.place_one(n, "cuda", launcher, lambda f: _time_launch(f, "cuda", 3),
                              budget_bytes=1 << 34, pool_key=key)
    assert info2["reused"] and buf2.data_ptr() == ptr
    assert P.va_reserved_bytes() == va
    launcher(buf2)()
    torch.cuda.synchronize()
    assert torch.equal(buf2, ref)
    del buf2
    P.release_pool()
