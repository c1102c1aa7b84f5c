"""Kernel-level GPU tests of libbdl_sgmcmc.so through the C-ABI.

* full-size parity (ViT-L/32: 306,535,400 params, 296 tensors): one fused step
  vs the reference's per-tensor op sequence executed with torch ops on the same
  GPU, same noise — bit-exact (the kernel rounds every op where torch does);
* edge sizes (n = 1, 3, 4, 5, 17, 4097, ...) and run boundaries inside float4
  groups, for every method;
* Philox noise: determinism, key separation, moments, KS vs N(0,1), and that
  the step in Philox mode equals the step fed the same draws as a buffer;
* posterior-sample and moment kernels vs their torch formulas.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _state(segments, readout, bias="informative", seed=0, **kw):
    from bayesdll_amd.flat import FlatState
    st = FlatState.from_segments(segments, readout, bias=bias, device=DEV, **kw)
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    st.theta.normal_(0.0, 0.02, generator=g)
    st.grad.normal_(0.0, 1e-3, generator=g)
    if st.mom is not None:
        st.mom.normal_(0.0, 1e-4, generator=g)
    if st.prior is not None:
        st.prior.normal_(0.0, 0.02, generator=g)
    if st.noise is not None:
        st.noise.normal_(generator=g)
    return st


# ------------------------------------------------------------ torch references
def ref_csghmc(st, lrs, ns, alpha, prior_sig, add_noise):
    """methods/csghmc.py:759-778 with torch ops, per tensor, on the device."""
    th, v = st.theta.clone(), st.mom.clone()
    for (o, k, a) in zip(st.offsets, st.numels, st.attrs):
        h = 1 if a & 1 else 0
        p, g, vv = th[o:o + k], st.grad[o:o + k], v[o:o + k]
        gu = g + prior_sig * p
        nz = ns[h] * st.noise[o:o + k]
        vn = vv * (1 - alpha) - lrs[h] * gu
        if add_noise:
            vn = vn + nz
        vv.copy_(vn)
        p.add_(vn)
    return th, v


def ref_sgld(st, lrs, ns, sigma, N, mu, first, recip):
    """methods/sgld.py:476-484 + SGD(momentum) with torch ops on the device."""
    th, buf = st.theta.clone(), st.mom.clone()
    for (o, k, a) in zip(st.offsets, st.numels, st.attrs):
        h = 1 if a & 1 else 0
        p, p0, g = th[o:o + k], st.prior[o:o + k], st.grad[o:o + k]
        nz = ns[h] * st.noise[o:o + k]
        if a & 2:
            d = p - p0
            if recip:  # torch's HIP kernel: x * fl(1/s)
                gp = g + (d / (sigma ** 2) / N + nz)
            else:
                s2 = torch.tensor(np.float32(sigma ** 2))
                nn_ = torch.tensor(np.float32(N))
                gp = g + ((d.cpu() / s2 / nn_).to(DEV) + nz)
        else:
            gp = g + nz
        b = buf[o:o + k]
        if mu != 0:
            if first:
                b.copy_(gp)
            else:
                b.mul_(mu).add_(gp)
            gp = b
        p.add_(gp, alpha=-lrs[h])
    return th, buf


# ------------------------------------------------------------------- tests
def test_full_size_vit_csghmc_step_bitexact_vs_torch():
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.shapes import vit_l_32
    segs, readout = vit_l_32()
    st = _state(segs, readout, need_noise=True)
    assert st.n == 306_535_400 and len(segs) == 296
    lrs, alpha, psig = (1e-4, 1e-2), 0.18, 1.0
    N, nd = 1840.0, 0.01
    ns = [nd * np.sqrt(2 * alpha * lr) / N for lr in lrs]
    for add_noise in (False, True):
        th_ref, v_ref = ref_csghmc(st, lrs, ns, alpha, psig, add_noise)
        K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns,
                      noise_mode=L.NOISE_BUFFER if add_noise else L.NOISE_NONE,
                      one_minus_alpha=1 - alpha, prior_sig=psig)
        torch.cuda.synchronize()
        assert torch.equal(st.theta, th_ref)
        assert torch.equal(st.mom, v_ref)


def test_full_size_vit_sgld_uninformative_many_runs():
    """296 tensors with uninformative biases -> ~300 runs; the recip-division
    path is bit-exact with torch's own device kernels."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.shapes import vit_l_32
    segs, readout = vit_l_32()
    st = _state(segs, readout, bias="uninformative", need_prior=True, need_noise=True, seed=1)
    assert st.nruns > 290
    lrs, sigma, N, nd, mu = (1e-4, 1e-2), 1.0, 1840.0 * 1e3, 0.01, 0.5
    ns = [nd * np.sqrt(2 / (N * lr)) for lr in lrs]
    for first in (True, False):
        th_ref, b_ref = ref_sgld(st, lrs, ns, sigma, N, mu, first, recip=True)
        K.sgmcmc_step(st, L.SGLD, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_BUFFER,
                      prior_sig=sigma, sigma2=sigma ** 2, n_data=N, mu=mu, first_step=first,
                      momentum=True, div_mode="recip")
        torch.cuda.synchronize()
        # add_(alpha=-lr) may or may not be contracted to an FMA by torch's
        # device kernel: allow 1 ulp on theta, exact on the buffer
        assert torch.equal(st.mom, b_ref)
        np.testing.assert_allclose(st.theta.cpu().numpy(), th_ref.cpu().numpy(), rtol=2e-7,
                                   atol=1e-12)
        st.theta.copy_(th_ref)


SMALL = [1, 3, 4, 5, 7, 17, 64, 1023, 4097, 65537]


@pytest.mark.parametrize("n", SMALL)
def test_edge_sizes_csghmc_and_sgld(n):
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    # split n into odd-sized tensors with a trailing head + bias
    rng = np.random.default_rng(n)
    cuts = sorted(set(rng.integers(1, n, size=min(5, max(n - 1, 0))).tolist())) if n > 1 else []
    bounds = [0] + cuts + [n]
    segs = []
    for i in range(len(bounds) - 1):
        k = bounds[i + 1] - bounds[i]
        name = ("fc." if i == len(bounds) - 2 else f"l{i}.") + ("bias" if i % 2 else "weight")
        segs.append((name, (k,)))
    st = _state(segs, "fc", need_noise=True, need_prior=True)
    lrs, alpha = (0.01, 0.05), 0.1
    ns = [0.3, 0.7]
    th_ref, v_ref = ref_csghmc(st, lrs, ns, alpha, 0.5, True)
    K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_BUFFER,
                  one_minus_alpha=1 - alpha, prior_sig=0.5)
    torch.cuda.synchronize()
    assert torch.equal(st.theta, th_ref) and torch.equal(st.mom, v_ref)

    st2 = _state(segs, "fc", bias="uninformative", need_noise=True, need_prior=True, seed=5)
    th_ref, b_ref = ref_sgld(st2, lrs, ns, 0.8, 50.0, 0.9, False, recip=False)
    K.sgmcmc_step(st2, L.SGLD, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_BUFFER, sigma2=0.8 ** 2,
                  n_data=50.0, mu=0.9, momentum=True, first_step=False, div_mode="true")
    torch.cuda.synchronize()
    assert torch.equal(st2.mom, b_ref)
    np.testing.assert_allclose(st2.theta.cpu().numpy(), th_ref.cpu().numpy(), rtol=2e-7, atol=0)


def test_zero_length_is_a_noop():
    from bayesdll_amd import _lib as L
    a = L.StepArgs()
    a.n = 0
    assert L.lib().bdl_sgmcmc_step(a, None) == 0


def test_philox_determinism_and_key_separation():
    from bayesdll_amd.kernels import philox_normal
    n = 1 << 20
    a = philox_normal(n, 42, 0, 7)
    b = philox_normal(n, 42, 0, 7)
    assert torch.equal(a, b)
    for other in (philox_normal(n, 43, 0, 7), philox_normal(n, 42, 1, 7),
                  philox_normal(n, 42, 0, 8)):
        c = torch.corrcoef(torch.stack([a, other]))[0, 1].item()
        assert abs(c) < 6 / math.sqrt(n)
        assert not torch.equal(a, other)
    # prefix consistency: element i does not depend on n
    assert torch.equal(philox_normal(1001, 42, 0, 7), a[:1001])


def test_philox_moments_and_ks():
    from scipy import stats
    from bayesdll_amd.kernels import philox_normal
    n = 1 << 22
    z = philox_normal(n, 1234, 3, 99).double()
    assert abs(z.mean().item()) < 5 / math.sqrt(n)
    assert abs(z.var().item() - 1) < 5 * math.sqrt(2 / n)
    assert abs(((z ** 3).mean()).item()) < 5 * math.sqrt(15 / n)
    assert abs(((z ** 4).mean()).item() - 3) < 5 * math.sqrt(96 / n)
    assert torch.isfinite(z).all()
    ks = stats.kstest(z[:1 << 20].cpu().numpy(), "norm")
    assert ks.pvalue > 1e-4, ks


def test_philox_step_equals_buffer_step():
    """The step in Philox mode consumes exactly bdl_philox_normal's stream."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.shapes import mlp_mnist
    segs, readout = mlp_mnist()
    a = _state(segs, readout, need_noise=True, seed=3)
    b = _state(segs, readout, need_noise=True, seed=3)
    kw = dict(lrs=(1e-3, 1e-2), noise_scale=(1e-2, 3e-2), one_minus_alpha=0.82, prior_sig=1.0,
              seed=42, chain=5, step=123)
    K.sgmcmc_step(a, L.CSGHMC, noise_mode=L.NOISE_PHILOX, **kw)
    b.noise.copy_(K.philox_normal(b.n, 42, 5, 123))
    K.sgmcmc_step(b, L.CSGHMC, noise_mode=L.NOISE_BUFFER, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a.theta, b.theta) and torch.equal(a.mom, b.mom)


def test_fused_welford_and_running_mean_match_torch():
    """Collect variants: the moments use the UPDATED theta, as the reference
    (parameters_to_vector after the step)."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.shapes import mlp_mnist
    segs, readout = mlp_mnist()
    st = _state(segs, readout, need_noise=True, seed=9)
    m1 = torch.randn(st.n, device=DEV)
    m2 = torch.rand(st.n, device=DEV)
    kw = dict(lrs=(1e-3, 1e-2), noise_scale=(1e-2, 3e-2), one_minus_alpha=0.82, prior_sig=1.0)
    th_ref, _ = ref_csghmc(st, kw["lrs"], kw["noise_scale"], 0.18, 1.0, True)
    e1, e2 = m1.clone(), m2.clone()
    d = th_ref - e1
    e1 += d / 5
    d2 = th_ref - e1
    e2 += d * d2
    K.sgmcmc_step(st, L.CSGHMC, noise_mode=L.NOISE_BUFFER, collect=L.COLLECT_WELFORD, mom1=m1,
                  mom2=m2, collect_a=5.0, div_mode="recip", **kw)
    torch.cuda.synchronize()
    assert torch.equal(st.theta, th_ref)
    assert torch.equal(m1, e1) and torch.equal(m2, e2)

    x = torch.randn(st.n, device=DEV)
    a1, a2 = torch.randn(st.n, device=DEV), torch.rand(st.n, device=DEV)
    r1 = (x + 3 * a1) / 4
    r2 = (x ** 2 + 3 * a2) / 4
    K.moments_update(x, a1, a2, L.COLLECT_MEAN, 3.0, 4.0, div_mode="recip")
    torch.cuda.synchronize()
    assert torch.equal(a1, r1) and torch.equal(a2, r2)
    b1, b2 = torch.empty_like(x), torch.empty_like(x)
    K.moments_update(x, b1, b2, L.COLLECT_MEAN_INIT)
    torch.cuda.synchronize()
    assert torch.equal(b1, x * 1.0) and torch.equal(b2, x ** 2)


def test_posterior_sample_matches_torch_formula():
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    n = 1_000_003
    m1 = torch.randn(n, device=DEV)
    m2 = m1 ** 2 + torch.rand(n, device=DEV) * 0.1
    m2[::7] = m1[::7] ** 2 - 1e-3  # negative variance -> clamp to 1e-12
    eps = torch.randn(n, device=DEV)
    ratio = 5 / 4
    var = (ratio * (m2 - m1 ** 2)).clamp_(min=1e-12)
    ref = m1 + var.sqrt() * eps
    out = torch.empty_like(m1)
    K.posterior_sample(out, m1, m2, var_mode=L.VAR_RAW_MOMENTS, ratio=ratio, noise=eps)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # Welford form and single-sample form
    var = (m2 / 3).clamp_(min=1e-12)
    K.posterior_sample(out, m1, m2, var_mode=L.VAR_WELFORD, ratio=3.0, noise=eps)
    torch.cuda.synchronize()
    # torch divides by the scalar as x*(1/3) on the device, the kernel as x/3:
    # <= 1 ulp on var, compared on the whole vector
    want = (m1 + var.sqrt() * eps).cpu().numpy().astype(np.float64)
    got = out.cpu().numpy().astype(np.float64)
    assert np.max(np.abs(got - want)) / np.max(np.abs(want)) < 1e-6
    K.posterior_sample(out, m1, None, var_mode=L.VAR_GIVEN, noise=eps)
    torch.cuda.synchronize()
    assert torch.equal(out, m1 + torch.full_like(m1, 1e-12).sqrt() * eps)


@pytest.mark.parametrize("floor", [1e-12, 2.0 ** -96, 2.0 ** -97, 1e-40, 0.0])
def test_posterior_sample_sqrt_at_every_floor(floor):
    """The sample sweep takes v_sqrt_f32 + residual correction when the floor
    is >= 2^-96 and the compiler's full sqrtf otherwise: both give torch's
    device sqrt bit for bit over variances spanning zero, subnormals, the
    2^-96 boundary, large values and inf (NaN stays NaN)."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(5)
    n = (1 << 20) + 7  # a partial last iteration and a partial last float4 group
    e = torch.randint(-149, 128, (n,), device=DEV, generator=g).float()
    var = torch.rand(n, device=DEV, generator=g) * torch.exp2(e)  # every binade, subnormals too
    var[:64] = torch.tensor([0.0, 2.0 ** -96, 2.0 ** -97, 2.0 ** -95, 1e-45, float("inf"),
                             float("nan"), 3.4e38] * 8, device=DEV)
    m1 = torch.randn(n, device=DEV, generator=g)
    eps = torch.randn(n, device=DEV, generator=g)
    out = torch.empty_like(m1)
    K.posterior_sample(out, m1, var, var_mode=L.VAR_GIVEN, var_floor=floor, noise=eps)
    v = var.clone()
    keep = torch.isnan(v)
    v = torch.where(keep, v, v.clamp(min=torch.tensor(floor, dtype=torch.float32).item()))
    want = m1 + v.sqrt() * eps
    torch.cuda.synchronize()
    nan = torch.isnan(want)
    assert torch.equal(torch.isnan(out), nan)
    assert torch.equal(out[~nan].view(torch.int32), want[~nan].view(torch.int32))
    # and with Philox noise: the stream the buffer mode is fed by bdl_philox_normal
    K.posterior_sample(out, m1, var, var_mode=L.VAR_GIVEN, var_floor=floor, seed=9, chain=2, step=4)
    z = K.philox_normal(n, 9, 2, 4, device=DEV)
    want = m1 + v.sqrt() * z
    torch.cuda.synchronize()
    nan = torch.isnan(want)
    assert torch.equal(torch.isnan(out), nan)
    assert torch.equal(out[~nan].view(torch.int32), want[~nan].view(torch.int32))


# ------------------------------------------------------- clipped SGLD (csgld)
def ref_clip_sgld(st, max_norm, lrs, ns, sigma, N, mu, first):
    """methods/csgld.py:250-253 on the device with torch ops: the sampler
    gradient of csgld.py:665-680 per tensor, torch.nn.utils.clip_grad_norm_
    over the tensors that have a gradient, then SGD(momentum)."""
    th, buf = st.theta.clone(), st.mom.clone()
    plist, segs = [], []
    for (o, k, a) in zip(st.offsets, st.numels, st.attrs):
        if a & 4:  # no .grad: not in the norm, not stepped
            if first and mu != 0:
                # torch SGD holds no buffer for it; the flat buffer holds 0, so a
                # later first gradient gives buf = mu*0 + g == clone(g)
                buf[o:o + k].zero_()
            continue
        h = 1 if a & 1 else 0
        p, p0, g = th[o:o + k], st.prior[o:o + k], st.grad[o:o + k]
        nz = ns[h] * st.noise[o:o + k]
        gp = g + ((p - p0) / (sigma ** 2) / N + nz) if a & 2 else g + nz
        w = torch.nn.Parameter(torch.empty_like(gp))
        w.grad = gp
        plist.append(w)
        segs.append((o, k, h))
    total = torch.nn.utils.clip_grad_norm_(plist, max_norm)
    for w, (o, k, h) in zip(plist, segs):
        gp, b = w.grad, buf[o:o + k]
        if mu != 0:
            if first:
                b.copy_(gp)
            else:
                b.mul_(mu).add_(gp)
            gp = b
        th[o:o + k].add_(gp, alpha=-lrs[h])
    return th, buf, float(total)


def _vec_rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _freeze(st, idx):
    from bayesdll_amd.flat import build_runs, segment_attrs
    st.requires_grad = [i not in idx for i in range(len(st.names))]
    st.attrs = segment_attrs(st.names, st.readout_name, st.bias, st.requires_grad)
    st.runs = build_runs(st.offsets, st.numels, st.attrs, st.n).to(st.device)
    st.nruns = int(st.runs.shape[0])


def _clipped_case(st, scale_vs_norm, first, mu=0.5, lrs=(1e-3, 2e-3), sigma=0.8, N=500.0, nd=0.05):
    from bayesdll_amd import kernels as K
    from bayesdll_amd import _lib as L
    ns = [nd * np.sqrt(2 / (N * lr)) for lr in lrs]
    _, _, total = ref_clip_sgld(st, 1e30, lrs, ns, sigma, N, mu, first)
    max_norm = scale_vs_norm * total
    th_ref, b_ref, _ = ref_clip_sgld(st, max_norm, lrs, ns, sigma, N, mu, first)
    th0, b0 = st.theta.clone(), st.mom.clone()
    ws = K.sgld_step_clipped(st, max_norm, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_BUFFER,
                             sigma2=sigma ** 2, n_data=N, mu=mu, first_step=first,
                             momentum=mu != 0, div_mode="recip")
    torch.cuda.synchronize()
    norm, coef = ws[0].item(), ws[1].item()
    assert abs(norm - total) <= 1e-5 * total
    assert coef == pytest.approx(min(1.0, max_norm / (total + 1e-6)), rel=1e-5)
    assert _vec_rel(st.theta, th_ref) <= 1e-5
    assert _vec_rel(st.mom, b_ref) <= 1e-5
    frozen = [(o, k) for o, k, a in zip(st.offsets, st.numels, st.attrs) if a & 4]
    for o, k in frozen:  # theta untouched; buffer untouched after the first step
        assert torch.equal(st.theta[o:o + k], th0[o:o + k])
        assert torch.equal(st.mom[o:o + k], b_ref[o:o + k])
    st.theta.copy_(th0)
    st.mom.copy_(b0)
    return norm, coef


@pytest.mark.parametrize("n", [1, 5, 17, 4097, 65537, 1 << 20])
def test_clipped_sgld_edge_sizes_and_frozen_tensors(n):
    rng = np.random.default_rng(n + 7)
    cuts = sorted(set(rng.integers(1, n, size=min(7, max(n - 1, 0))).tolist())) if n > 1 else []
    bounds = [0] + cuts + [n]
    segs = []
    for i in range(len(bounds) - 1):
        name = ("fc." if i == len(bounds) - 2 else f"l{i}.") + ("bias" if i % 2 else "weight")
        segs.append((name, (bounds[i + 1] - bounds[i],)))
    st = _state(segs, "fc", bias="uninformative", need_noise=True, need_prior=True, seed=n)
    if len(segs) > 2:
        _freeze(st, {1})
    for scale in (0.5, 2.0):
        for first in (True, False):
            _, coef = _clipped_case(st, scale, first)
            assert (coef < 1.0) == (scale < 1.0)


def test_clipped_sgld_full_size_vit():
    """ViT-L/32 (306,535,400 params, 296 tensors): clipping active and inactive."""
    from bayesdll_amd.shapes import vit_l_32
    segs, readout = vit_l_32()
    st = _state(segs, readout, need_prior=True, need_noise=True, seed=3)
    _clipped_case(st, 0.25, False)
    _clipped_case(st, 4.0, True, mu=0.0)


def test_clipped_sgld_philox_equals_buffer():
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    segs = [("l0.weight", (300, 301)), ("l0.bias", (301,)), ("fc.weight", (10, 301)),
            ("fc.bias", (10,))]
    st = _state(segs, "fc", need_noise=True, need_prior=True, seed=11)
    th0, b0 = st.theta.clone(), st.mom.clone()
    kw = dict(lrs=(1e-3, 1e-2), noise_scale=(0.3, 0.1), sigma2=1.0, n_data=100.0, mu=0.9,
              momentum=True, first_step=True, seed=1234, chain=2, step=9)
    ws = K.sgld_step_clipped(st, 5.0, noise_mode=L.NOISE_PHILOX, **kw)
    torch.cuda.synchronize()
    th_p, b_p, ws_p = st.theta.clone(), st.mom.clone(), ws[:2].clone()
    st.theta.copy_(th0)
    st.mom.copy_(b0)
    st.noise.copy_(K.philox_normal(st.n, 1234, 2, 9))
    ws = K.sgld_step_clipped(st, 5.0, noise_mode=L.NOISE_BUFFER, **kw)
    torch.cuda.synchronize()
    assert ws_p[1].item() < 1.0
    assert torch.equal(ws[:2], ws_p)
    assert torch.equal(st.theta, th_p) and torch.equal(st.mom, b_p)


def test_clipped_sgld_rejects_bad_arguments():
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    st = _state([("fc.weight", (64,))], "fc", need_noise=True, need_prior=True)
    with pytest.raises(RuntimeError, match="max_norm"):
        K.sgld_step_clipped(st, 0.0, lrs=(1e-3, 1e-3), noise_scale=(0.1, 0.1),
                            noise_mode=L.NOISE_BUFFER)
    with pytest.raises(RuntimeError, match="GRAD_READY"):
        K.sgld_step_clipped(st, 1.0, lrs=(1e-3, 1e-3), noise_scale=(0.1, 0.1),
                            noise_mode=L.NOISE_BUFFER, grad_ready=True)


# ----------------------------------------------- Adam-preconditioned SGHMC
def ref_adam(st, m, v, buf, *, lrs, alpha, b1, b2, aeps, t, sigma, N, nd, temp, grad_is_mom, mu,
             first, grad_only=False):
    """methods/adam_sghmc.py:512-553 / adam_csghmc.py:819-860 + SGD with torch
    ops on the device (per tensor, the reference's op order)."""
    th, vm_all, m_all, v_all, b_all = (st.theta.clone(), st.mom.clone(), m.clone(), v.clone(),
                                       None if buf is None else buf.clone())
    g_all = st.grad.clone()
    for (o, k, a) in zip(st.offsets, st.numels, st.attrs):
        if a & 4:
            if first and b_all is not None and mu != 0:
                b_all[o:o + k].zero_()
            continue
        lr = lrs[1] if a & 1 else lrs[0]
        p, p0, g = th[o:o + k], st.prior[o:o + k], st.grad[o:o + k]
        gs = g / temp
        gU = gs + (p - p0) / (sigma ** 2) / N if a & 2 else gs
        mm = b1 * m_all[o:o + k] + (1 - b1) * gU
        vv = b2 * v_all[o:o + k] + (1 - b2) * (gU * gU)
        m_hat = mm / (1 - b1 ** t)
        v_hat = vv / (1 - b2 ** t)
        pg = m_hat / (torch.sqrt(v_hat) + aeps)
        pt = 1.0 / (torch.sqrt(v_hat) + aeps)
        ns = nd * torch.sqrt(2 * alpha * pt / N)
        vm = vm_all[o:o + k] * (1 - alpha) + lr * pg + ns * st.noise[o:o + k]
        gp = vm.clone() if grad_is_mom else g + vm.clone()
        m_all[o:o + k] = mm
        v_all[o:o + k] = vv
        vm_all[o:o + k] = vm
        if grad_only:
            g_all[o:o + k] = gp
            continue
        d = gp
        if mu != 0:
            bb = b_all[o:o + k]
            if first:
                bb.copy_(gp)
            else:
                bb.mul_(mu).add_(gp)
            d = bb
        p.add_(d, alpha=-lr)
    return th, vm_all, m_all, v_all, b_all, g_all


def _adam_case(st, *, grad_is_mom, mu, first, t, temp=1.0, grad_only=False, nd=0.05):
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    gen = torch.Generator(device=DEV)
    gen.manual_seed(t)
    m = torch.randn(st.n, device=DEV, generator=gen) * 1e-3
    v = torch.rand(st.n, device=DEV, generator=gen) * 1e-6
    buf = torch.randn(st.n, device=DEV, generator=gen) * 1e-3 if mu != 0 else None
    kw = dict(lrs=(1e-3, 2e-3), alpha=0.18, b1=0.9, b2=0.99, aeps=1e-8, t=t, sigma=0.8, N=500.0,
              nd=nd, temp=temp, grad_is_mom=grad_is_mom, mu=mu, first=first)
    th_r, vm_r, m_r, v_r, b_r, g_r = ref_adam(st, m, v, buf, grad_only=grad_only, **kw)
    g0 = st.grad.clone()
    K.adam_step(st, L.ADAM_SGHMC_GRAD if grad_only else L.ADAM_SGHMC, adam_m=m, adam_v=v,
                sgd_buf=buf, beta1=kw["b1"], beta2=kw["b2"], eps=kw["aeps"], t=t,
                momentum_decay=kw["alpha"], nd=nd, temperature=temp, grad_is_mom=grad_is_mom,
                lrs=kw["lrs"], noise_mode=L.NOISE_BUFFER, sigma2=kw["sigma"] ** 2,
                n_data=kw["N"], mu=mu, first_step=first, momentum=mu != 0, div_mode="recip")
    torch.cuda.synchronize()
    # the recip-division path rounds every op where torch's device kernels do
    assert torch.equal(m, m_r) and torch.equal(v, v_r)
    assert torch.equal(st.mom, vm_r)
    if grad_only:
        assert torch.equal(st.grad, g_r)
    else:
        if buf is not None:
            assert torch.equal(buf, b_r)
        # add_(alpha=-lr): FMA or not in torch's kernel -> allow 1 ulp
        np.testing.assert_allclose(st.theta.cpu().numpy(), th_r.cpu().numpy(), rtol=2.5e-7,
                                   atol=0)
        st.theta.copy_(th_r)
        st.grad.copy_(g0)
    st.mom.copy_(vm_r)


def test_adam_sghmc_full_size_vit_matches_torch():
    """ViT-L/32 (306,535,400 params): adam_sghmc (g + v_mom, SGD momentum) and
    adam_csghmc (v_mom, temperature, SGD momentum 0) rules, first and later steps."""
    from bayesdll_amd.shapes import vit_l_32
    segs, readout = vit_l_32()
    st = _state(segs, readout, bias="uninformative", need_prior=True, need_noise=True, seed=7)
    _adam_case(st, grad_is_mom=False, mu=0.5, first=True, t=1)
    _adam_case(st, grad_is_mom=False, mu=0.5, first=False, t=7)
    _adam_case(st, grad_is_mom=True, mu=0.0, first=False, t=3, temp=0.5)


@pytest.mark.parametrize("n", [1, 5, 17, 4097, 65537])
def test_adam_sghmc_edge_sizes_frozen_and_grad_only(n):
    rng = np.random.default_rng(n + 11)
    cuts = sorted(set(rng.integers(1, n, size=min(7, max(n - 1, 0))).tolist())) if n > 1 else []
    bounds = [0] + cuts + [n]
    segs = []
    for i in range(len(bounds) - 1):
        name = ("fc." if i == len(bounds) - 2 else f"l{i}.") + ("bias" if i % 2 else "weight")
        segs.append((name, (bounds[i + 1] - bounds[i],)))
    st = _state(segs, "fc", bias="uninformative", need_noise=True, need_prior=True, seed=n)
    if len(segs) > 2:
        _freeze(st, {1})
    _adam_case(st, grad_is_mom=False, mu=0.9, first=True, t=1)
    _adam_case(st, grad_is_mom=True, mu=0.0, first=False, t=2, temp=2.0)
    _adam_case(st, grad_is_mom=False, mu=0.0, first=False, t=4, grad_only=True)


def test_adam_step_philox_equals_buffer():
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    segs = [("l0.weight", (300, 301)), ("l0.bias", (301,)), ("fc.weight", (10, 301)),
            ("fc.bias", (10,))]
    outs = []
    for mode in ("philox", "buffer"):
        st = _state(segs, "fc", need_noise=True, need_prior=True, seed=11)
        m = torch.zeros(st.n, device=DEV)
        v = torch.zeros(st.n, device=DEV)
        if mode == "buffer":
            st.noise.copy_(K.philox_normal(st.n, 99, 1, 5))
        K.adam_step(st, L.ADAM_SGHMC, adam_m=m, adam_v=v, beta1=0.9, beta2=0.999, eps=1e-8, t=1,
                    momentum_decay=0.1, nd=1.0, lrs=(1e-3, 1e-2),
                    noise_mode=L.NOISE_PHILOX if mode == "philox" else L.NOISE_BUFFER,
                    sigma2=1.0, n_data=100.0, seed=99, chain=1, step=5)
        torch.cuda.synchronize()
        outs.append((st.theta.clone(), st.mom.clone(), m, v))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def ref_sghmc(st, lrs, ns, alpha, sigma, N):
    """methods/sghmc.py:482-510 + SGD(momentum 0) with torch ops on the device."""
    th, v = st.theta.clone(), st.mom.clone()
    for (o, k, a) in zip(st.offsets, st.numels, st.attrs):
        h = 1 if a & 1 else 0
        p, p0, g = th[o:o + k], st.prior[o:o + k], st.grad[o:o + k]
        gU = g + (p - p0) / (sigma ** 2) / N if a & 2 else g
        vn = v[o:o + k] * (1 - alpha) + lrs[h] * gU + ns[h] * st.noise[o:o + k]
        v[o:o + k] = vn
        p.add_(g + vn.clone(), alpha=-lrs[h])
    return th, v


def test_full_size_vit_sghmc_matches_torch():
    """ViT-L/32, uninformative biases (~300 runs), recip rounding: the SGHMC
    momentum is bit-exact vs torch ops on the same GPU, theta within 1 ulp
    (torch's add_(alpha=-lr) may or may not contract to an FMA)."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.shapes import vit_l_32
    segs, readout = vit_l_32()
    st = _state(segs, readout, bias="uninformative", need_prior=True, need_noise=True, seed=4)
    lrs, alpha, sigma, N, nd = (1e-4, 1e-2), 0.18, 1.0, 1840.0, 0.01
    ns = [nd * np.sqrt(2 * alpha / (N * lr)) for lr in lrs]
    th_ref, v_ref = ref_sghmc(st, lrs, ns, alpha, sigma, N)
    K.sgmcmc_step(st, L.SGHMC, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_BUFFER,
                  one_minus_alpha=1 - alpha, sigma2=sigma ** 2, n_data=N, div_mode="recip")
    torch.cuda.synchronize()
    assert torch.equal(st.mom, v_ref)
    np.testing.assert_allclose(st.theta.cpu().numpy(), th_ref.cpu().numpy(), rtol=2e-7, atol=1e-12)


def test_full_size_vit_csghmc_sample_and_welford_collect_bitexact():
    """The headline schedule's sample steps at full ViT-L/32 size: Philox noise
    + Welford first sample (m1 = theta, M2 = 0) then a Welford update with the
    reference's doubled count (Q2: n = 3 for the second sample), against
    torch ops on the device fed the same Philox draws — bit-exact."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.shapes import vit_l_32
    segs, readout = vit_l_32()
    st = _state(segs, readout, seed=21)
    st.noise = torch.empty_like(st.theta)
    m1, m2 = torch.empty_like(st.theta), torch.empty_like(st.theta)
    lrs, alpha, psig, N, nd = (1e-4, 1e-2), 0.18, 1.0, 1840.0, 0.01
    ns = [nd * np.sqrt(2 * alpha * lr) / N for lr in lrs]
    r1 = r2 = None
    for k, (collect, n_) in enumerate(((L.COLLECT_WELFORD_INIT, 1.0), (L.COLLECT_WELFORD, 3.0))):
        st.noise.copy_(K.philox_normal(st.n, 42, 0, 100 + k))
        th_ref, v_ref = ref_csghmc(st, lrs, ns, alpha, psig, True)
        if collect == L.COLLECT_WELFORD_INIT:
            r1, r2 = th_ref.clone(), torch.zeros_like(th_ref)
        else:
            d = th_ref - r1
            r1 = r1 + d / n_
            r2 = r2 + d * (th_ref - r1)
        K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                      one_minus_alpha=1 - alpha, prior_sig=psig, collect=collect, mom1=m1,
                      mom2=m2, collect_a=n_, seed=42, chain=0, step=100 + k, div_mode="recip")
        torch.cuda.synchronize()
        assert torch.equal(st.theta, th_ref) and torch.equal(st.mom, v_ref)
        assert torch.equal(m1, r1) and torch.equal(m2, r2)


@pytest.mark.parametrize("n", [1, 3, 4, 5, 7, 17, 1023, 2048, 2049, 4097, 65537, 1_000_003])
def test_moments_and_sample_kernels_edge_sizes(n):
    """Stand-alone moments (all four collect kinds, with and without m2) and
    posterior-sample kernels (every variance source, Philox and buffer noise)
    at sizes around the unrolled fast path's block iteration (256 lanes x U
    float4 groups) and the float4 tail, vs the torch-on-device formulas."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(n)
    x = torch.randn(n, device=DEV, generator=g)
    a1 = torch.randn(n, device=DEV, generator=g)
    a2 = torch.rand(n, device=DEV, generator=g)
    # Welford update, recip rounding (torch on the device: x * fl(1/5))
    m1, m2 = a1.clone(), a2.clone()
    K.moments_update(x, m1, m2, L.COLLECT_WELFORD, 5.0, div_mode="recip")
    d = x - a1
    e1 = a1 + d * (1.0 / 5.0)
    e2 = a2 + d * (x - e1)
    torch.cuda.synchronize()
    assert torch.equal(m1, e1) and torch.equal(m2, e2)
    # Welford init, with and without m2
    m1, m2 = torch.full_like(x, 7.0), torch.full_like(x, 7.0)
    K.moments_update(x, m1, m2, L.COLLECT_WELFORD_INIT)
    torch.cuda.synchronize()
    assert torch.equal(m1, x) and torch.equal(m2, torch.zeros_like(x))
    m1 = torch.full_like(x, 7.0)
    K.moments_update(x, m1, None, L.COLLECT_WELFORD_INIT)
    torch.cuda.synchronize()
    assert torch.equal(m1, x)
    # running mean, true division, with and without m2
    m1, m2 = a1.clone(), a2.clone()
    K.moments_update(x, m1, m2, L.COLLECT_MEAN, 3.0, 4.0, div_mode="true")
    torch.cuda.synchronize()
    r1 = ((x + 3 * a1).cpu().double() / 4).float()
    r2 = ((x * x + 3 * a2).cpu().double() / 4).float()
    assert torch.equal(m1.cpu(), r1) and torch.equal(m2.cpu(), r2)
    m1 = a1.clone()
    K.moments_update(x, m1, None, L.COLLECT_MEAN, 3.0, 4.0, div_mode="recip")
    torch.cuda.synchronize()
    assert torch.equal(m1, (x + 3 * a1) * (1.0 / 4.0))
    # posterior draws
    eps = torch.randn(n, device=DEV, generator=g)
    q = a1 ** 2 + a2
    out = torch.full_like(x, float("nan"))
    K.posterior_sample(out, a1, q, var_mode=L.VAR_WELFORD, ratio=3.0, noise=eps, div_mode="recip")
    torch.cuda.synchronize()
    assert torch.equal(out, a1 + (q * (1.0 / 3.0)).clamp(min=1e-12).sqrt() * eps)
    K.posterior_sample(out, a1, a2, var_mode=L.VAR_GIVEN, noise=eps)
    torch.cuda.synchronize()
    assert torch.equal(out, a1 + a2.clamp(min=1e-12).sqrt() * eps)
    # Philox noise = the stream bdl_philox_normal produces for the same key
    K.posterior_sample(out, a1, q, var_mode=L.VAR_RAW_MOMENTS, ratio=1.25, seed=3, chain=1,
                       step=9)
    z = K.philox_normal(n, 3, 1, 9, device=DEV)
    torch.cuda.synchronize()
    assert torch.equal(out, a1 + (1.25 * (q - a1 * a1)).clamp(min=1e-12).sqrt() * z)
    K.posterior_sample(out, a1, None, var_mode=L.VAR_WELFORD, seed=3, chain=1, step=9)
    torch.cuda.synchronize()
    assert torch.equal(out, a1 + torch.full_like(a1, 1e-12).sqrt() * z)


def test_moment_pair_changes_nothing_but_the_addresses(monkeypatch):
    """flat.moment_pair (the cSGHMC Runner's per-cycle Welford buffers, two
    halves of one allocation at ViT sizes): the fused Welford collect steps and
    the posterior draws from them equal those into two separate allocations
    bit for bit."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.flat import MOMENT_PAIR_MIN_ELEMS, FlatState, moment_pair
    segs = [("l0.weight", (MOMENT_PAIR_MIN_ELEMS + 5,)), ("fc.weight", (1027,))]
    res = []
    for paired in (True, False):
        st = FlatState.from_segments(segs, "fc", device=DEV)
        if paired:
            m1, m2 = moment_pair(st.n, st.device)
            assert m1.untyped_storage().data_ptr() == m2.untyped_storage().data_ptr()
        else:
            m1, m2 = (torch.empty(st.n, device=st.device) for _ in range(2))
        g = torch.Generator(device=DEV).manual_seed(0)
        st.theta.normal_(0, 0.02, generator=g)
        st.grad.normal_(0, 1e-3, generator=g)
        for k, (collect, cnt) in enumerate(((L.COLLECT_WELFORD_INIT, 1.0), (L.COLLECT_WELFORD, 3.0),
                                            (L.COLLECT_WELFORD, 5.0))):
            K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-3, 1e-2), noise_scale=(1e-3, 1e-3),
                          noise_mode=L.NOISE_PHILOX, one_minus_alpha=0.9, prior_sig=1.0,
                          collect=collect, mom1=m1, mom2=m2, collect_a=cnt, seed=5, step=k)
        out = torch.empty(st.n, dtype=torch.float32, device=DEV)
        K.posterior_sample(out, m1, m2, var_mode=L.VAR_WELFORD, ratio=2.0, seed=7, chain=1, step=3)
        torch.cuda.synchronize()
        res.append([t.clone() for t in (st.theta, st.mom, m1, m2, out)])
        del st, m1, m2, out
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_posterior_draw_geometry_changes_nothing_and_is_tuned_once():
    """bdl_sample_args.blocks_per_cu / unroll (ABI v7): every geometry draws
    the same bits; kernels.posterior_sample tunes it once per device and size
    for vectors of >= SAMPLE_TUNE_MIN elements and reuses the choice."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    n = K.SAMPLE_TUNE_MIN + 4093
    g = torch.Generator(device=DEV).manual_seed(2)
    m1 = torch.randn(n, device=DEV, generator=g) * 0.02
    m2 = torch.rand(n, device=DEV, generator=g) * 1e-4
    outs = []
    for geo in ((1, 4), (2, 4), (3, 4), (4, 1), (8, 1), (0, 0)):
        out = torch.empty(n, device=DEV)
        K.posterior_sample(out, m1, m2, var_mode=L.VAR_WELFORD, ratio=3.0, seed=5, chain=2,
                           step=7, geometry=geo)
        outs.append(out)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    K._SAMPLE_GEOM.pop((torch.device(DEV).index or 0, n), None)
    out = torch.empty(n, device=DEV)
    K.posterior_sample(out, m1, m2, var_mode=L.VAR_WELFORD, ratio=3.0, seed=5, chain=2, step=7)
    torch.cuda.synchronize()
    assert K.sample_geometry(n, out.device) in K.SAMPLE_GEOMETRIES
    assert torch.equal(out, outs[0])
    with pytest.raises(RuntimeError, match="blocks_per_cu"):
        K.posterior_sample(out, m1, m2, var_mode=L.VAR_WELFORD, ratio=3.0, geometry=(9, 4))
    with pytest.raises(RuntimeError, match="unroll"):
        K.posterior_sample(out, m1, m2, var_mode=L.VAR_WELFORD, ratio=3.0, geometry=(2, 2))


@pytest.mark.parametrize("nr,nw", [(2, 1), (3, 2), (4, 2), (3, 4), (5, 4), (7, 5)])
def test_stream_mix_writes_the_first_read_stream(nr, nw):
    """bdl_stream_mix_schedule (the bench's access-mix ceiling): in every issue
    schedule, every written vector receives reads[0] (+ 0 x the others), at a
    ragged size and three geometries (the pipelined schedule's iteration
    counts differ per block); unsupported mixes and schedules are refused."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    n = 3 * (1 << 18) + 5
    g = torch.Generator(device=DEV).manual_seed(nr * 10 + nw)
    reads = [torch.randn(n, device=DEV, generator=g) for _ in range(nr)]
    for sched in (L.MIX_BARE, L.MIX_PIPELINED, L.MIX_PACED):
        for bpc, u in ((1, 4), (2, 2), (3, 1)):
            writes = [torch.full((n,), 7.0, device=DEV) for _ in range(nw)]
            K.stream_mix(reads, writes, bpc, u, schedule=sched)
            torch.cuda.synchronize()
            for w in writes:
                assert torch.equal(w, reads[0]), (sched, bpc, u)
    with pytest.raises(RuntimeError, match="supported"):
        K.stream_mix(reads[:1] * 6, [reads[0]], 1, 4)
    with pytest.raises(RuntimeError, match="schedule"):
        K.stream_mix(reads, [torch.empty_like(reads[0])] * nw, 1, 4, schedule=3)


@pytest.mark.parametrize("unroll", [1, 2, 4])
def test_bare_step_keeps_values_and_copies_the_init_moments(unroll):
    """bdl_sgmcmc_step_bare (the bench's step-shaped ceiling): the cSGHMC
    sweep of every collect kind with its arithmetic removed writes theta, mom
    and the steady-state moments back unchanged and the init moments as the
    step does (Welford m1 = theta, m2 = 0; running mean m1 = theta, m2 =
    theta^2), over a ragged many-run state at each unroll depth (fast,
    multi-run and guarded iterations); other methods are refused."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    segs = [(f"layer{i}.weight", (3 + 5 * i, 7 + i)) for i in range(37)] + [("fc.weight", (10, 33)),
                                                                        ("fc.bias", (10,))]
    st = _state(segs, "fc", need_noise=True)
    K.set_launch_config(2, unroll, 1)
    try:
        th0, v0 = st.theta.clone(), st.mom.clone()
        kw = dict(lrs=(1e-3, 1e-2), noise_scale=(0.0, 0.0), noise_mode=L.NOISE_NONE,
                  one_minus_alpha=0.9, prior_sig=1.0)
        K.sgmcmc_step_bare(st, **kw)
        m1 = torch.randn_like(st.theta)
        m2 = torch.rand_like(st.theta)
        a1, a2 = m1.clone(), m2.clone()
        for collect in (L.COLLECT_WELFORD, L.COLLECT_MEAN):
            K.sgmcmc_step_bare(st, collect=collect, mom1=m1, mom2=m2, collect_a=3.0,
                               collect_b=4.0, **kw)
        torch.cuda.synchronize()
        assert torch.equal(st.theta, th0) and torch.equal(st.mom, v0)
        assert torch.equal(m1, a1) and torch.equal(m2, a2)
        K.sgmcmc_step_bare(st, collect=L.COLLECT_WELFORD_INIT, mom1=m1, mom2=m2, **kw)
        torch.cuda.synchronize()
        assert torch.equal(m1, th0) and torch.equal(m2, torch.zeros_like(m2))
        K.sgmcmc_step_bare(st, collect=L.COLLECT_MEAN_INIT, mom1=m1, mom2=m2, **kw)
        torch.cuda.synchronize()
        assert torch.equal(m1, th0) and torch.equal(m2, th0 * th0)
        assert torch.equal(st.theta, th0) and torch.equal(st.mom, v0)
    finally:
        K.set_launch_config(0, 0, 0)
    st2 = _state(segs, "fc", need_prior=True)
    a = K._step_args(st2, L.SGLD, lrs=(1e-3, 1e-2), noise_scale=(0.0, 0.0),
                     noise_mode=L.NOISE_NONE)
    with pytest.raises(RuntimeError, match="cSGHMC only"):
        L.check(L.lib().bdl_sgmcmc_step_bare(a, None), "bdl_sgmcmc_step_bare")
