"""The multi-run path (bdl_kernels.hpp chunk_multi / adam_multi) and the
per-run loop of the plain cSGHMC sweep (fast_run).

A block iteration that crosses tensor boundaries — all of them on float4
groups, in runs that all allow the fast path — reads each lane's gradient
from its own tensor with 16-B loads and applies that tensor's attributes per
element; the plain cSGHMC sweep walks the full iterations inside one run with
no LDS access between them.  Over a table of 60 tensors (mostly 4-aligned
sizes, so most boundaries take the multi-run path, a few odd sizes that force
the guarded path, a readout head, uninformative biases), the per-tensor
gradient read (separate allocations through the run / base table) must give
bit for bit what the flat gradient vector gives, for every method and step
kind, at launch geometries from one group per lane to four, grid-stride and
contiguous spans (reference: methods/csghmc.py:747-778, methods/sgld.py:469-484,
methods/sghmc.py:482-510, methods/adam_sghmc.py:500-553).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

GEOMETRIES = [(1, 1, 1), (3, 1, 1), (2, 2, 1), (1, 4, 1), (2, 4, 0)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _segments():
    rng = np.random.default_rng(5)
    aligned = [4, 8, 12, 64, 100, 256, 1000, 1024, 3000, 4096, 5000, 20000]
    segs = []
    for i in range(58):
        k = int(rng.choice(aligned))
        if i == 17:  # between these two odd sizes (3 + 5) the offsets are not 4-aligned
            k = 3
        if i == 41:
            k = 5
        nm = f"layer{i // 2}." + ("bias" if i % 2 else "weight")
        segs.append((nm, (k,)))
    segs += [("head.weight", (1000,)), ("head.bias", (10,))]
    return segs


def _pair(seed, bias="informative", need_prior=False, extra=()):
    """(per-tensor-gradient state, flat-gradient state) over identical values."""
    from bayesdll_amd.flat import FlatState
    segs = _segments()
    kw = dict(bias=bias, device=DEV, need_prior=need_prior, extra=extra)
    st_f = FlatState.from_segments(segs, "head", **kw)
    st_t = FlatState.from_segments(segs, "head", **kw)
    g = torch.Generator(device=DEV).manual_seed(seed)
    st_f.theta.normal_(0.0, 0.02, generator=g)
    st_f.grad.normal_(0.0, 1e-2, generator=g)
    st_f.mom.normal_(0.0, 1e-4, generator=g)
    if need_prior:
        st_f.prior.normal_(0.0, 0.02, generator=g)
        st_t.prior.copy_(st_f.prior)
    for nm in extra:
        st_f.extra[nm].uniform_(0.0, 1e-6, generator=g)
        st_t.extra[nm].copy_(st_f.extra[nm])
    st_t.theta.copy_(st_f.theta)
    st_t.mom.copy_(st_f.mom)
    grads = [st_f.grad[o:o + k].clone() for o, k in zip(st_f.offsets, st_f.numels)]
    st_t.use_tensor_grads(grads)
    st_t._keep = grads  # the per-tensor gradients live as long as the state
    assert st_t.nruns == len(grads) and st_t.gbase is not None
    return st_t, st_f


def _run(st, case, m1, m2):
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    lrs, N, nd = (1e-3, 2e-2), 1840.0, 0.01
    for t in range(3):
        kw = dict(seed=11, chain=2, step=t)
        if case.startswith("csghmc"):
            noise = case != "csghmc_explore"
            collect = {"csghmc_collect": (L.COLLECT_WELFORD_INIT if t == 0 else L.COLLECT_WELFORD)
                       }.get(case, L.COLLECT_NONE)
            K.sgmcmc_step(st, L.CSGHMC, lrs=lrs,
                          noise_scale=[nd * np.sqrt(2 * 0.18 * x) / N for x in lrs],
                          noise_mode=L.NOISE_PHILOX if noise else L.NOISE_NONE,
                          one_minus_alpha=0.82, prior_sig=1.0, collect=collect,
                          mom1=m1 if collect else None, mom2=m2 if collect else None,
                          collect_a=float(2 * t + 1), **kw)
        elif case.startswith("sgld"):
            collect = L.COLLECT_MEAN if t == 2 else L.COLLECT_NONE
            K.sgmcmc_step(st, L.SGLD, lrs=lrs,
                          noise_scale=[nd * np.sqrt(2 / (N * x)) for x in lrs],
                          noise_mode=L.NOISE_PHILOX, prior_sig=1.0, sigma2=1.0, n_data=N,
                          mu=0.5, first_step=t == 0, momentum=True, collect=collect,
                          mom1=m1 if collect else None, mom2=m2 if collect else None,
                          collect_a=2.0, collect_b=3.0, **kw)
        elif case == "sghmc":
            K.sgmcmc_step(st, L.SGHMC, lrs=lrs,
                          noise_scale=[nd * np.sqrt(2 * 0.18 / (N * x)) for x in lrs],
                          noise_mode=L.NOISE_PHILOX, one_minus_alpha=0.82, sigma2=1.0,
                          n_data=N, **kw)
        elif case == "adam":
            m, v, buf = (st.extra[k] for k in ("adam_m", "adam_v", "sgd_buf"))
            K.adam_step(st, L.ADAM_SGHMC, adam_m=m, adam_v=v, sgd_buf=buf, beta1=0.9,
                        beta2=0.999, eps=1e-8, t=t + 1, momentum_decay=0.18, nd=nd, lrs=lrs,
                        noise_mode=L.NOISE_PHILOX, sigma2=1.0, n_data=N, mu=0.5,
                        first_step=t == 0, momentum=True, **kw)


@pytest.mark.parametrize("case", ["csghmc_explore", "csghmc_sample", "csghmc_collect",
                                  "sgld", "sgld_uninformative", "sghmc", "adam"])
def test_per_tensor_gradients_equal_flat_gradient_at_every_geometry(case):
    from bayesdll_amd import kernels as K
    need_prior = not case.startswith("csghmc")
    extra = ("adam_m", "adam_v", "sgd_buf") if case == "adam" else ()
    bias = "uninformative" if case == "sgld_uninformative" else "informative"
    try:
        for geo in GEOMETRIES:
            K.set_launch_config(*geo)
            outs = []
            for st in _pair(7, bias=bias, need_prior=need_prior, extra=extra):
                m1 = torch.zeros(st.n, device=DEV)
                m2 = torch.zeros(st.n, device=DEV)
                _run(st, case, m1, m2)
                torch.cuda.synchronize()
                vecs = [st.theta, st.mom, m1, m2] + [st.extra[k] for k in extra]
                outs.append(torch.cat(vecs).clone())
                assert int(st.nonfinite.item()) == 0
            assert torch.equal(outs[0], outs[1]), (case, geo)
    finally:
        K.set_launch_config(0, 0, 0)


def test_segment_table_exercises_the_multi_run_path():
    """The table above has many 4-aligned boundaries inside one block
    iteration at every geometry (the multi-run path's case) and two odd sizes
    (the guarded path's)."""
    segs = _segments()
    sizes = [s[0] for _, s in segs]
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    aligned = sum(1 for o in offs[1:] if o % 4 == 0)
    assert aligned >= 20 and aligned < len(offs) - 1
    # boundaries that fall inside one 1024-element (depth-1) iteration
    crowded = sum(1 for a, b in zip(offs[1:], offs[2:]) if b - a < 1024)
    assert crowded >= 10
