"""INTEGRATION.md's reference-side binding (examples/reference_binding.py, the
ctypes stub a maintainer adds to methods/csghmc.py:747-778) on the GPU: the
same cSGHMC steps through it and through the product's own binding
(bayesdll_amd.kernels) land bit for bit on the same theta and v."""
import importlib.util
import os

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _binding():
    path = os.path.join(ROOT, "examples", "reference_binding.py")
    spec = importlib.util.spec_from_file_location("reference_binding", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_reference_binding_matches_product_binding():
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.flat import FlatState
    rb = _binding()
    lib = rb.load(L.LIB_PATH)
    segs = [("enc.weight", (1000, 785)), ("enc.bias", (1000,)), ("head.weight", (10, 1000)),
            ("head.bias", (10,))]
    runs, nr = rb.run_table(lib, [(nm, int(np.prod(s))) for nm, s in segs], "head")
    runs_dev = torch.tensor([[runs[i].end, runs[i].attr] for i in range(nr)], dtype=torch.int64,
                            device="cuda")
    st = FlatState.from_segments(segs, "head", device="cuda")
    g = torch.Generator(device="cuda").manual_seed(3)
    st.theta.normal_(0, 0.05, generator=g)
    st.grad.normal_(0, 1e-2, generator=g)
    theta, grad, mom = st.theta.clone(), st.grad.clone(), torch.zeros_like(st.theta)
    lrs, alpha, sig, N, nd = (1e-3, 1e-2), 0.18, 1.0, 1840.0, 0.01
    for k in range(6):
        sample = k % 3 == 2
        rb.csghmc_step(lib, theta, grad, mom, runs_dev, nr, lrs, alpha, sig, N, nd, sample,
                       seed=42, chain=1, step=k)
        K.sgmcmc_step(st, L.CSGHMC, lrs=lrs,
                      noise_scale=[nd * np.sqrt(2 * alpha * x) / N for x in lrs],
                      noise_mode=L.NOISE_PHILOX if sample else L.NOISE_NONE,
                      one_minus_alpha=1 - alpha, prior_sig=sig, seed=42, chain=1, step=k)
    torch.cuda.synchronize()
    assert torch.equal(theta, st.theta) and torch.equal(mom, st.mom)
    assert not torch.equal(mom, torch.zeros_like(mom))
