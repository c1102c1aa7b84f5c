"""Diagnose bitwise differences between the fused Adam-SGHMC kernel and the
reference's torch op sequence on the same GPU (counts of mismatching v_mom
elements under variants that isolate the noise and preconditioner terms)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import FlatState  # noqa: E402

DEV = "cuda"


def run(nd, zero_noise=False, t=1):
    segs = [("l0.weight", (1000, 1000)), ("fc.weight", (10, 1000))]
    st = FlatState.from_segments(segs, "fc", device=DEV, need_prior=True, need_noise=True)
    g = torch.Generator(device=DEV).manual_seed(1)
    st.theta.normal_(0, 0.02, generator=g)
    st.grad.normal_(0, 1e-3, generator=g)
    st.mom.normal_(0, 1e-4, generator=g)
    st.prior.normal_(0, 0.02, generator=g)
    st.noise.normal_(generator=g)
    if zero_noise:
        st.noise.zero_()
    m = torch.randn(st.n, device=DEV, generator=g) * 1e-3
    v = torch.rand(st.n, device=DEV, generator=g) * 1e-6
    b1, b2, ae, a, N, sig, lr = 0.9, 0.99, 1e-8, 0.18, 500.0, 0.8, 1e-3
    # torch reference (single tensor; all elements body lr)
    p, p0, gg = st.theta, st.prior, st.grad
    gU = gg / 1.0 + (p - p0) / (sig ** 2) / N
    mm = b1 * m + (1 - b1) * gU
    vv = b2 * v + (1 - b2) * (gU * gU)
    mh = mm / (1 - b1 ** t)
    vh = vv / (1 - b2 ** t)
    den = torch.sqrt(vh) + ae
    pg = mh / den
    pt = 1.0 / den
    ns = nd * torch.sqrt(2 * a * pt / N)
    nz = ns * st.noise
    vm_ref = st.mom * (1 - a) + lr * pg + nz
    K.adam_step(st, L.ADAM_SGHMC_GRAD, adam_m=m, adam_v=v, beta1=b1, beta2=b2, eps=ae, t=t,
                momentum_decay=a, nd=nd, lrs=(lr, lr), noise_mode=L.NOISE_BUFFER,
                sigma2=sig ** 2, n_data=N, div_mode="recip")
    torch.cuda.synchronize()
    bad = (st.mom != vm_ref)
    idx = torch.nonzero(bad).flatten()[:3]
    print(f"nd={nd} zero_noise={zero_noise} t={t}: m {(m != mm).sum().item()} v "
          f"{(v != vv).sum().item()} vm {bad.sum().item()} / {st.n}")
    for i in idx.tolist():
        print(f"   i={i} kern={st.mom[i].item():.9e} ref={vm_ref[i].item():.9e} "
              f"pg={pg[i].item():.9e} nz={nz[i].item():.9e} a={(st.mom[i]).item()}")


for nd, zn, t in [(0.0, False, 1), (0.05, True, 1), (0.05, False, 1), (0.05, False, 5)]:
    run(nd, zn, t)
