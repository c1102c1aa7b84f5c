"""Launch geometry changes speed only: every candidate geometry (workgroups
per CU, float4 groups in flight, contiguous spans or grid-stride) gives the
same bits for the production kernels; and a state's tuned geometry is
re-installed when another state's is active (kernels._use_geometry)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

GEOMETRIES = [(1, 1, 0), (1, 2, 1), (1, 4, 1), (2, 1, 1), (2, 4, 0), (3, 2, 1), (4, 4, 1)]


def _state(n, seed):
    from bayesdll_amd import _lib as L
    from bayesdll_amd.flat import FlatState
    segs = [("body.weight", (n - 37,)), ("body.bias", (30,)), ("head.weight", (7,))]
    st = FlatState.from_segments(segs, "head", device="cuda", need_mom=True, need_prior=True)
    g = torch.Generator(device="cuda").manual_seed(seed)
    for v in (st.theta, st.grad, st.mom, st.prior):
        v.copy_(torch.randn(st.n, device="cuda", generator=g))
    return st, L


@pytest.mark.parametrize("method", ["csghmc", "sgld"])
def test_results_do_not_depend_on_launch_geometry(method):
    from bayesdll_amd import kernels as K
    n = 3 * (1 << 20) + 13  # ragged: partial float4 group and partial block iterations
    outs = []
    try:
        for geo in GEOMETRIES:
            st, L = _state(n, 1)
            m1 = torch.zeros(n, device="cuda")
            m2 = torch.zeros(n, device="cuda")
            K.set_launch_config(*geo)
            for t in range(3):
                if method == "csghmc":
                    K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-3, 2e-3), noise_scale=(1e-2, 2e-2),
                                  noise_mode=L.NOISE_PHILOX, one_minus_alpha=0.9, prior_sig=1.0,
                                  collect=L.COLLECT_WELFORD_INIT if t == 0 else L.COLLECT_WELFORD,
                                  mom1=m1, mom2=m2, collect_a=float(t + 1), seed=3, chain=1,
                                  step=t)
                else:
                    K.sgmcmc_step(st, L.SGLD, lrs=(1e-3, 2e-3), noise_scale=(1e-2, 2e-2),
                                  noise_mode=L.NOISE_PHILOX, prior_sig=1.0, sigma2=1.0,
                                  n_data=100.0, mu=0.5, first_step=t == 0, momentum=True,
                                  collect=L.COLLECT_MEAN, mom1=m1, mom2=m2,
                                  collect_a=float(t + 1), collect_b=float(t + 2), seed=3,
                                  chain=1, step=t)
            torch.cuda.synchronize()
            outs.append(torch.cat([st.theta, st.mom, m1, m2]).clone())
    finally:
        K.set_launch_config(0, 0, 0)
    for geo, o in zip(GEOMETRIES[1:], outs[1:]):
        assert torch.equal(o, outs[0]), geo


def test_state_geometry_is_reinstalled():
    from bayesdll_amd import kernels as K
    st, L = _state(1 << 16, 2)
    try:
        st.launch_cfg = (3, 2, 1)
        K.set_launch_config(1, 1, 0)  # "another state's" geometry
        K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-3, 1e-3), noise_scale=(0.0, 0.0),
                      noise_mode=L.NOISE_NONE, one_minus_alpha=0.9, prior_sig=1.0)
        assert K._ACTIVE[0] == (3, 2, 1)
        prev = K.set_launch_config(0, 0, 0)
        assert prev == (1 << 24) | (3 << 8) | 2  # packed (grid_stride, blocks_per_cu, unroll)
    finally:
        K.set_launch_config(0, 0, 0)
