"""Launch geometry changes speed only: every candidate geometry (workgroups
per CU, float4 groups in flight, contiguous spans or grid-stride) gives the
same bits for the production kernels; and a state's tuned geometry is
re-installed when another state's is active (kernels._use_geometry)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

GEOMETRIES = [(1, 1, 0), (1, 2, 1), (1, 4, 1), (2, 1, 1), (2, 4, 0), (3, 2, 1), (4, 4, 1)]


def _state(n, seed, need_noise=False):
    from bayesdll_amd import _lib as L
    from bayesdll_amd.flat import FlatState
    segs = [("body.weight", (n - 37,)), ("body.bias", (30,)), ("head.weight", (7,))]
    st = FlatState.from_segments(segs, "head", device="cuda", need_mom=True, need_prior=True,
                                 need_noise=need_noise)
    g = torch.Generator(device="cuda").manual_seed(seed)
    for v in (st.theta, st.grad, st.mom, st.prior) + ((st.noise,) if need_noise else ()):
        v.copy_(torch.randn(st.n, device="cuda", generator=g))
    return st, L


# sghmc / *_buffer: the instances that run on the re-read argument view at
# depth 2 and 4 (bdl_kernels.hpp fresh_step_args) against their depth-1 form
@pytest.mark.parametrize("method", ["csghmc", "sgld", "adam", "sghmc", "sgld_buffer",
                                    "sghmc_buffer"])
def test_results_do_not_depend_on_launch_geometry(method):
    from bayesdll_amd import kernels as K
    n = 3 * (1 << 20) + 13  # ragged: partial float4 group and partial block iterations
    outs = []
    try:
        for geo in GEOMETRIES:
            st, L = _state(n, 1, need_noise=method.endswith("_buffer"))
            nmode = L.NOISE_BUFFER if method.endswith("_buffer") else L.NOISE_PHILOX
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
                elif method == "adam":  # the software-pipelined Adam-SGHMC + SGD sweep
                    if t == 0:
                        am, av, ab = (torch.zeros(n, device="cuda") for _ in range(3))
                    K.adam_step(st, L.ADAM_SGHMC, adam_m=am, adam_v=av, sgd_buf=ab, beta1=0.9,
                                beta2=0.999, eps=1e-8, t=t + 1, momentum_decay=0.1, nd=1.0,
                                lrs=(1e-3, 2e-3), noise_mode=L.NOISE_PHILOX, sigma2=1.0,
                                n_data=100.0, mu=0.5, first_step=t == 0, momentum=True,
                                collect=L.COLLECT_MEAN if t else L.COLLECT_NONE, mom1=m1,
                                mom2=m2, collect_a=float(t), collect_b=float(t + 1), seed=3,
                                chain=1, step=t)
                elif method.startswith("sghmc"):  # SGHMC + SGD(0) + running moments
                    K.sgmcmc_step(st, L.SGHMC, lrs=(1e-3, 2e-3), noise_scale=(1e-2, 2e-2),
                                  noise_mode=nmode, one_minus_alpha=0.9, sigma2=1.0,
                                  n_data=100.0, collect=L.COLLECT_MEAN_INIT if t == 0 else
                                  L.COLLECT_MEAN, mom1=m1, mom2=m2, collect_a=float(t + 1),
                                  collect_b=float(t + 2), seed=3, chain=1, step=t)
                else:
                    K.sgmcmc_step(st, L.SGLD, lrs=(1e-3, 2e-3), noise_scale=(1e-2, 2e-2),
                                  noise_mode=nmode, prior_sig=1.0, sigma2=1.0,
                                  n_data=100.0, mu=0.5, first_step=t == 0, momentum=True,
                                  collect=L.COLLECT_MEAN, mom1=m1, mom2=m2,
                                  collect_a=float(t + 1), collect_b=float(t + 2), seed=3,
                                  chain=1, step=t)
            torch.cuda.synchronize()
            extra = [am, av, ab] if method == "adam" else []
            outs.append(torch.cat([st.theta, st.mom, m1, m2] + extra).clone())
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


@pytest.mark.parametrize("method", ["csghmc", "sgld"])
def test_tuning_on_the_state_leaves_the_chain_unchanged(method):
    """kernels.request_state_tuning (the Runners' and bench.py's geometry
    tuning): the first launch of each kind times every candidate on the
    state's own vectors with that launch's arguments and restores what they
    wrote, so the chain equals one run at a fixed geometry bit for bit; the
    tuned geometries are installed per kind."""
    from bayesdll_amd import kernels as K
    n = (1 << 20) + 13
    outs = []
    try:
        for tune in (False, True):
            st, L = _state(n, 9)
            m1 = torch.zeros(n, device="cuda")
            m2 = torch.zeros(n, device="cuda")
            K.set_launch_config(2, 1, 1)
            if tune:
                K.request_state_tuning(st, method)
            for t in range(3):
                collect = L.COLLECT_WELFORD if method == "csghmc" else L.COLLECT_MEAN
                ck = dict(collect=collect, mom1=m1, mom2=m2, collect_a=float(t + 1),
                          collect_b=float(t + 2)) if t == 2 else {}
                if method == "csghmc":
                    K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-3, 2e-3), noise_scale=(1e-2, 2e-2),
                                  noise_mode=L.NOISE_PHILOX, one_minus_alpha=0.9, prior_sig=1.0,
                                  seed=3, chain=1, step=t, **ck)
                else:
                    K.sgmcmc_step(st, L.SGLD, lrs=(1e-3, 2e-3), noise_scale=(1e-2, 2e-2),
                                  noise_mode=L.NOISE_PHILOX, prior_sig=1.0, sigma2=1.0,
                                  n_data=100.0, mu=0.5, first_step=t == 0, momentum=True,
                                  seed=3, chain=1, step=t, **ck)
                    if tune and t == 0:
                        # a first step (SGD buffer written only) is not tuned on
                        assert "step" in st._tune_pending and "step" not in st.tuned
            torch.cuda.synchronize()
            outs.append(torch.cat([st.theta, st.mom, m1, m2]).clone())
            if tune:
                # the cycle-init kind was never launched: still pending
                assert set(st.tuned) == {"step", "collect"} and st._tune_pending == {"init"}
                assert st.launch_cfg in K.AUTOTUNE_BY_METHOD[method]
                assert st.collect_cfg is not None
                assert int(st.nonfinite.item()) == 0
    finally:
        K.set_launch_config(0, 0, 0)
    assert torch.equal(outs[0], outs[1])
