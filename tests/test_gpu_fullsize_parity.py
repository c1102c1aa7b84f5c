"""Config-size parity against reference-produced data.

tests/golden/gen_golden.py ran the REFERENCE Runners' own step loops
(methods/csghmc.py:246-384 + :747-778 for C2; methods/sgld.py:193-250 +
:469-484 + torch SGD(momentum 0.5) + the running moments :236-246 for C3) on a
FakeNet with the real parameter shapes of the config's backbone — mlp_mnist
(8 tensors, 2,797,010 params), ResNet-101 C=1000 (314 tensors, 44,549,160) and,
for the headline C4, ViT-L/32 C=1000 (296 tensors, 306,535,400: two cycles of
10 steps, Welford init + 2 updates per cycle with the Q2 doubled count, the
cycle-end likelihood draws) — prescribed gradients and a deterministic per-tensor noise stream in place
of torch.randn_like.  The fixtures hold a 4096-element index subsample,
float64 norms and the SHA-256 of the exact fp32 bytes of every final vector.

The product Runners replay the same run on the GPU through the C-ABI:
  * div_mode "true" (torch-CPU's rounding of a scalar division): every final
    vector — theta, momentum / SGD buffer, the posterior moments — is
    BIT-EXACT (SHA-256 of the full vector);
  * div_mode "recip" (production: torch-on-GPU's x * fl(1/s)): within the
    north star's 1e-5 relative on the updated parameter vector.
"""
import hashlib
import logging
import os
import tempfile
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from golden_util import load

pytestmark = pytest.mark.gpu

RTOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    yield
    _STREAMS.clear()  # the cached streams hold tens of GB of HBM
    torch.cuda.empty_cache()


class DetProvider:
    """gen_golden's torch.randn_like replacement, draw by draw (one det_normal
    per parameter tensor, counter over training and posterior draws), served
    from the precomputed device table of full-vector draws."""

    def __init__(self, numels, table):
        self.numels, self.table, self.k = numels, table, 0

    def __call__(self, step, buf):
        buf.copy_(self.table[self.k // len(self.numels)])
        self.k += len(self.numels)


_STREAMS = {}


def streams(name, fx, numels):
    """The fixture's prescribed gradients (fakenet.grads_for_step, one per
    training step) and noise draws (one det_normal per tensor per call, as
    concatenated vectors), generated ONCE per fixture on the host in a thread
    pool — every vector is its own numpy stream, so they are independent —
    and kept on the device for both division modes (ViT-L/32: 42 vectors,
    ~52 GB of HBM)."""
    if name in _STREAMS:
        return _STREAMS[name]
    from concurrent.futures import ThreadPoolExecutor
    from fakenet import det_normal, grads_for_step
    cfg = fx["config"]
    n, T = int(fx["n"]), len(numels)
    steps = cfg["epochs"] * cfg["bpe"]
    calls = int(fx["draws"]) // T

    def grad(t):
        return torch.from_numpy(grads_for_step(cfg["grad_seed"], t, n, cfg["grad_scale"])).cuda()

    def noise(c):
        return torch.from_numpy(np.concatenate(
            [det_normal(cfg["noise_seed"], c * T + i, k) for i, k in enumerate(numels)])).cuda()

    _STREAMS.clear()  # one fixture's streams at a time
    with ThreadPoolExecutor(min(16, os.cpu_count() or 4)) as ex:
        g = list(ex.map(grad, range(steps)))
        z = list(ex.map(noise, range(calls)))
    _STREAMS[name] = (g, z)
    return g, z


def sha(v):
    return hashlib.sha256(np.ascontiguousarray(v, np.float32).tobytes()).hexdigest()


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def replay(name, fx, div_mode):
    import bayesdll_amd.csghmc as csghmc
    import bayesdll_amd.sgld as sgld
    from bayesdll_amd.shapes import segments
    from fakenet import FakeNet, fake_loader, init_vector, numel_of
    cfg = fx["config"]
    segs, readout = segments(cfg["backbone"], cfg["num_classes"])
    n = numel_of(segs)
    assert n == int(fx["n"]) and int(fx["draws"]) % len(segs) == 0
    gtab, ztab = streams(name, fx, [int(np.prod(sh)) for _, sh in segs])
    theta_init = init_vector(cfg["init_seed"], n, cfg["init_scale"])
    net0 = None
    if cfg.get("prior_seed") is not None:
        prior = init_vector(cfg["prior_seed"], n, cfg["prior_scale"])
        theta_init = (prior + theta_init).astype(np.float32)
        net0 = FakeNet(segs, readout, init=prior).cuda()
    net = FakeNet(segs, readout, grad_seed=cfg["grad_seed"], grad_scale=cfg["grad_scale"],
                  init=theta_init, grad_table=gtab).cuda()
    args = SimpleNamespace(device="cuda", ND=cfg["ND"],
                           pretrained=("fake" if net0 is not None else None), lr=cfg["lr"],
                           lr_head=cfg["lr_head"], momentum=cfg.get("momentum", 0.0),
                           epochs=cfg["epochs"], num_cycles=cfg.get("num_cycles", 2),
                           proportion_exploration=cfg.get("beta", 0.5), full_sample=False,
                           test_eval_freq=1, ece_num_bins=15, log_dir=tempfile.mkdtemp(),
                           num_classes=cfg["num_classes"], noise_mode="external",
                           hparams={k: str(v) for k, v in cfg["hparams"].items()})
    mod = {"csghmc": csghmc, "sgld": sgld}[cfg["method"]]
    runner = mod.Runner(net, net0, args, logging.getLogger("fullsize"))
    runner.model.div_mode = div_mode
    prov = DetProvider([p.numel() for p in runner.net.parameters()], ztab)
    runner.model.noise_provider = prov
    loader = fake_loader(cfg["bpe"], device="cuda")
    if cfg["method"] == "csghmc":
        for ep in range(cfg["epochs"]):
            runner.cyclical_scheduler.current_epoch = ep
            runner.train_one_epoch(loader)
    else:
        bi = 0
        for ep in range(cfg["epochs"]):
            if ep == runner.burnin:
                runner.seed_moments()
            _, _, bi = runner.train_one_epoch(loader, collect=(ep >= runner.burnin), bi=bi)
    torch.cuda.synchronize()
    st = runner.model.flat
    vecs = {"theta": st.theta, "mom": st.mom}
    if cfg["method"] == "csghmc":
        for c in sorted(runner.cycle_theta_mom1):
            vecs[f"cycle{c}_mom1"] = runner.cycle_theta_mom1[c]
            vecs[f"cycle{c}_mom2"] = runner.cycle_theta_mom2[c]
    else:
        vecs["post_mom1"] = runner.post_theta_mom1
        vecs["post_mom2"] = runner.post_theta_mom2
    return runner, prov, {k: v.detach().cpu().numpy() for k, v in vecs.items()}


@pytest.mark.parametrize("div_mode", ["true", "recip"])
@pytest.mark.parametrize("name", ["fullsize_c2_csghmc", "fullsize_c3_sgld", "fullsize_c4_csghmc"])
def test_config_size_replay_matches_reference(name, div_mode):
    fx = load(name)
    runner, prov, vecs = replay(name, fx, div_mode)
    cfg = fx["config"]
    assert prov.k == int(fx["draws"])  # same number and order of noise draws
    keys = sorted(k[:-4] for k in fx if k.endswith("_sha"))
    assert sorted(vecs) == keys
    if cfg["method"] == "csghmc":
        np.testing.assert_array_equal(sorted(runner.cycle_theta_mom1), fx["cycles"])
        np.testing.assert_array_equal(
            [runner.samples_per_cycle[c] for c in sorted(runner.cycle_theta_mom1)],
            fx["samples_per_cycle"])  # quirk Q2: the doubled count
        assert runner.samples_collected == int(fx["samples_collected"])
    else:
        assert runner.post_theta_cnt == int(fx["post_cnt"])
    idx = fx["idx"]
    for key in keys:
        v = vecs[key]
        if div_mode == "true":
            assert sha(v) == str(fx[f"{key}_sha"]), key  # bit-exact, whole vector
        assert rel(v[idx], fx[f"{key}_sub"]) <= RTOL, key
        norm = np.linalg.norm(v.astype(np.float64))
        assert abs(norm - float(fx[f"{key}_norm"])) <= RTOL * float(fx[f"{key}_norm"]), key
