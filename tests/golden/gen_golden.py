"""Generate the golden fixtures from the REFERENCE sampler (container-only tool).

Runs the reference's own Runner/Model code (methods/{csghmc,csgld,sgld,sghmc}.py,
methods/cyclical.py) imported read-only from /root/reference, on a FakeNet whose
backward returns prescribed gradients (tests/fakenet.py), and records:

  * per step: the lrs handed to Model.forward, should_sample (csghmc), and every
    torch.randn_like draw made inside Model.forward (one per tensor per step,
    named_parameters order: methods/csghmc.py:766, methods/sgld.py:478/483,
    methods/sghmc.py:501), captured by wrapping torch.randn_like;
  * theta and the momentum / SGD buffer before every step and after the last;
  * the final posterior moments, counts and per-cycle dictionaries;
  * cyclical schedule tables (methods/cyclical.py:29-74) for several configs,
    including K % M != 0 (quirk Q3).

Usage (in the build container, where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
The outputs are the small .npz files next to this script; the reference
itself never leaves the container.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import sys
import tempfile
import types
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # tests/ for fakenet
from fakenet import (TOY_SEGMENTS, TOY_READOUT, FakeNet, det_normal, fake_loader,  # noqa: E402
                     init_vector, numel_of, synthetic_mnist)

REF = "/root/reference"


def import_reference():
    tv = types.ModuleType("torchvision")
    for sub in ["transforms", "models", "datasets"]:
        m = types.ModuleType("torchvision." + sub)
        setattr(tv, sub, m)
        sys.modules["torchvision." + sub] = m
    sys.modules["torchvision"] = tv
    sys.path[:0] = [REF, os.path.join(REF, "src")]
    import methods.adam_csghmc
    import methods.adam_sghmc
    import methods.csghmc
    import methods.csghmc_fs
    import methods.csgld
    import methods.cyclical
    import methods.sghmc
    import methods.sgld
    return methods


class Capture:
    """Wrap torch.randn_like; record draws made while `active`."""

    def __init__(self):
        self.active = False
        self.draws = []
        self._orig = torch.randn_like

    def __enter__(self):
        orig = self._orig

        def wrapped(t, *a, **k):
            out = orig(t, *a, **k)
            if self.active:
                self.draws.append(out.detach().clone().reshape(-1))
            return out

        torch.randn_like = wrapped
        return self

    def __exit__(self, *exc):
        torch.randn_like = self._orig


def flat(params):
    return torch.nn.utils.parameters_to_vector([p.detach() for p in params]).numpy().copy()


def make_args(tmp, **kw):
    a = dict(device="cpu", ND=50, pretrained=None, lr=0.05, lr_head=0.1, momentum=0.5, epochs=4,
             num_cycles=2, proportion_exploration=0.5, full_sample=False, test_eval_freq=1,
             ece_num_bins=15, log_dir=tmp, num_classes=10)
    a.update(kw)
    return SimpleNamespace(**a)


def run_method(methods, method, cfg):
    """Drive one reference Runner for cfg['epochs'] epochs; return the record."""
    torch.manual_seed(cfg["torch_seed"])
    n = numel_of(TOY_SEGMENTS)
    theta_init = init_vector(cfg["init_seed"], n, cfg["init_scale"])
    net = FakeNet(grad_seed=cfg["grad_seed"], grad_scale=cfg["grad_scale"], init=theta_init)
    net0 = None
    prior = np.zeros(n, np.float32)
    if cfg.get("prior_seed") is not None:
        prior = init_vector(cfg["prior_seed"], n, 0.3)
        net0 = FakeNet(init=prior)
    tmp = tempfile.mkdtemp(prefix="bdl_golden_")
    args = make_args(tmp, pretrained=("fake" if net0 is not None else None), epochs=cfg["epochs"],
                     num_cycles=cfg.get("num_cycles", 2), lr=cfg["lr"], lr_head=cfg["lr_head"],
                     momentum=cfg.get("momentum", 0.0), ND=cfg["ND"],
                     proportion_exploration=cfg.get("beta", 0.5),
                     hparams={k: str(v) for k, v in cfg["hparams"].items()},
                     **({"clip_grad": cfg["clip_grad"]} if "clip_grad" in cfg else {}))
    logger = logging.getLogger("golden")
    mod = getattr(methods, method)
    runner = mod.Runner(net, net0, args, logger)
    model_cls = mod.Model

    adam = method.startswith("adam_")
    rec = dict(lrs=[], should_sample=[], theta=[], mom=[], noise=[], adam_m=[], adam_v=[],
               sgd_buf=[])
    cap = Capture()
    orig_forward = model_cls.forward

    def state_mom():
        if method in ("csghmc", "csghmc_fs", "sghmc", "adam_sghmc", "adam_csghmc"):
            if not hasattr(runner.model, "momentum_buffer"):
                return np.zeros(n, np.float32)
            return torch.cat([runner.model.momentum_buffer[nm].reshape(-1)
                              for nm, _ in runner.net.named_parameters()]).numpy().copy()
        bufs = []
        for p in runner.net.parameters():
            st = runner.optimizer.state.get(p, {})
            b = st.get("momentum_buffer")
            bufs.append(np.zeros(p.numel(), np.float32) if b is None else b.reshape(-1).numpy())
        return np.concatenate(bufs).astype(np.float32)

    def adam_state(attr):
        d = getattr(runner.model, attr, None)
        if not isinstance(d, dict):
            return np.zeros(n, np.float32)
        return torch.cat([d[nm].reshape(-1) for nm, _ in runner.net.named_parameters()]).numpy().copy()

    def sgd_bufs():
        bufs = []
        for p in runner.net.parameters():
            b = runner.optimizer.state.get(p, {}).get("momentum_buffer")
            bufs.append(np.zeros(p.numel(), np.float32) if b is None else b.reshape(-1).numpy())
        return np.concatenate(bufs).astype(np.float32)

    def record_state():
        rec["mom"].append(state_mom())
        if adam:
            rec["adam_m"].append(adam_state("m"))
            rec["adam_v"].append(adam_state("v"))
            rec["sgd_buf"].append(sgd_bufs())

    def fwd(self, x, y, net_, net0_, criterion, lrs, Ninflate=1.0, nd=1.0, **kw):
        rec["lrs"].append([float(v) for v in lrs])
        rec["should_sample"].append(bool(kw.get("should_sample", False)))
        rec["theta"].append(flat(runner.net.parameters()))
        record_state()
        cap.active, cap.draws = True, []
        try:
            return orig_forward(self, x, y, net_, net0_, criterion, lrs, Ninflate, nd, **kw)
        finally:
            cap.active = False
            rec["noise"].append(torch.cat(cap.draws).numpy().copy())

    model_cls.forward = fwd
    try:
        with cap:
            loader = fake_loader(cfg["bpe"])
            if method in ("csghmc", "csghmc_fs", "csgld", "adam_csghmc"):
                for ep in range(cfg["epochs"]):
                    runner.cyclical_scheduler.current_epoch = ep
                    runner.train_one_epoch(loader)
            else:  # sgld / sghmc: Runner.train's epoch loop minus evaluation
                bi = 0
                for ep in range(cfg["epochs"]):
                    if ep == runner.burnin:
                        with torch.no_grad():
                            tv = torch.nn.utils.parameters_to_vector(runner.net.parameters())
                            runner.post_theta_mom1 = tv * 1.0
                            if runner.nst > 0:
                                runner.post_theta_mom2 = tv ** 2
                        runner.post_theta_cnt = 1
                    _, _, bi = runner.train_one_epoch(loader, collect=(ep >= runner.burnin), bi=bi)
    finally:
        model_cls.forward = orig_forward

    out = dict(
        config=json.dumps(dict(cfg, method=method)),
        segments=json.dumps([[nm, list(s)] for nm, s in TOY_SEGMENTS]),
        readout=TOY_READOUT,
        theta_init=theta_init,
        prior_mean=prior,
        lrs=np.array(rec["lrs"], np.float64),
        should_sample=np.array(rec["should_sample"], bool),
        noise=np.stack(rec["noise"]).astype(np.float32),
        theta=np.stack(rec["theta"] + [flat(runner.net.parameters())]).astype(np.float32),
    )
    record_state()
    out["mom"] = np.stack(rec["mom"]).astype(np.float32)
    if adam:
        out["adam_m"] = np.stack(rec["adam_m"]).astype(np.float32)
        out["adam_v"] = np.stack(rec["adam_v"]).astype(np.float32)
        out["sgd_buf"] = np.stack(rec["sgd_buf"]).astype(np.float32)
    if method in ("csghmc", "csghmc_fs", "csgld", "adam_csghmc"):
        cycles = sorted(runner.cycle_theta_mom1.keys())
        out["cycles"] = np.array(cycles, np.int64)
        out["cycle_mom1"] = np.stack([runner.cycle_theta_mom1[c].numpy() for c in cycles]) \
            if cycles else np.zeros((0, n), np.float32)
        out["cycle_mom2"] = np.stack([runner.cycle_theta_mom2[c].numpy() for c in cycles]) \
            if cycles else np.zeros((0, n), np.float32)
        out["samples_per_cycle"] = np.array([runner.samples_per_cycle[c] for c in cycles], np.int64)
        out["samples_collected"] = np.int64(runner.samples_collected)
        out["current_cycle"] = np.int64(runner.current_cycle)
        out["ckpt_files"] = np.array(sorted(os.listdir(tmp)))
    else:
        out["post_mom1"] = runner.post_theta_mom1.numpy()
        out["post_mom2"] = runner.post_theta_mom2.numpy() if runner.nst > 0 else np.zeros(0, np.float32)
        out["post_cnt"] = np.int64(runner.post_theta_cnt)
    return out


CLIP_MAX_NORM = 40.0
ADAM_CLIP_MAX_NORM = 4.4

CONFIGS = {
    # cSGHMC (config 2 hyper-parameters, scaled to make every term visible)
    "csghmc_k20": ("csghmc", dict(epochs=4, bpe=5, num_cycles=2, beta=0.5, lr=0.05, lr_head=0.1,
                                  ND=50, torch_seed=7, init_seed=11, init_scale=0.5, grad_seed=101,
                                  grad_scale=0.5,
                                  hparams=dict(prior_sig=0.7, bias="informative",
                                               momentum_decay=0.18, Ninflate=1.0, nd=1.0,
                                               burnin=0, thin=2, nst=2))),
    # K % M != 0: lr restarts and cycle numbers drift apart, last_in_cycle never fires (Q3)
    "csghmc_k21": ("csghmc", dict(epochs=3, bpe=7, num_cycles=2, beta=0.5, lr=0.05, lr_head=0.2,
                                  ND=40, torch_seed=8, init_seed=12, init_scale=0.5, grad_seed=102,
                                  grad_scale=0.3,
                                  hparams=dict(prior_sig=1.0, bias="uninformative",
                                               momentum_decay=0.3, Ninflate=2.0, nd=0.5,
                                               burnin=0, thin=1, nst=2))),
    # csghmc_fs: csghmc + momentum zeroed after every completed cycle
    "csghmc_fs_k20": ("csghmc_fs", dict(epochs=4, bpe=5, num_cycles=2, beta=0.5, lr=0.05,
                                        lr_head=0.1, ND=50, torch_seed=20, init_seed=23,
                                        init_scale=0.5, grad_seed=113, grad_scale=0.5,
                                        hparams=dict(prior_sig=0.7, bias="informative",
                                                     momentum_decay=0.18, Ninflate=1.0, nd=1.0,
                                                     burnin=0, thin=2, nst=2))),
    "csgld_k20": ("csgld", dict(epochs=4, bpe=5, num_cycles=2, beta=0.5, lr=0.05, lr_head=0.1,
                                momentum=0.5, ND=50, torch_seed=9, init_seed=13, init_scale=0.5,
                                grad_seed=103, grad_scale=0.5,
                                hparams=dict(prior_sig=0.7, bias="informative", Ninflate=1.0,
                                             nd=1.0, nst=2, thin=2))),
    # args.clip_grad: clip_grad_norm_ between Model.forward and optimizer.step
    # (methods/csgld.py:250-251); max_norm chosen so some steps clip and some do not
    "csgld_clip": ("csgld", dict(epochs=4, bpe=5, num_cycles=2, beta=0.5, lr=0.05, lr_head=0.1,
                                 momentum=0.5, ND=50, torch_seed=19, init_seed=18, init_scale=0.5,
                                 grad_seed=108, grad_scale=0.5, clip_grad=CLIP_MAX_NORM,
                                 hparams=dict(prior_sig=0.7, bias="informative", Ninflate=1.0,
                                              nd=1.0, nst=2, thin=2))),
    "sgld_inf": ("sgld", dict(epochs=3, bpe=5, lr=0.05, lr_head=0.1, momentum=0.5, ND=50,
                              torch_seed=10, init_seed=14, init_scale=0.5, grad_seed=104,
                              grad_scale=0.5, prior_seed=21,
                              hparams=dict(prior_sig=0.8, bias="informative", Ninflate=1.0,
                                           nd=1.0, burnin=1, thin=2, nst=2))),
    "sgld_uninf_nomom": ("sgld", dict(epochs=3, bpe=5, lr=0.02, lr_head=0.05, momentum=0.0,
                                      ND=30, torch_seed=11, init_seed=15, init_scale=0.5,
                                      grad_seed=105, grad_scale=0.5, prior_seed=22,
                                      hparams=dict(prior_sig=0.5, bias="uninformative",
                                                   Ninflate=10.0, nd=0.1, burnin=1, thin=3,
                                                   nst=0))),
    # Adam-preconditioned SGHMC (methods/adam_sghmc.py): SGD with args.momentum
    "adam_sghmc_inf": ("adam_sghmc", dict(epochs=3, bpe=5, lr=0.05, lr_head=0.1, momentum=0.5,
                                          ND=50, torch_seed=14, init_seed=19, init_scale=0.5,
                                          grad_seed=109, grad_scale=0.5, prior_seed=25,
                                          hparams=dict(prior_sig=0.8, bias="informative",
                                                       momentum_decay=0.18, Ninflate=1.0,
                                                       nd=1.0, burnin=1, thin=2, nst=2,
                                                       beta1=0.9, beta2=0.99, epsilon=1e-8))),
    "adam_sghmc_uninf_nomom": ("adam_sghmc", dict(epochs=3, bpe=4, lr=0.02, lr_head=0.04,
                                                  momentum=0.0, ND=30, torch_seed=15,
                                                  init_seed=20, init_scale=0.5, grad_seed=110,
                                                  grad_scale=0.5, prior_seed=26,
                                                  hparams=dict(prior_sig=1.5,
                                                               bias="uninformative",
                                                               momentum_decay=0.3, Ninflate=5.0,
                                                               nd=0.2, burnin=1, thin=1, nst=0,
                                                               beta1=0.8, beta2=0.95,
                                                               epsilon=1e-6))),
    # cyclical Adam-SGHMC (methods/adam_csghmc.py): p.grad = v_mom, g / temperature,
    # v_mom / m / v zeroed and t reset at the end of every cycle
    "adam_csghmc_k20": ("adam_csghmc", dict(epochs=4, bpe=5, num_cycles=2, beta=0.5, lr=0.05,
                                            lr_head=0.1, ND=50, torch_seed=16, init_seed=21,
                                            init_scale=0.5, grad_seed=111, grad_scale=0.5,
                                            prior_seed=27,
                                            hparams=dict(prior_sig=0.7, bias="informative",
                                                         momentum_decay=0.18, Ninflate=1.0,
                                                         nd=1.0, nst=2, thin=1, burnin=0,
                                                         beta1=0.9, beta2=0.99, epsilon=1e-8,
                                                         temperature=0.5))),
    "adam_csghmc_clip": ("adam_csghmc", dict(epochs=4, bpe=5, num_cycles=2, beta=0.5, lr=0.05,
                                             lr_head=0.1, ND=50, torch_seed=17, init_seed=22,
                                             init_scale=0.5, grad_seed=112, grad_scale=0.5,
                                             prior_seed=28, clip_grad=ADAM_CLIP_MAX_NORM,
                                             hparams=dict(prior_sig=0.7, bias="uninformative",
                                                          momentum_decay=0.18, Ninflate=2.0,
                                                          nd=0.5, nst=2, thin=1, burnin=0,
                                                          beta1=0.9, beta2=0.999,
                                                          epsilon=1e-8))),
    "sghmc_inf": ("sghmc", dict(epochs=3, bpe=5, lr=0.05, lr_head=0.1, ND=50, torch_seed=12,
                                init_seed=16, init_scale=0.5, grad_seed=106, grad_scale=0.5,
                                prior_seed=23,
                                hparams=dict(prior_sig=0.8, bias="informative",
                                             momentum_decay=0.18, Ninflate=1.0, nd=1.0,
                                             burnin=1, thin=2, nst=2))),
    "sghmc_uninf": ("sghmc", dict(epochs=3, bpe=4, lr=0.02, lr_head=0.04, ND=30, torch_seed=13,
                                  init_seed=17, init_scale=0.5, grad_seed=107, grad_scale=0.5,
                                  prior_seed=24,
                                  hparams=dict(prior_sig=1.5, bias="uninformative",
                                               momentum_decay=0.3, Ninflate=5.0, nd=0.2,
                                               burnin=1, thin=2, nst=2))),
}

SCHEDULES = [(4, 5, 2, 0.5), (3, 7, 2, 0.5), (10, 7, 3, 0.3), (7, 10, 3, 0.5), (5, 3, 4, 0.25),
             (2, 115, 4, 0.5)]


def schedule_tables(methods):
    C = methods.cyclical.CyclicalSGMCMC
    out = {}
    for (E, B, M, beta) in SCHEDULES:
        s = C(base_lr=0.1, nbr_of_cycles=M, epochs=E, proportion_exploration=beta)
        rows = []
        for ep in range(E):
            for b in range(B):
                rows.append((float(s.calculate_lr(ep, b, B)), bool(s.should_sample(ep, b, B)),
                             bool(s.last_in_cycle(ep, b, B)), int(s.get_cycle_number(ep, b, B))))
        key = f"E{E}_B{B}_M{M}_beta{beta}"
        out[key + "_lr"] = np.array([r[0] for r in rows], np.float64)
        out[key + "_sample"] = np.array([r[1] for r in rows], bool)
        out[key + "_last"] = np.array([r[2] for r in rows], bool)
        out[key + "_cycle"] = np.array([r[3] for r in rows], np.int64)
    out["configs"] = json.dumps(SCHEDULES)
    return out


# --------------------------------------------------------------------------
# Runner.train() end to end on the reference's real mlp_mnist backbone
# (networks/small_nets.py), synthetic MNIST-shaped data (config 1 / 2).  The
# torch.randn_like stream is replaced by a deterministic numpy stream
# (fakenet.det_normal, draw counter k) so the product can replay it on the GPU
# without storing 2.8M-element draws; the draw ORDER is pinned by the
# FakeNet fixtures above, which capture torch's own stream.
# --------------------------------------------------------------------------
MLP_CONFIGS = {
    # config 2: mlp_mnist cSGHMC (hparams of pretrain_resnet101.py:127)
    "mlp_csghmc_c2": ("csghmc", dict(epochs=4, ntrain=512, ntest=256, batch=128, num_cycles=2,
                                     beta=0.5, lr=0.02, lr_head=0.02, ND=30000, data_seed=1,
                                     init_seed=2, noise_seed=3,
                                     hparams=dict(prior_sig=1.0, bias="informative",
                                                  momentum_decay=0.18, Ninflate=1.0, nd=0.01,
                                                  burnin=0, thin=1, nst=2))),
    # config 1: mlp_mnist SGLD (README.md:83 hparams; burnin/epochs shortened)
    "mlp_sgld_c1": ("sgld", dict(epochs=3, ntrain=512, ntest=256, batch=128, lr=1e-2,
                                 lr_head=1e-2, momentum=0.5, ND=30000, data_seed=4, init_seed=5,
                                 noise_seed=6,
                                 hparams=dict(prior_sig=1.0, bias="informative", Ninflate=1e3,
                                              nd=1.0, burnin=1, thin=2, nst=2))),
}
SUBSET = 4096


def subset_idx(n, seed=99):
    return np.sort(np.random.default_rng(seed).choice(n, size=SUBSET, replace=False))


def run_mlp(methods, method, cfg):
    from networks import small_nets
    torch.manual_seed(0)
    net = small_nets.MLP(input_dim=784, output_dim=10, width=1000, depth=3)
    net.readout_name = "classifier"
    n = sum(p.numel() for p in net.parameters())
    theta0 = init_vector(cfg["init_seed"], n, 0.03)
    with torch.no_grad():
        torch.nn.utils.vector_to_parameters(torch.tensor(theta0), net.parameters())
    train = synthetic_mnist(cfg["data_seed"], cfg["ntrain"], cfg["batch"])
    test = synthetic_mnist(cfg["data_seed"] + 100, cfg["ntest"], cfg["batch"])
    tmp = tempfile.mkdtemp(prefix="bdl_golden_mlp_")
    args = make_args(tmp, epochs=cfg["epochs"], num_cycles=cfg.get("num_cycles", 2), lr=cfg["lr"],
                     lr_head=cfg["lr_head"], momentum=cfg.get("momentum", 0.0), ND=cfg["ND"],
                     proportion_exploration=cfg.get("beta", 0.5), test_eval_freq=1,
                     hparams={k: str(v) for k, v in cfg["hparams"].items()})
    mod = getattr(methods, method)
    runner = mod.Runner(net, None, args, logging.getLogger("golden"))
    counter = [0]
    orig = torch.randn_like

    def det_randn_like(t, *a, **k):
        out = torch.from_numpy(det_normal(cfg["noise_seed"], counter[0], t.numel())).reshape(t.shape)
        counter[0] += 1
        return out.to(t.dtype)

    evals = []
    orig_eval = mod.Runner.evaluate

    def ev(self, loader):
        r = orig_eval(self, loader)
        evals.append(r)
        return r

    torch.randn_like = det_randn_like
    mod.Runner.evaluate = ev
    try:
        res = runner.train(train, None, test)
    finally:
        torch.randn_like = orig
        mod.Runner.evaluate = orig_eval
    idx = subset_idx(n)
    theta = torch.nn.utils.parameters_to_vector(runner.net.parameters()).detach().numpy()
    out = dict(config=json.dumps(dict(cfg, method=method)), idx=idx, theta_sub=theta[idx],
               theta_norm=np.float64(np.linalg.norm(theta.astype(np.float64))),
               draws=np.int64(counter[0]))
    if res is not None:
        out["losses_train"] = res["losses_train"]
        out["errors_train"] = res["errors_train"]
        out["losses_test"] = res["losses_test"]
        out["errors_test"] = res["errors_test"]
    last = evals[-1]
    out["eval_loss"] = np.float64(last[0])
    out["eval_err"] = np.float64(last[1])
    out["eval_logits"] = last[3].astype(np.float32)
    out["n_evals"] = np.int64(len(evals))
    if method in ("csghmc", "csgld"):
        cyc = sorted(runner.cycle_theta_mom1.keys())
        out["cycles"] = np.array(cyc)
        out["samples_per_cycle"] = np.array([runner.samples_per_cycle[c] for c in cyc])
        out["cycle_mom1_sub"] = np.stack([runner.cycle_theta_mom1[c].numpy()[idx] for c in cyc])
        out["cycle_mom2_sub"] = np.stack([runner.cycle_theta_mom2[c].numpy()[idx] for c in cyc])
        out["cycle_likelihoods"] = np.stack([np.asarray(runner.cycle_likelihoods[c])
                                             for c in sorted(runner.cycle_likelihoods)])
    else:
        out["post_mom1_sub"] = runner.post_theta_mom1.numpy()[idx]
        out["post_mom2_sub"] = runner.post_theta_mom2.numpy()[idx]
        out["post_cnt"] = np.int64(runner.post_theta_cnt)
    return out


# --------------------------------------------------------------------------
# Checkpoint interop: a checkpoint WRITTEN BY THE
# REFERENCE Runner, then loaded into a FRESH reference Runner and evaluated.
# The product must load the same file (weights_only) and predict the same.
# A narrow mlp (width 16) keeps the .pt fixtures small; noise is the
# deterministic det_normal stream (draw counter restarted at 0 for the
# evaluation), which the product replays with its "external" noise source.
# --------------------------------------------------------------------------
CKPT_CONFIGS = {
    "csghmc": dict(epochs=4, ntrain=256, ntest=128, batch=64, num_cycles=2, beta=0.5, lr=0.02,
                   lr_head=0.02, ND=256, data_seed=21, init_seed=22, noise_seed=23,
                   eval_noise_seed=24, width=16, ckpt="2_ckpt.pt",
                   hparams=dict(prior_sig=1.0, bias="informative", momentum_decay=0.18,
                                Ninflate=1.0, nd=0.01, burnin=0, thin=1, nst=2)),
    "sgld": dict(epochs=3, ntrain=256, ntest=128, batch=64, lr=1e-2, lr_head=1e-2, momentum=0.5,
                 ND=256, data_seed=25, init_seed=26, noise_seed=27, eval_noise_seed=28, width=16,
                 ckpt="ckpt.pt",
                 hparams=dict(prior_sig=1.0, bias="informative", Ninflate=1e3, nd=1.0, burnin=1,
                              thin=1, nst=2)),
}


def run_ckpt_interop(methods, method, cfg):
    import shutil
    from networks import small_nets
    mod = getattr(methods, method)
    train = synthetic_mnist(cfg["data_seed"], cfg["ntrain"], cfg["batch"])
    test = synthetic_mnist(cfg["data_seed"] + 100, cfg["ntest"], cfg["batch"])
    counter = [0]
    seed = [cfg["noise_seed"]]
    orig = torch.randn_like

    def det_randn_like(t, *a, **k):
        out = torch.from_numpy(det_normal(seed[0], counter[0], t.numel())).reshape(t.shape)
        counter[0] += 1
        return out.to(t.dtype)

    def make_runner(init_seed):
        torch.manual_seed(0)
        net = small_nets.MLP(input_dim=784, output_dim=10, width=cfg["width"], depth=3)
        net.readout_name = "classifier"
        n = sum(p.numel() for p in net.parameters())
        with torch.no_grad():
            torch.nn.utils.vector_to_parameters(torch.tensor(init_vector(init_seed, n, 0.03)),
                                                net.parameters())
        tmp = tempfile.mkdtemp(prefix="bdl_golden_ckpt_")
        args = make_args(tmp, epochs=cfg["epochs"], num_cycles=cfg.get("num_cycles", 2),
                         lr=cfg["lr"], lr_head=cfg["lr_head"], momentum=cfg.get("momentum", 0.0),
                         ND=cfg["ND"], proportion_exploration=cfg.get("beta", 0.5),
                         test_eval_freq=1,
                         hparams={k: str(v) for k, v in cfg["hparams"].items()})
        return mod.Runner(net, None, args, logging.getLogger("golden")), tmp

    torch.randn_like = det_randn_like
    try:
        runner, tmp = make_runner(cfg["init_seed"])
        runner.train(train, None, test)
        src = os.path.join(tmp, cfg["ckpt"])
        dst = os.path.join(HERE, f"ckpt_ref_{method}.pt")
        shutil.copyfile(src, dst)
        # a fresh Runner (different init) restores the file and evaluates
        fresh, _ = make_runner(cfg["init_seed"] + 1000)
        epoch = fresh.load_ckpt(dst)
        seed[0], counter[0] = cfg["eval_noise_seed"], 0
        loss, err, targets, logits, logits_all = fresh.evaluate(test)
        draws = counter[0]
    finally:
        torch.randn_like = orig
    return dict(config=json.dumps(dict(cfg, method=method)), epoch=np.int64(epoch),
                eval_loss=np.float64(loss), eval_err=np.float64(err), targets=targets,
                logits=logits.astype(np.float32), logits_all=logits_all.astype(np.float32),
                eval_draws=np.int64(draws))


# --------------------------------------------------------------------------
# Config-size pins: the reference Runners' own step
# loop on a FakeNet with the REAL parameter shapes of the config's backbone
# (mlp_mnist: 8 tensors, 2,797,010; ResNet-101 C=1000: 314 tensors,
# 44,549,160 — bayesdll_amd/shapes.py), prescribed gradients
# (fakenet.grads_for_step) and the deterministic det_normal stream in place
# of torch.randn_like (one draw per tensor per step, counter k).  The vectors
# are too large to store: the fixture keeps a 4096-element index subsample,
# float64 norms and a SHA-256 of the exact fp32 bytes of every final vector.
# --------------------------------------------------------------------------
FULLSIZE_CONFIGS = {
    # config 2: mlp_mnist cSGHMC (pretrain_resnet101.py:127 hparams; ND = MNIST 60k x 0.5)
    "fullsize_c2_csghmc": ("csghmc", "mlp_mnist", 10, dict(
        epochs=4, bpe=5, num_cycles=2, beta=0.5, lr=1e-2, lr_head=1e-2, ND=30000, init_seed=41,
        init_scale=0.03, grad_seed=42, grad_scale=1e-2, noise_seed=43,
        hparams=dict(prior_sig=1.0, bias="informative", momentum_decay=0.18, Ninflate=1.0,
                     nd=0.01, burnin=0, thin=2, nst=5))),
    # config 3: ResNet-101 (C=1000) SGLD + SGD(momentum 0.5), informative prior
    # theta0 ~ N(0, 0.02^2) (the IMAGENET1K_V1 stand-in), theta = theta0 +
    # N(0, 1e-3^2), g ~ N(0, 1e-3^2), ND = Pets trainval x 0.5 (README.md:111)
    "fullsize_c3_sgld": ("sgld", "resnet101", 1000, dict(
        epochs=3, bpe=4, lr=1e-4, lr_head=1e-2, momentum=0.5, ND=1840, init_seed=44,
        init_scale=1e-3, prior_seed=45, prior_scale=0.02, grad_seed=46, grad_scale=1e-3,
        noise_seed=47,
        hparams=dict(prior_sig=1.0, bias="informative", Ninflate=1e3, nd=0.01, burnin=1,
                     thin=2, nst=2))),
    # config 4 (the headline): ViT-L/32 (C=1000, 296 tensors, 306,535,400) cSGHMC
    # with the csghmc hparams of pretrain_resnet101.py:127 (alpha_m 0.18,
    # nd 0.01, Ninflate 1) and the vision demos' lr 1e-4 / lr_head 1e-2, ND =
    # Pets trainval x 0.5 (README.md:139).  Two cycles of 10 steps: the
    # sampling half is one epoch of 5 batches, thin 2 on the batch index
    # (quirk Q4) -> batches 0, 2, 4 -> Welford init + 2 updates per cycle, the
    # Q2 doubled count, and each cycle's end (likelihoods + checkpoint).
    "fullsize_c4_csghmc": ("csghmc", "vit_l_32", 1000, dict(
        epochs=4, bpe=5, num_cycles=2, beta=0.5, lr=1e-4, lr_head=1e-2, ND=1840, init_seed=48,
        init_scale=0.02, grad_seed=49, grad_scale=1e-3, noise_seed=50,
        hparams=dict(prior_sig=1.0, bias="informative", momentum_decay=0.18, Ninflate=1.0,
                     nd=0.01, burnin=0, thin=2, nst=1))),
}


def vec_digest(v):
    import hashlib
    v = np.ascontiguousarray(np.asarray(v, np.float32))
    return dict(sha=hashlib.sha256(v.tobytes()).hexdigest(),
                norm=np.float64(np.linalg.norm(v.astype(np.float64))))


def run_fullsize(methods, method, backbone, num_classes, cfg):
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from bayesdll_amd.shapes import segments
    segs, readout = segments(backbone, num_classes)
    n = numel_of(segs)
    theta_init = init_vector(cfg["init_seed"], n, cfg["init_scale"])
    net0, prior = None, None
    if cfg.get("prior_seed") is not None:
        prior = init_vector(cfg["prior_seed"], n, cfg["prior_scale"])
        theta_init = (prior + theta_init).astype(np.float32)  # theta = theta0 + N(0, s^2)
        net0 = FakeNet(segs, readout, init=prior)
    net = FakeNet(segs, readout, grad_seed=cfg["grad_seed"], grad_scale=cfg["grad_scale"],
                  init=theta_init)
    tmp = tempfile.mkdtemp(prefix="bdl_golden_full_")
    args = make_args(tmp, pretrained=("fake" if net0 is not None else None), epochs=cfg["epochs"],
                     num_cycles=cfg.get("num_cycles", 2), lr=cfg["lr"], lr_head=cfg["lr_head"],
                     momentum=cfg.get("momentum", 0.0), ND=cfg["ND"],
                     proportion_exploration=cfg.get("beta", 0.5), num_classes=num_classes,
                     hparams={k: str(v) for k, v in cfg["hparams"].items()})
    mod = getattr(methods, method)
    runner = mod.Runner(net, net0, args, logging.getLogger("golden"))
    counter = [0]
    orig = torch.randn_like

    def det_randn_like(t, *a, **k):
        out = torch.from_numpy(det_normal(cfg["noise_seed"], counter[0], t.numel())).reshape(t.shape)
        counter[0] += 1
        return out.to(t.dtype)

    torch.randn_like = det_randn_like
    try:
        loader = fake_loader(cfg["bpe"])
        if method == "csghmc":
            for ep in range(cfg["epochs"]):
                runner.cyclical_scheduler.current_epoch = ep
                runner.train_one_epoch(loader)
        else:  # sgld: Runner.train's epoch loop minus evaluation (methods/sgld.py:193-250)
            bi = 0
            for ep in range(cfg["epochs"]):
                if ep == runner.burnin:
                    with torch.no_grad():
                        tv = torch.nn.utils.parameters_to_vector(runner.net.parameters())
                        runner.post_theta_mom1 = tv * 1.0
                        if runner.nst > 0:
                            runner.post_theta_mom2 = tv ** 2
                    runner.post_theta_cnt = 1
                _, _, bi = runner.train_one_epoch(loader, collect=(ep >= runner.burnin), bi=bi)
    finally:
        torch.randn_like = orig
    idx = subset_idx(n)
    names = [nm for nm, _ in runner.net.named_parameters()]
    vecs = {"theta": flat(runner.net.parameters())}
    if method == "csghmc":
        vecs["mom"] = torch.cat([runner.model.momentum_buffer[nm].reshape(-1)
                                 for nm in names]).numpy()
        cyc = sorted(runner.cycle_theta_mom1.keys())
        for c in cyc:
            vecs[f"cycle{c}_mom1"] = runner.cycle_theta_mom1[c].numpy()
            vecs[f"cycle{c}_mom2"] = runner.cycle_theta_mom2[c].numpy()
        extra = dict(cycles=np.array(cyc, np.int64),
                     samples_per_cycle=np.array([runner.samples_per_cycle[c] for c in cyc]),
                     samples_collected=np.int64(runner.samples_collected),
                     current_cycle=np.int64(runner.current_cycle))
    else:
        vecs["mom"] = np.concatenate([runner.optimizer.state[p]["momentum_buffer"].reshape(-1).numpy()
                                      for p in runner.net.parameters()])
        vecs["post_mom1"] = runner.post_theta_mom1.numpy()
        vecs["post_mom2"] = runner.post_theta_mom2.numpy()
        extra = dict(post_cnt=np.int64(runner.post_theta_cnt))
    out = dict(config=json.dumps(dict(cfg, method=method, backbone=backbone,
                                      num_classes=num_classes)),
               n=np.int64(n), idx=idx, draws=np.int64(counter[0]), **extra)
    for key, v in vecs.items():
        d = vec_digest(v)
        out[f"{key}_sub"] = np.asarray(v, np.float32)[idx]
        out[f"{key}_sha"] = d["sha"]
        out[f"{key}_norm"] = d["norm"]
    return out


def calibration_fixture():
    """Reference calibration.analyze / find_optimal_temperature on seeded
    logits (the metrics the Runners log after a new best evaluation)."""
    import matplotlib
    matplotlib.use("Agg")
    import calibration
    rng = np.random.default_rng(2024)
    out = {}
    tmp = tempfile.mkdtemp(prefix="bdl_golden_calib_")
    for name, (n, k, scale) in {"c10": (200, 10, 3.0), "c37": (64, 37, 1.5)}.items():
        logits = (rng.standard_normal((n, k)) * scale).astype(np.float32)
        labels = rng.integers(0, k, size=n)
        labels[: n // 2] = logits[: n // 2].argmax(1)        # half of them confidently right
        vlogits = (rng.standard_normal((n, k)) * scale).astype(np.float32)
        vlabels = rng.integers(0, k, size=n)
        vlabels[: n // 2] = vlogits[: n // 2].argmax(1)
        out[f"{name}_logits"], out[f"{name}_labels"] = logits, labels
        out[f"{name}_vlogits"], out[f"{name}_vlabels"] = vlogits, vlabels
        for t in (1.0, 1.7):
            out[f"{name}_analyze_T{t}"] = np.array(calibration.analyze(
                labels, logits, num_bins=15, plot_save_path=os.path.join(tmp, "r.png"),
                temperature=t), dtype=np.float64)
        topt, ok = calibration.find_optimal_temperature(vlabels, vlogits,
                                                        os.path.join(tmp, "t.png"))
        out[f"{name}_topt"] = np.asarray(topt, dtype=np.float64)
        out[f"{name}_topt_ok"] = np.bool_(ok)
    return out


def main():
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    logging.basicConfig(level=logging.WARNING)
    methods = import_reference()
    torch.set_num_threads(1)
    only = os.environ.get("GOLDEN_ONLY")
    if only == "calib":
        np.savez_compressed(os.path.join(HERE, "calibration.npz"), **calibration_fixture())
        print("wrote calibration.npz")
        return
    if only == "ckpt":
        torch.set_num_threads(8)
        recs = {}
        for method, cfg in CKPT_CONFIGS.items():
            rec = run_ckpt_interop(methods, method, copy.deepcopy(cfg))
            recs.update({f"{method}_{k}": v for k, v in rec.items()})
            print(f"wrote ckpt_ref_{method}.pt epoch={int(rec['epoch'])} "
                  f"eval_draws={int(rec['eval_draws'])} loss={float(rec['eval_loss']):.6f}")
        np.savez_compressed(os.path.join(HERE, "ckpt_ref.npz"), **recs)
        return
    if only == "fullsize":
        torch.set_num_threads(8)
        pick = os.environ.get("GOLDEN_FULLSIZE")  # comma list; default: every config
        for name, (method, backbone, classes, cfg) in FULLSIZE_CONFIGS.items():
            if pick and name not in pick.split(","):
                continue
            rec = run_fullsize(methods, method, backbone, classes, copy.deepcopy(cfg))
            np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
            print(f"wrote {name}.npz n={int(rec['n'])} draws={int(rec['draws'])} "
                  f"theta_norm={float(rec['theta_norm']):.6f}")
        return
    if only == "mlp":
        torch.set_num_threads(8)
        for name, (method, cfg) in MLP_CONFIGS.items():
            rec = run_mlp(methods, method, copy.deepcopy(cfg))
            np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
            print(f"wrote {name}.npz draws={int(rec['draws'])} evals={int(rec['n_evals'])}")
        return
    for name, (method, cfg) in CONFIGS.items():
        if only and name not in only.split(","):
            continue
        rec = run_method(methods, method, copy.deepcopy(cfg))
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **rec)
        print(f"wrote {path}: steps={rec['lrs'].shape[0]} n={rec['theta'].shape[1]}")
    if only:
        return
    np.savez_compressed(os.path.join(HERE, "schedule.npz"), **schedule_tables(methods))
    print("wrote schedule.npz")


if __name__ == "__main__":
    main()
