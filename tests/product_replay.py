"""Drive the PRODUCT Runners (bayesdll_amd) on a FakeNet exactly the way
tests/golden/gen_golden.py drove the reference's, replaying the captured
reference noise through noise_mode="external", and record the same
trajectories (theta and momentum before every step and after the last)."""
import logging
import tempfile
from types import SimpleNamespace

import numpy as np
import torch

from fakenet import FakeNet, fake_loader


def make_args(fx, tmp, device, **over):
    cfg = fx["config"]
    a = dict(device=device, ND=cfg["ND"],
             pretrained=("fake" if cfg.get("prior_seed") is not None else None),
             lr=cfg["lr"], lr_head=cfg["lr_head"], momentum=cfg.get("momentum", 0.0),
             epochs=cfg["epochs"], num_cycles=cfg.get("num_cycles", 2),
             proportion_exploration=cfg.get("beta", 0.5), full_sample=False, test_eval_freq=1,
             ece_num_bins=15, log_dir=tmp, num_classes=10,
             hparams={k: str(v) for k, v in cfg["hparams"].items()})
    if cfg.get("clip_grad") is not None:
        a["clip_grad"] = cfg["clip_grad"]
    a.update(over)
    return SimpleNamespace(**a)


def replay(fx, device="cuda", noise_mode="external", div_mode="true", runner_hook=None):
    import bayesdll_amd.adam_csghmc as adam_csghmc
    import bayesdll_amd.adam_sghmc as adam_sghmc
    import bayesdll_amd.csghmc as csghmc
    import bayesdll_amd.csghmc_fs as csghmc_fs
    import bayesdll_amd.csgld as csgld
    import bayesdll_amd.sghmc as sghmc
    import bayesdll_amd.sgld as sgld
    mods = dict(csghmc=csghmc, csghmc_fs=csghmc_fs, csgld=csgld, sgld=sgld, sghmc=sghmc, adam_sghmc=adam_sghmc,
                adam_csghmc=adam_csghmc)
    cfg = fx["config"]
    method = cfg["method"]
    net = FakeNet(grad_seed=cfg["grad_seed"], grad_scale=cfg["grad_scale"],
                  init=fx["theta_init"]).to(device)
    net0 = FakeNet(init=fx["prior_mean"]).to(device) if cfg.get("prior_seed") is not None else None
    tmp = tempfile.mkdtemp(prefix="bdl_replay_")
    args = make_args(fx, tmp, device)
    runner = mods[method].Runner(net, net0, args, logging.getLogger("replay"))
    model = runner.model
    model.noise_mode = noise_mode
    model.div_mode = div_mode
    if noise_mode == "external":
        noise = torch.from_numpy(fx["noise"]).to(device)
        model.noise_provider = lambda step, buf: buf.copy_(noise[step])
    if runner_hook:
        runner_hook(runner)

    adam = method.startswith("adam_")
    rec = dict(theta=[], mom=[], adam_m=[], adam_v=[], sgd_buf=[])
    orig = type(model).forward

    def record(st):
        rec["theta"].append(st.theta.detach().cpu().numpy().copy())
        rec["mom"].append(st.mom.detach().cpu().numpy().copy())
        if adam:
            m, v = model.adam_buffers(st)
            rec["adam_m"].append(m.cpu().numpy().copy())
            rec["adam_v"].append(v.cpu().numpy().copy())
            b = model.sgd_buffer
            rec["sgd_buf"].append(np.zeros(st.n, np.float32) if b is None else b.cpu().numpy())

    def fwd(self, *a, **k):
        record(self.state_for(runner.net, getattr(runner, "net0", None)))
        return orig(self, *a, **k)

    model.forward = fwd.__get__(model)
    loader = fake_loader(cfg["bpe"], device=device)
    if method in ("csghmc", "csghmc_fs", "csgld", "adam_csghmc"):
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
    record(model.flat)
    out = {k: np.stack(v) for k, v in rec.items() if v}
    if method in ("csghmc", "csghmc_fs", "csgld", "adam_csghmc"):
        cycles = sorted(runner.cycle_theta_mom1.keys())
        out["cycles"] = np.array(cycles, np.int64)
        out["cycle_mom1"] = np.stack([runner.cycle_theta_mom1[c].cpu().numpy() for c in cycles])
        out["cycle_mom2"] = np.stack([runner.cycle_theta_mom2[c].cpu().numpy() for c in cycles])
        out["samples_per_cycle"] = np.array([runner.samples_per_cycle[c] for c in cycles])
        out["samples_collected"] = runner.samples_collected
        out["current_cycle"] = runner.current_cycle
    else:
        out["post_mom1"] = runner.post_theta_mom1.cpu().numpy()
        out["post_mom2"] = (runner.post_theta_mom2.cpu().numpy() if runner.nst > 0
                            else np.zeros(0, np.float32))
        out["post_cnt"] = runner.post_theta_cnt
    out["runner"] = runner
    return out
