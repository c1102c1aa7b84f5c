"""SGLD — drop-in for the reference's methods/sgld.py (== src/bayesdll/sgld.py).

Reference step (methods/sgld.py:459-484, then torch.optim.SGD.step at :226):

    p.grad = g + (theta - theta0)/sigma^2/N + nd*sqrt(2/(N*lr)) * eps
             (uninformative bias: g + nd*sqrt(2/(N*lr)) * eps)
    buf    = grad (first step) | mu*buf + grad ;  theta -= lr*buf

plus, every `thin` iterations after burn-in, the running moments
m1 = (theta + cnt*m1)/(cnt+1), m2 = (theta^2 + cnt*m2)/(cnt+1) (:236-246).

Here the Runner hands the SGD configuration to the Model, which applies the
gradient, the SGD step and (on collect steps) the moment update in ONE
kernel: 24 B/element (theta r/w, g r, theta0 r, buf r/w), +16 B on collect
steps.  Used stand-alone (no `sgd=`), Model.forward keeps the reference
contract: it only fills .grad (one BDL_SGLD_GRAD sweep) for the caller's own
optimizer.step().
"""
from __future__ import annotations

import copy
import os
import time

import numpy as np
import torch

from . import _lib as L
from . import _runner as R
from . import kernels as K
from ._base import FusedModelBase


class FusedSGD:
    """torch.optim.SGD (weight_decay 0, dampening 0, no nesterov) fused into the step."""

    def __init__(self, optimizer, momentum):
        self.optimizer = optimizer
        self.momentum = float(momentum)
        self.has_buffer = False

    def lrs(self):
        g = self.optimizer.param_groups
        return (g[0]["lr"], g[1]["lr"] if len(g) > 1 else g[0]["lr"])

    def export_state(self, state, buf=None):
        """Expose the flat momentum buffer (state.mom, or `buf`) as the
        optimizer's per-param momentum_buffer (so optimizer.state_dict()
        matches torch's layout)."""
        if self.momentum == 0 or not self.has_buffer:
            return
        for p, v in zip(state.params, state.views(state.mom if buf is None else buf)):
            self.optimizer.state[p]["momentum_buffer"] = v

    def import_state(self, state, buf=None):
        """Inverse of export_state after optimizer.load_state_dict()."""
        bufs = [self.optimizer.state.get(p, {}).get("momentum_buffer") for p in state.params]
        dst = state.mom if buf is None else buf
        if dst is not None and bufs and all(b is not None for b in bufs):
            with torch.no_grad():
                for v, b in zip(state.views(dst), bufs):
                    v.copy_(b)
            self.has_buffer = True


class Runner:

    def __init__(self, net, net0, args, logger):
        self.args = R.bind_chain_log_dir(args)
        self.diverged_epochs = []
        self.logger = logger
        if args.pretrained is None:
            self.net0 = copy.deepcopy(net)
            with torch.no_grad():
                for _, p in self.net0.named_parameters():
                    p.zero_()
        else:
            self.net0 = net0
        self.net0 = self.net0.to(args.device)
        self.net = net.to(args.device)
        hparams = args.hparams
        self.model = self._make_model(args, hparams).to(args.device)
        if getattr(args, "noise_mode", None):
            self.model.noise_mode = args.noise_mode
        if getattr(args, "seed", None) is not None:
            self.model.seed = int(args.seed)
        if getattr(args, "graph", None) is not None:
            self.model.graph = bool(args.graph)
        if getattr(args, "overlap", None) is not None:
            self.model.overlap = bool(args.overlap)
        self.optimizer = torch.optim.SGD(
            [{"params": [p for pn, p in self.net.named_parameters()
                         if self.net.readout_name not in pn], "lr": args.lr},
             {"params": [p for pn, p in self.net.named_parameters()
                         if self.net.readout_name in pn], "lr": args.lr_head}],
            momentum=self._momentum(args), weight_decay=0)
        self.sgd = FusedSGD(self.optimizer, self._momentum(args))
        self.criterion = torch.nn.CrossEntropyLoss()
        self.Ninflate = float(hparams["Ninflate"])
        self.nd = float(hparams["nd"])
        self.burnin = int(hparams["burnin"])
        self.thin = int(hparams["thin"])
        self.nst = int(hparams["nst"])

    def _make_model(self, args, hparams):
        return Model(ND=args.ND, prior_sig=float(hparams["prior_sig"]), bias=str(hparams["bias"]))

    @staticmethod
    def _momentum(args):
        return args.momentum

    def _state(self):
        return self.model.state_for(self.net, self.net0)

    # ------------------------------------------------------------------ train
    def seed_moments(self):
        """methods/sgld.py:95-102: m1 = theta*1.0, m2 = theta**2, cnt = 1."""
        st = self._state()
        self.post_theta_mom1 = torch.empty_like(st.theta)
        self.post_theta_mom2 = torch.empty_like(st.theta) if self.nst > 0 else None
        K.moments_update(st.theta, self.post_theta_mom1, self.post_theta_mom2, L.COLLECT_MEAN_INIT,
                         div_mode=self.model.div_mode)
        self.post_theta_cnt = 1

    def train(self, train_loader, val_loader, test_loader, start_epoch=0):
        """methods/sgld.py:69-190; start_epoch > 0 continues a chain restored
        with load_ckpt(..., resume=True)."""
        args, logger = self.args, self.logger
        logger.info("Start training...")
        losses_train = np.zeros(args.epochs)
        errors_train = np.zeros(args.epochs)
        losses_test = np.zeros(args.epochs)
        errors_test = np.zeros(args.epochs)
        losses_val = np.zeros(args.epochs) if val_loader is not None else None
        errors_val = np.zeros(args.epochs) if val_loader is not None else None
        best_loss = np.inf
        tic0 = time.time()
        bi = start_epoch * len(train_loader)  # the global iteration count thinning uses
        for ep in range(start_epoch, args.epochs):
            if ep == self.burnin:
                logger.info("(leaving burnin period) start collecting posterior samples")
                self.seed_moments()
            tic = time.time()
            losses_train[ep], errors_train[ep], bi = self.train_one_epoch(
                train_loader, collect=(ep >= self.burnin), bi=bi)
            R.check_divergence(self, ep)
            R.log_update_stats(self, ep)
            logger.info(f"[Epoch {ep}/{args.epochs}] Training summary: loss = "
                        f"{losses_train[ep]:.4f}, prediction error = {errors_train[ep]:.4f} "
                        f"(time: {time.time() - tic:.4f} seconds)")
            if ep % args.test_eval_freq == 0 and ep >= self.burnin:
                if val_loader is not None:
                    losses_val[ep], errors_val[ep], tv, lv, lav = self.evaluate(val_loader)
                    logger.info(f"(Epoch {ep}) Validation summary: loss = {losses_val[ep]:.4f}, "
                                f"prediction error = {errors_val[ep]:.4f}")
                losses_test[ep], errors_test[ep], tt, lt, lat = self.evaluate(test_loader)
                logger.info(f"(Epoch {ep}) Test summary: loss = {losses_test[ep]:.4f}, "
                            f"prediction error = {errors_test[ep]:.4f}")
                loss_now = losses_val[ep] if val_loader is not None else losses_test[ep]
                if loss_now < best_loss:
                    best_loss = loss_now
                    logger.info(f"Best evaluation loss so far! @epoch {ep}: loss = {loss_now}")
                    self.save_ckpt(ep)
                    if val_loader is not None:
                        R.save_logits(args, tv, lv, lav, suffix="val")
                    R.save_logits(args, tt, lt, lat, suffix="test")
                    R.log_calibration(self, tt, lt, *((tv, lv) if val_loader is not None
                                                      else (None, None)))
        toc0 = time.time()
        logger.info("Training done! Total time = %f (average per epoch = %f) seconds" %
                    (toc0 - tic0, (toc0 - tic0) / args.epochs))

    def train_one_epoch(self, train_loader, collect, bi):
        """methods/sgld.py:193-250 with Model + SGD step + moments fused."""
        R.defer_loss(self)
        args, logger = self.args, self.logger
        self.net.train()
        loss, error, nb = 0, 0, 0
        errs = []
        for x, y in train_loader:
            x, y = x.to(args.device), y.to(args.device)
            do_collect = collect and (bi + 1) % self.thin == 0
            spec = None
            if do_collect:
                spec = (L.COLLECT_MEAN, self.post_theta_mom1,
                        self.post_theta_mom2 if self.nst > 0 else None,
                        float(self.post_theta_cnt), float(self.post_theta_cnt + 1))
            loss_, out = self.model(x, y, self.net, self.net0, self.criterion,
                                    [pg["lr"] for pg in self.optimizer.param_groups],
                                    self.Ninflate, self.nd, sgd=self.sgd, collect=spec)
            pred = out.data.max(dim=1)[1]
            err = pred.ne(y.data).sum()
            loss = R.add_loss(loss, loss_, len(y))
            errs.append(err)  # summed once per epoch: no second host sync per step
            nb += len(y)
            bi += 1
            if do_collect:
                logger.info("(post-burnin) accumulate posterior samples")
                self.post_theta_cnt += 1
        error = int(torch.stack(errs).sum().item()) if errs else 0
        self.model.defer_loss = False  # Model called directly: loss.item() again
        return float(loss) / nb, error / nb, bi

    # --------------------------------------------------------------- evaluate
    def get_var_source(self):
        """methods/sgld.py:324-350: ratio = cnt/(cnt-1) (1.0 if cnt <= 1)."""
        cnt = self.post_theta_cnt
        ratio = cnt / (cnt - 1) if cnt > 1 else 1.0
        return self.post_theta_mom2, L.VAR_RAW_MOMENTS, ratio

    def get_mean_vars_from_moments(self):
        """methods/sgld.py:324-350: net-shaped posterior mean and (if nst > 0)
        variance ratio*(m2 - m1^2) clamped at 1e-12.  The fused evaluation
        path (`evaluate`) never materialises these; this is the reference's
        public helper, computed with the same torch ops on the device."""
        with torch.no_grad():
            post_theta_mean = copy.deepcopy(self.net)
            torch.nn.utils.vector_to_parameters(self.post_theta_mom1,
                                                post_theta_mean.parameters())
        post_theta_vars = None
        if self.nst > 0:
            cnt = self.post_theta_cnt
            ratio = cnt / (cnt - 1) if cnt > 1 else 1.0
            with torch.no_grad():
                vec = ratio * (self.post_theta_mom2 - self.post_theta_mom1 ** 2)
                vec.clamp_(min=1e-12)
                post_theta_vars = copy.deepcopy(self.net)
                torch.nn.utils.vector_to_parameters(vec, post_theta_vars.parameters())
        return post_theta_mean, post_theta_vars

    def evaluate(self, test_loader):
        m2, mode, ratio = self.get_var_source() if self.nst > 0 else (None, L.VAR_GIVEN, 1.0)
        return R.sample_average_evaluate(self, test_loader, self.post_theta_mom1, m2, mode, ratio)

    def save_logits(self, targets, logits, logits_all, suffix=None):
        return R.save_logits(self.args, targets, logits, logits_all, suffix)

    def save_ckpt(self, epoch):
        """methods/sgld.py:367-385 — same file name and keys."""
        fname = os.path.join(self.args.log_dir, "ckpt.pt")
        self._export_sgd()
        torch.save({"last_theta": self.net.state_dict(),
                    "post_theta_mom1": self.post_theta_mom1,
                    "post_theta_mom2": self.post_theta_mom2 if self.nst > 0 else None,
                    "post_theta_cnt": self.post_theta_cnt,
                    "prior_sig": self.model.prior_sig,
                    "optimizer": self.optimizer.state_dict(),
                    **self._extra_ckpt(),
                    **({"resume": R.resume_state(self.model, self._state(), sgd=self.sgd)}
                       if getattr(self.args, "resume_state", False) else {}),
                    "epoch": epoch}, fname)
        return fname

    def load_ckpt(self, ckpt_path, exact_count=False, resume=False):
        """methods/sgld.py:388-398. The reference sets post_theta_cnt = epoch
        (:394); kept by default for drop-in parity, exact_count=True restores
        the saved count instead.  resume=True (checkpoint saved under
        args.resume_state) restores theta, the sampler's buffers, step counter
        and RNG states as well, so train(..., start_epoch=epoch + 1) continues
        the chain exactly."""
        ckpt = R.load_checkpoint(ckpt_path, self.args.device)
        self.post_theta_mom1 = ckpt["post_theta_mom1"]
        if ckpt["post_theta_mom2"] is not None:
            self.post_theta_mom2 = ckpt["post_theta_mom2"]
        exact = exact_count or resume
        self.post_theta_cnt = ckpt["post_theta_cnt"] if exact else ckpt["epoch"]
        self.model.prior_sig = ckpt["prior_sig"]
        self.optimizer.load_state_dict(ckpt["optimizer"])
        self._load_extra(ckpt)
        if resume:
            R.restore_resume_state(self.model, self._state(), ckpt, sgd=self.sgd)
        return ckpt["epoch"]

    # checkpoint hooks: SGLD's flat state.mom is the SGD momentum buffer
    def _export_sgd(self):
        self.sgd.export_state(self._state())

    def _extra_ckpt(self):
        return {}

    def _load_extra(self, ckpt):
        self.sgd.import_state(self._state())


class Model(FusedModelBase):
    """SGLD sampler step (methods/sgld.py:401-486), fused on device."""

    need_prior = True
    need_mom = True  # SGD momentum buffer (used when momentum != 0)

    def __init__(self, ND, prior_sig=1.0, bias="informative"):
        super().__init__()
        self.ND = ND
        self.prior_sig = prior_sig
        self.bias = bias

    def forward(self, x, y, net, net0, criterion, lrs, Ninflate=1.0, nd=1.0, sgd=None,
                collect=None, clip_grad=None):
        N = self.ND * Ninflate
        lr_body, lr_head = (lrs[0], lrs[0]) if len(lrs) == 1 else (lrs[0], lrs[1])
        st = self.state_for(net, net0)
        loss, out = self.forward_backward(st, net, x, y, criterion)
        nmode = self.draw_noise(st)
        ns = [nd * np.sqrt(2 / (N * lr)) for lr in (lr_body, lr_head)]
        common = dict(lrs=(lr_body, lr_head), noise_scale=ns, noise_mode=nmode,
                      prior_sig=self.prior_sig, sigma2=self.prior_sig ** 2, n_data=N,
                      seed=self.seed, chain=self.chain, step=self.step_count,
                      div_mode=self.div_mode)
        if sgd is None:
            # reference contract: only .grad is written (the caller steps)
            K.sgmcmc_step(st, L.SGLD_GRAD, **common)
        else:
            ckind, m1, m2, ca, cb = (L.COLLECT_NONE, None, None, 1.0, 1.0) if collect is None \
                else collect
            mom = sgd.momentum != 0
            first = mom and not sgd.has_buffer
            kw = dict(common, lrs=sgd.lrs(), mu=sgd.momentum, first_step=first, momentum=mom,
                      collect=ckind, mom1=m1, mom2=m2, collect_a=ca, collect_b=cb)
            if clip_grad is not None:
                # csgld.py:250-253: clip_grad_norm_ between Model.forward and
                # optimizer.step -- norm, coefficient and update all on device
                K.sgld_step_clipped(st, clip_grad, **kw)
            else:
                K.sgmcmc_step(st, L.SGLD, **kw)
            if mom:
                sgd.has_buffer = True
        self.step_count += 1
        return self._result(loss, out)
