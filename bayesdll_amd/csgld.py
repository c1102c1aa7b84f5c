"""Cyclical SGLD — drop-in for the reference's methods/csgld.py Runner/Model.

The Model is SGLD's (methods/csgld.py:598-682 is methods/sgld.py:401-486);
the Runner drives it with the cyclical step size (methods/cyclical.py), the
SGD step with momentum (methods/csgld.py:48-52, :253) and per-cycle running
moments on sample steps (methods/csgld.py:264-293):

    first sample of cycle c:  m1 = theta,  m2 = theta^2
    later:  cc = spc[c] + 1;  m = (x + (cc-1)*m) / cc   for x in {theta, theta^2}

all fused into the step's single sweep.
"""
from __future__ import annotations

import copy
import os
import time

import numpy as np
import torch

from . import _lib as L
from . import _runner as R
from .cyclical import CyclicalSGMCMC
from .sgld import FusedSGD
from .sgld import Model as _SGLDModel


class Model(_SGLDModel):
    """methods/csgld.py:598-682 (identical to SGLD's Model)."""


class Runner:

    def __init__(self, net, net0, args, logger):
        self.args = R.bind_chain_log_dir(args)
        self.diverged_epochs = []
        self.logger = logger
        # beyond the reference: a process group for a
        # data-parallel likelihood pass, and GMM weights over the chains
        self.likelihood_group = None
        self.gmm_over_chains = bool(getattr(args, "gmm_over_chains", False))
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
        self.cyclical_scheduler = CyclicalSGMCMC(
            base_lr=args.lr,
            nbr_of_cycles=args.num_cycles if hasattr(args, "num_cycles") else 10,
            epochs=args.epochs,
            proportion_exploration=(args.proportion_exploration
                                    if hasattr(args, "proportion_exploration") else 0.5))
        self.criterion = torch.nn.CrossEntropyLoss()
        self.Ninflate = float(hparams["Ninflate"])
        self.nd = float(hparams["nd"])
        self.nst = int(hparams["nst"])
        self.thin = int(hparams["thin"])
        self.samples_collected = 0
        self.current_cycle = 0
        self.samples_per_cycle = {}
        self.cycle_theta_mom1 = {}
        self.cycle_theta_mom2 = {}
        self.cycle_likelihoods = {}
        self.cycle_states = {}
        self.all_samples = {}

    def _make_model(self, args, hparams):
        return Model(ND=args.ND, prior_sig=float(hparams["prior_sig"]), bias=str(hparams["bias"]))

    @staticmethod
    def _momentum(args):
        return args.momentum

    def _state(self):
        return self.model.state_for(self.net, self.net0)

    def _cycle_end(self, cycle_number):
        """Hook at every last_in_cycle step, before the cycle bookkeeping."""

    def _cycle_completed(self, cycle_number):
        """Hook after a newly completed cycle was scored and checkpointed."""

    def train(self, train_loader, val_loader, test_loader, start_epoch=0):
        args, logger = self.args, self.logger
        logger.info("Start training with Cyclical SGLD (fused MI355X kernel)...")
        losses_train = np.zeros(args.epochs)
        errors_train = np.zeros(args.epochs)
        losses_test = np.zeros(args.epochs)
        errors_test = np.zeros(args.epochs)
        losses_val = np.zeros(args.epochs) if val_loader is not None else None
        errors_val = np.zeros(args.epochs) if val_loader is not None else None
        best_loss = np.inf
        tic0 = time.time()
        for ep in range(start_epoch, args.epochs):
            self.cyclical_scheduler.current_epoch = ep
            tic = time.time()
            losses_train[ep], errors_train[ep], cycle_updated = self.train_one_epoch(train_loader)
            R.check_divergence(self, ep)
            R.log_update_stats(self, ep)
            logger.info(f"[Epoch {ep}/{args.epochs}] Training summary: loss = "
                        f"{losses_train[ep]:.4f}, prediction error = {errors_train[ep]:.4f} "
                        f"(time: {time.time() - tic:.4f} seconds)")
            if cycle_updated:
                if val_loader is not None:
                    losses_val[ep], errors_val[ep], tv, lv, lav = self.evaluate(val_loader)
                losses_test[ep], errors_test[ep], tt, lt, lat = self.evaluate(test_loader)
                logger.info(f"(Epoch {ep}) Test summary: loss = {losses_test[ep]:.4f}, "
                            f"prediction error = {errors_test[ep]:.4f}")
                loss_now = losses_val[ep] if val_loader is not None else losses_test[ep]
                if loss_now < best_loss:
                    best_loss = loss_now
                    if val_loader is not None:
                        R.save_logits(args, tv, lv, lav, suffix="val")
                    R.save_logits(args, tt, lt, lat, suffix="test")
                    R.log_calibration(self, tt, lt, *((tv, lv) if val_loader is not None
                                                      else (None, None)))
        toc0 = time.time()
        logger.info(f"Training done! Total time = {toc0 - tic0:.4f} seconds")
        return {"losses_train": losses_train, "errors_train": errors_train,
                "losses_val": losses_val, "errors_val": errors_val, "losses_test": losses_test,
                "errors_test": errors_test, "samples_per_cycle": self.samples_per_cycle}

    def train_one_epoch(self, train_loader):
        """methods/csgld.py:195-331, with Model + clip + SGD + moments fused."""
        R.defer_loss(self)
        args, logger = self.args, self.logger
        self.net.train()
        loss, error, nb = 0, 0, 0
        errs = []
        cycle_updated = False
        bpe = len(train_loader)
        sched = self.cyclical_scheduler
        st = self._state()
        for batch_idx, (x, y) in enumerate(train_loader):
            ep = sched.current_epoch
            current_lr = sched.calculate_lr(epoch=ep, batch=batch_idx, batches_per_epoch=bpe)
            should_sample = sched.should_sample(epoch=ep, batch=batch_idx,
                                                batches_per_epoch=bpe) and batch_idx % self.thin == 0
            last_in_cycle = sched.last_in_cycle(epoch=ep, batch=batch_idx, batches_per_epoch=bpe)
            for i, pg in enumerate(self.optimizer.param_groups):
                pg["lr"] = current_lr * (args.lr_head / args.lr) if i == 1 else current_lr
            x, y = x.to(args.device), y.to(args.device)

            spec, cycle_number = None, None
            if should_sample:
                cycle_number = sched.get_cycle_number(epoch=ep, batch=batch_idx,
                                                      batches_per_epoch=bpe)
                if cycle_number not in self.cycle_theta_mom1:
                    self.cycle_theta_mom1[cycle_number] = torch.empty_like(st.theta)
                    self.cycle_theta_mom2[cycle_number] = torch.empty_like(st.theta)
                    spec = (L.COLLECT_MEAN_INIT, self.cycle_theta_mom1[cycle_number],
                            self.cycle_theta_mom2[cycle_number], 1.0, 1.0)
                else:
                    cc = self.samples_per_cycle.get(cycle_number, 0) + 1
                    spec = (L.COLLECT_MEAN, self.cycle_theta_mom1[cycle_number],
                            self.cycle_theta_mom2[cycle_number], float(cc - 1), float(cc))

            clip = args.clip_grad if hasattr(args, "clip_grad") else None
            loss_, out = self.model(x, y, self.net, self.net0, self.criterion,
                                    [pg["lr"] for pg in self.optimizer.param_groups],
                                    self.Ninflate, self.nd, sgd=self.sgd, collect=spec,
                                    clip_grad=clip)
            pred = out.data.max(dim=1)[1]
            err = pred.ne(y.data).sum()
            loss = R.add_loss(loss, loss_, len(y))
            errs.append(err)  # summed once per epoch: no second host sync per step
            nb += len(y)

            if should_sample:
                if args.full_sample if hasattr(args, "full_sample") else False:
                    self.all_samples[f"{ep}_{batch_idx}"] = st.theta.clone()
                self.samples_collected += 1
                self.samples_per_cycle[cycle_number] = self.samples_per_cycle.get(cycle_number, 0) + 1
                if batch_idx % 50 == 0:
                    logger.info(f"Sampling phase: collecting posterior sample at lr={current_lr:.6f}")
            if last_in_cycle:
                cycle_number = sched.get_cycle_number(epoch=ep, batch=batch_idx,
                                                      batches_per_epoch=bpe)
                self._cycle_end(cycle_number)
                self.cycle_states[cycle_number] = copy.deepcopy(self.net.state_dict())
                if cycle_number > self.current_cycle:
                    cycle_updated = True
                    self.current_cycle = cycle_number
                    likelihood = np.array(self.full_batch_likelihoods(train_loader))
                    self.cycle_likelihoods[cycle_number] = likelihood
                    with torch.no_grad():
                        self.save_ckpt(epoch=sched.current_epoch)
                    self._cycle_completed(cycle_number)
        error = int(torch.stack(errs).sum().item()) if errs else 0
        self.model.defer_loss = False  # Model called directly: loss.item() again
        return float(loss) / nb, error / nb, cycle_updated

    def _variance_source(self, cycle):
        """methods/csgld.py:394-400: ratio*(m2 - m1^2) (ratio = spc/(spc-1)
        when spc > 1, else no ratio); the reference computes spc/(spc-1) before
        its `> 1` test and so raises ZeroDivisionError on a 1-sample cycle —
        that case is treated as ratio 1 here."""
        spc = self.samples_per_cycle.get(cycle, 0)
        ratio = spc / (spc - 1) if spc > 1 else 1.0
        return self.cycle_theta_mom2[cycle], L.VAR_RAW_MOMENTS, ratio

    def evaluate(self, test_loader):
        return R.mixture_evaluate(self, test_loader, self._variance_source)

    def evaluate_point_estimate(self, data_loader, net_to_evaluate, desc_prefix="Point Estimate"):
        return R.evaluate_point_estimate(self, data_loader, net_to_evaluate)

    def save_logits(self, targets, logits, logits_all, suffix=None):
        return R.save_logits(self.args, targets, logits, logits_all, suffix)

    def save_ckpt(self, epoch):
        fname = os.path.join(self.args.log_dir, f"{self.current_cycle}_ckpt.pt")
        torch.save({"last_theta": self._state().theta.detach().clone(),
                    "cycle_theta_mom1": self.cycle_theta_mom1,
                    "cycle_theta_mom2": self.cycle_theta_mom2,
                    "cycle_likelihoods": self.cycle_likelihoods,
                    "cycle_states": self.cycle_states,
                    "epoch": epoch, "current_cycle": self.current_cycle,
                    "samples_per_cycle": self.samples_per_cycle,
                    **({"resume": R.resume_state(self.model, self._state(), sgd=self.sgd,
                                                 samples_collected=self.samples_collected)}
                       if getattr(self.args, "resume_state", False) else {})}, fname)
        return fname

    def load_ckpt(self, ckpt_path, resume=False):
        """methods/csgld.py (same keys restored); resume=True as in csghmc."""
        ckpt = R.load_checkpoint(ckpt_path, self.args.device)
        self.cycle_theta_mom1 = ckpt.get("cycle_theta_mom1", {})
        self.cycle_theta_mom2 = ckpt.get("cycle_theta_mom2", {})
        self.cycle_likelihoods = ckpt.get("cycle_likelihoods", {})
        self.current_cycle = ckpt.get("current_cycle", 0)
        self.samples_per_cycle = ckpt.get("samples_per_cycle", {})
        if resume:
            self.cycle_states = ckpt.get("cycle_states", self.cycle_states)
            extra = R.restore_resume_state(self.model, self._state(), ckpt, sgd=self.sgd)
            self.samples_collected = extra.get("samples_collected", self.samples_collected)
            self._cycle_completed(self.current_cycle)  # as csghmc.Runner.load_ckpt
        return ckpt["epoch"]

    def full_batch_likelihoods(self, train_loader, group=None):
        """methods/csgld.py:508-594 (as csghmc.Runner.full_batch_likelihoods)."""
        c = self.current_cycle
        m2, mode, ratio = self._variance_source(c)
        return R.full_batch_likelihoods(self, train_loader, self.cycle_theta_mom1[c], m2, mode,
                                        ratio, self._state().theta,
                                        group=group if group is not None else
                                        self.likelihood_group)

    def calculate_gmm_weights(self):
        return R.gmm_weights(self.cycle_likelihoods)
