"""Cyclical SGHMC — drop-in for the reference's methods/csghmc.py Runner/Model.

Same constructor, `train`, `train_one_epoch`, `evaluate`, `save_ckpt`,
`load_ckpt`, `full_batch_likelihoods`, `calculate_gmm_weights` and the same
`Model.forward(x, y, net, net0, criterion, lrs, Ninflate, nd, should_sample)`
contract (methods/csghmc.py:17-670, :673-780).  After autograd, ONE fused HIP
kernel applies, over the flat chain state,

    v     <- v*(1-a) - lr*(g + prior_sig*theta) [+ nd*sqrt(2*a*lr)/N * eps]
    theta <- theta + v

(methods/csghmc.py:759-778; Q1: the prior term is prior_sig*theta on both
branches, theta0 is never read) and, on sample steps, the Welford update of the
current cycle's moments on the new theta (methods/csghmc.py:327-345) in the
same sweep: 20 B/element on explore steps, 36 B/element on collect steps.

Reproducibility: the fused update gives the same bits in any process for the
same inputs and Philox key; the gradients come from PyTorch-ROCm autograd,
whose kernel choice for a shape can depend on what the process ran before.
A chain repeats bit for bit across processes with deterministic convolutions,
the math attention backend and a fresh process per chain.
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
from .cyclical import CyclicalSGMCMC
from .flat import moment_pair


class Runner:

    def __init__(self, net, net0, args, logger):
        self.args = R.bind_chain_log_dir(args)
        self.diverged_epochs = []
        self.logger = logger
        # beyond the reference: a process group for a
        # data-parallel likelihood pass, and GMM weights over the chains
        self.likelihood_group = None
        self.gmm_over_chains = bool(getattr(args, "gmm_over_chains", False))
        # prior backbone (zeros if not pretrained) — kept for API parity; the
        # cSGHMC update never reads it (Q1, methods/csghmc.py:759-762)
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
        self.model = Model(ND=args.ND, prior_sig=float(hparams["prior_sig"]), runner=self,
                           bias=str(hparams["bias"]),
                           momentum_decay=float(hparams["momentum_decay"])).to(args.device)
        if hasattr(args, "noise_mode") and args.noise_mode:
            self.model.noise_mode = args.noise_mode
        if hasattr(args, "seed") and args.seed is not None:
            self.model.seed = int(args.seed)
        if getattr(args, "graph", None) is not None:
            self.model.graph = bool(args.graph)
        if getattr(args, "overlap", None) is not None:
            self.model.overlap = bool(args.overlap)

        # lr holder with the reference's two param groups (body, head)
        self.optimizer = torch.optim.SGD(
            [{"params": [p for pn, p in self.net.named_parameters()
                         if self.net.readout_name not in pn], "lr": args.lr},
             {"params": [p for pn, p in self.net.named_parameters()
                         if self.net.readout_name in pn], "lr": args.lr_head}],
            momentum=0, weight_decay=0)

        self.cyclical_scheduler = CyclicalSGMCMC(
            base_lr=args.lr,
            nbr_of_cycles=args.num_cycles if hasattr(args, "num_cycles") else 10,
            epochs=args.epochs,
            proportion_exploration=(args.proportion_exploration
                                    if hasattr(args, "proportion_exploration") else 0.5))
        self.criterion = torch.nn.CrossEntropyLoss()

        self.Ninflate = float(hparams["Ninflate"])
        self.nd = float(hparams["nd"])
        self.burnin = int(hparams["burnin"])
        self.thin = int(hparams["thin"])
        self.nst = int(hparams["nst"])

        self.samples_collected = 0
        self.current_cycle = 0
        self.samples_per_cycle = {}
        self.cycle_theta_mom1 = {}
        self.cycle_theta_mom2 = {}
        self.cycle_likelihoods = {}
        self.cycle_states = {}

    # ------------------------------------------------------------------ train
    def train(self, train_loader, val_loader, test_loader, start_epoch=0):
        """methods/csghmc.py:87-209; start_epoch > 0 continues a chain restored
        with load_ckpt(..., resume=True)."""
        args, logger = self.args, self.logger
        logger.info("Start training with Cyclical SGHMC (fused MI355X kernel)...")
        losses_train = np.zeros(args.epochs)
        errors_train = np.zeros(args.epochs)
        losses_val = np.zeros(args.epochs) if val_loader is not None else None
        errors_val = np.zeros(args.epochs) if val_loader is not None else None
        losses_test = np.zeros(args.epochs)
        errors_test = np.zeros(args.epochs)
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
            self._epoch_end(ep, train_loader, val_loader, test_loader)
            if cycle_updated:
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
                    if val_loader is not None:
                        R.save_logits(args, tv, lv, lav, suffix="val")
                    R.save_logits(args, tt, lt, lat, suffix="test")
                    R.log_calibration(self, tt, lt, *((tv, lv) if val_loader is not None
                                                      else (None, None)))
        toc0 = time.time()
        logger.info(f"Training done! Total time = {toc0 - tic0:.4f} "
                    f"(average per epoch = {(toc0 - tic0) / args.epochs:.4f}) seconds")
        logger.info(f"Total samples collected: {self.samples_collected} across "
                    f"{self.current_cycle} cycles")
        return {"losses_train": losses_train, "errors_train": errors_train,
                "losses_val": losses_val, "errors_val": errors_val, "losses_test": losses_test,
                "errors_test": errors_test, "samples_per_cycle": self.samples_per_cycle}

    def evaluate_point_estimate(self, data_loader, net_to_evaluate, desc_prefix="Point Estimate"):
        return R.evaluate_point_estimate(self, data_loader, net_to_evaluate)

    def _collect_spec(self, cycle_number):
        """Welford bookkeeping exactly as methods/csghmc.py:333-348 (quirk Q2:
        samples_per_cycle is bumped twice per sample). Returns the kernel's
        collect mode, buffers and divisor, plus the count to store."""
        st = self.model.state_for(self.net)
        if cycle_number not in self.cycle_theta_mom1:
            m1, m2 = moment_pair(st.n, st.device)
            self.cycle_theta_mom1[cycle_number] = m1
            self.cycle_theta_mom2[cycle_number] = m2
            return (L.COLLECT_WELFORD_INIT, m1, m2, 1.0), 1
        n = self.samples_per_cycle.get(cycle_number, 0) + 1
        return (L.COLLECT_WELFORD, self.cycle_theta_mom1[cycle_number],
                self.cycle_theta_mom2[cycle_number], float(n)), n

    def train_one_epoch(self, train_loader):
        """methods/csghmc.py:246-384 with the update + Welford fused on device."""
        R.defer_loss(self)
        args, logger = self.args, self.logger
        self.net.train()
        loss, error, nb_samples = 0, 0, 0
        errs = []
        cycle_updated = False
        bpe = len(train_loader)
        sched = self.cyclical_scheduler
        for batch_idx, (x, y) in enumerate(train_loader):
            ep = sched.current_epoch
            current_lr = sched.calculate_lr(epoch=ep, batch=batch_idx, batches_per_epoch=bpe)
            should_sample = sched.should_sample(epoch=ep, batch=batch_idx,
                                                batches_per_epoch=bpe) and batch_idx % self.thin == 0
            last_in_cycle = sched.last_in_cycle(epoch=ep, batch=batch_idx, batches_per_epoch=bpe)
            for i, pg in enumerate(self.optimizer.param_groups):
                pg["lr"] = current_lr * (args.lr_head / args.lr) if i == 1 else current_lr
            x, y = x.to(args.device), y.to(args.device)

            collect, new_count, cycle_number = None, None, None
            if should_sample:
                cycle_number = sched.get_cycle_number(epoch=ep, batch=batch_idx,
                                                      batches_per_epoch=bpe)
                collect, new_count = self._collect_spec(cycle_number)

            loss_, out = self.model(x, y, self.net, self.net0, self.criterion,
                                    [pg["lr"] for pg in self.optimizer.param_groups],
                                    self.Ninflate, self.nd, should_sample=should_sample,
                                    collect=collect)
            if hasattr(args, "clip_grad") and args.clip_grad is not None:
                # after the update, as in the reference (:301-302): no effect on theta
                torch.nn.utils.clip_grad_norm_(self.net.parameters(), args.clip_grad)

            pred = out.data.max(dim=1)[1]
            err = pred.ne(y.data).sum()
            loss = R.add_loss(loss, loss_, len(y))
            errs.append(err)  # summed once per epoch: no second host sync per step
            nb_samples += len(y)

            if should_sample:
                if batch_idx % 50 == 0:
                    logger.info(f"Sampling phase: collecting posterior sample at lr={current_lr:.6f}")
                self.samples_per_cycle[cycle_number] = new_count
                self.samples_collected += 1
                self.samples_per_cycle[cycle_number] = self.samples_per_cycle.get(cycle_number, 0) + 1
            elif batch_idx % 50 == 0:
                logger.info(f"Exploration phase: lr={current_lr:.6f}")

            if last_in_cycle:
                cycle_number = sched.get_cycle_number(epoch=ep, batch=batch_idx,
                                                      batches_per_epoch=bpe)
                self.cycle_states[cycle_number] = copy.deepcopy(self.net.state_dict())
                if cycle_number > self.current_cycle:
                    cycle_updated = True
                    self.current_cycle = cycle_number
                    logger.info(f"Completed cycle {cycle_number}")
                    likelihood = np.array(self.full_batch_likelihoods(train_loader))
                    self.cycle_likelihoods[cycle_number] = likelihood
                    logger.info(f"Cycle {cycle_number} full batch likelihood: "
                                f"{likelihood.mean():.6e}")
                    with torch.no_grad():
                        self.save_ckpt(epoch=sched.current_epoch)
                    self._cycle_completed(cycle_number)
        error = int(torch.stack(errs).sum().item()) if errs else 0
        self.model.defer_loss = False  # Model called directly: loss.item() again
        return float(loss) / nb_samples, error / nb_samples, cycle_updated

    def _cycle_completed(self, cycle_number):
        """Hook after a newly completed cycle was scored and checkpointed."""

    def _epoch_end(self, ep, train_loader, val_loader, test_loader):
        """Hook after each epoch's training summary (before evaluation)."""

    # --------------------------------------------------------------- evaluate
    def _variance_source(self, cycle):
        """Welford variance M2/(n-1), or 1e-12 for a single sample (:451-459)."""
        n_samples = self.samples_per_cycle.get(cycle, 0)
        if cycle in self.cycle_theta_mom2 and n_samples > 1:
            return self.cycle_theta_mom2[cycle], L.VAR_WELFORD, float(n_samples - 1)
        return None, L.VAR_GIVEN, 1.0

    def evaluate(self, test_loader):
        return R.mixture_evaluate(self, test_loader, self._variance_source)

    def save_logits(self, targets, logits, logits_all, suffix=None):
        return R.save_logits(self.args, targets, logits, logits_all, suffix)

    def save_ckpt(self, epoch):
        """methods/csghmc.py:530-549 — same file name and keys; the flat theta
        buffer IS parameters_to_vector(net.parameters()).  With
        args.resume_state (not in the reference, whose resume is inexact: it
        saves no momentum) a "resume" entry adds what an exact
        continuation needs: momentum, the sampler's step counter (the Philox
        key), samples_collected and the torch RNG states."""
        fname = os.path.join(self.args.log_dir, f"{self.current_cycle}_ckpt.pt")
        st = self.model.state_for(self.net)
        ck = {"last_theta": st.theta.detach().clone(),
              "cycle_theta_mom1": self.cycle_theta_mom1,
              "cycle_theta_mom2": self.cycle_theta_mom2,
              "cycle_likelihoods": self.cycle_likelihoods,
              "cycle_states": self.cycle_states,
              "epoch": epoch,
              "current_cycle": self.current_cycle,
              "samples_per_cycle": self.samples_per_cycle}
        if getattr(self.args, "resume_state", False):
            ck["resume"] = R.resume_state(self.model, st, samples_collected=self.samples_collected)
        torch.save(ck, fname)
        return fname

    def load_ckpt(self, ckpt_path, resume=False):
        """methods/csghmc.py:552-566 (same keys restored).  resume=True (with a
        checkpoint saved under args.resume_state) also restores theta, the
        momentum, the step counter and RNG states, so that
        `train(..., start_epoch=epoch + 1)` continues the chain exactly."""
        ckpt = R.load_checkpoint(ckpt_path, self.args.device)
        self.cycle_theta_mom1 = ckpt.get("cycle_theta_mom1", {})
        self.cycle_theta_mom2 = ckpt.get("cycle_theta_mom2", {})
        self.cycle_likelihoods = ckpt.get("cycle_likelihoods", {})
        self.current_cycle = ckpt.get("current_cycle", 0)
        self.samples_per_cycle = ckpt.get("samples_per_cycle", {})
        if resume:
            self.cycle_states = ckpt.get("cycle_states", self.cycle_states)
            st = self.model.state_for(self.net)
            extra = R.restore_resume_state(self.model, st, ckpt)
            self.samples_collected = extra.get("samples_collected", self.samples_collected)
            # the checkpoint is written at a cycle's completion, before the
            # cycle-end hook (momentum / optimizer reset, cold restart): replay it
            self._cycle_completed(self.current_cycle)
        return ckpt["epoch"]

    def full_batch_likelihoods(self, train_loader, group=None):
        """methods/csghmc.py:568-638: nst draws from the current cycle's
        Gaussian, each scored on the full training set; returns exp(-loss).
        group (or self.likelihood_group): a data-parallel pass over the
        group's ranks, one all-reduce of the loss sums (_runner)."""
        c = self.current_cycle
        m2, var_mode, ratio = self._variance_source(c)
        return R.full_batch_likelihoods(self, train_loader, self.cycle_theta_mom1[c], m2,
                                        var_mode, ratio, self.model.state_for(self.net).theta,
                                        group=group if group is not None else
                                        self.likelihood_group)

    def calculate_gmm_weights(self):
        return R.gmm_weights(self.cycle_likelihoods)


class Model(FusedModelBase):
    """cSGHMC sampler step (methods/csghmc.py:673-780), fused on device."""

    need_prior = False  # Q1: theta0 never enters the csghmc update
    need_mom = True
    tune_method = "csghmc"

    def __init__(self, ND, runner=None, prior_sig=1.0, bias="informative", momentum_decay=0.05):
        super().__init__()
        self.ND = ND
        self.prior_sig = prior_sig
        self.bias = bias
        self.momentum_decay = momentum_decay
        self.runner = runner

    def forward(self, x, y, net, net0, criterion, lrs, Ninflate=1.0, nd=1.0, should_sample=False,
                collect=None):
        N = self.ND * Ninflate
        lr_body, lr_head = (lrs[0], lrs[0]) if len(lrs) == 1 else (lrs[0], lrs[1])
        st = self.state_for(net)
        noise_scale = [nd * np.sqrt((2 * self.momentum_decay * lr)) / N for lr in (lr_body, lr_head)]
        ckind, m1, m2, ca = (L.COLLECT_NONE, None, None, 1.0) if collect is None else collect
        kw = dict(lrs=(lr_body, lr_head), noise_scale=noise_scale,
                  one_minus_alpha=1 - self.momentum_decay, prior_sig=self.prior_sig,
                  collect=ckind, collect_a=ca, seed=self.seed, chain=self.chain,
                  step=self.step_count, div_mode=self.div_mode)
        if self.can_overlap(st):
            # update overlapped with backward, bucket by bucket (identical result)
            sl = (lambda v, a, b: None if v is None else v[a:b])
            nm = L.NOISE_PHILOX if should_sample else L.NOISE_NONE
            loss, out = self.forward_backward_overlapped(
                st, net, x, y, criterion,
                lambda sub, start: K.sgmcmc_step(
                    sub, L.CSGHMC, noise_mode=nm, mom1=sl(m1, start, start + sub.n),
                    mom2=sl(m2, start, start + sub.n), philox_offset=start // 4, **kw),
                kind=(nm, ckind, m2 is None))
            self.step_count += 1
            return self._result(loss, out)
        loss, out = self.forward_backward(st, net, x, y, criterion)
        # the reference draws randn_like on every step, even when the noise is
        # dropped (:766): the torch/external sources are advanced every step
        nmode = self.draw_noise(st)
        K.sgmcmc_step(st, L.CSGHMC, noise_mode=nmode if should_sample else L.NOISE_NONE,
                      mom1=m1, mom2=m2, **kw)
        self.step_count += 1
        return self._result(loss, out)
