"""Cyclical SGHMC with cycle restarts and full-sample BMA — drop-in for the
reference's methods/csghmc_fs.py.

The per-step update and the per-cycle Welford moments are csghmc's
(methods/csghmc_fs.py:904-984 is methods/csghmc.py:673-780; quirks Q1/Q2
included), i.e. the same fused kernel.  What the variant adds around it:

* after a newly completed cycle is scored and checkpointed, the momentum is
  zeroed (`_reset_optimizer_states`, :119-131, :590-591) — a memset of the
  flat momentum buffer — and, with hparams perform_cold_restarts=true, the
  network is re-initialised (:93-117, :593-597), in place in the flat theta;
* in the last epochs of every cycle (:176-180) the network's state_dict is
  saved as full_samples_net_ep{ep}.pth and all such checkpoints are evaluated
  as an equal-weight Bayesian model average (`evaluate_full_samples`,
  :260-418), with results in bma_evaluation_results.pkl and
  logits_test_bma.pkl.
"""
from __future__ import annotations

import os
import pickle

import numpy as np
import torch

from . import _runner as R
from .csghmc import Model  # noqa: F401  (methods/csghmc_fs.py's Model is csghmc's)
from .csghmc import Runner as _CSGHMCRunner


class Runner(_CSGHMCRunner):
    """methods/csghmc_fs.py:17-900."""

    def __init__(self, net, net0, args, logger):
        super().__init__(net, net0, args, logger)
        hp = args.hparams
        self.perform_cold_restarts = str(hp.get("perform_cold_restarts", False)).lower() == "true"
        logger.info("Performing cold restarts: re-initializing network parameters at the start "
                    "of each cycle." if self.perform_cold_restarts else
                    "Cold restarts disabled: keeping network parameters across cycles.")
        self.cycle_last_models_metadata = {}
        self.all_model_metadata = []
        self.model_counter = 0
        self.models_dir = os.path.join(args.log_dir, "collected_models")
        os.makedirs(self.models_dir, exist_ok=True)

    # ---------------------------------------------------------- cycle ends
    def _reset_optimizer_states(self):
        """:119-131: zero the momentum (the csghmc Model has no m / v)."""
        st = self.model.flat
        if st is not None and st.mom is not None:
            st.mom.zero_()
        self.model.t = 0
        self.logger.info("All optimizer states (momentum, m, v, t) reset for new cycle.")

    def _reinitialize_network_fresh(self):
        """Cold restart: `_runner.reinit_network`, in place in the flat theta."""
        from . import _runner as R
        R.reinit_network(self.net)
        if self.model.flat is not None:
            self.model.flat.check_bound()

    def _cycle_completed(self, cycle_number):
        """:590-597."""
        self._reset_optimizer_states()
        if self.perform_cold_restarts and cycle_number >= 1:
            self.logger.info(f"Performing COLD RESTART for cycle {cycle_number + 1}")
            self._reinitialize_network_fresh()

    # ------------------------------------------------------- full samples
    def _epoch_end(self, ep, train_loader, val_loader, test_loader):
        """:165-180: point-estimate validation every 5 epochs; full-sample
        snapshots in the last epochs of each cycle, then the BMA evaluation."""
        args = self.args
        if val_loader is not None and (ep % 5 == 0 or ep == args.epochs - 1):
            pl, pe = self.evaluate_point_estimate(val_loader, self.net)
            self.logger.info(f"(Epoch {ep}) Point Estimate Val (Cycle {self.current_cycle} "
                             f"Mean): loss = {pl:.4f}, prediction error = {pe:.4f}")
        L = args.epochs // args.num_cycles
        if L > 0 and L - 4 < ep % L < L - 1:
            torch.save(self.net.state_dict(),
                       os.path.join(args.log_dir, f"full_samples_net_ep{ep}.pth"))
            self.evaluate_full_samples(train_loader, val_loader, test_loader,
                                       desc_prefix=f"Full Samples Epoch {ep}")

    def evaluate_full_samples(self, train_loader, val_loader, test_loader, desc_prefix="Full BMA"):
        """:260-418: equal-weight average of the saved networks' logits."""
        args = self.args
        files = sorted(f for f in os.listdir(args.log_dir)
                       if f.startswith("full_samples_net_ep") and f.endswith(".pth"))
        if not files:
            return None
        eval_net = R.PosteriorDraw(self.net, "philox", 0, 0).net  # detached copy
        results = {}
        for name, loader in (("train", train_loader), ("val", val_loader), ("test", test_loader)):
            if loader is None:
                continue
            targets, logit_sum, individual = None, None, []
            tot_loss, tot_err, tot_n, nmod = 0.0, 0, 0, 0
            for f in files:
                sd = torch.load(os.path.join(args.log_dir, f), map_location=args.device,
                                weights_only=True)
                eval_net.load_state_dict(sd)
                eval_net.eval()
                ys, outs, ml, me, mn = [], [], 0.0, 0, 0
                with torch.no_grad():
                    for x, y in loader:
                        x, y = x.to(args.device), y.to(args.device)
                        out = eval_net(x)
                        ml += self.criterion(out, y).item() * len(y)
                        me += out.data.max(dim=1)[1].ne(y.data).sum().item()
                        mn += len(y)
                        ys.append(y.cpu().numpy())
                        outs.append(out.cpu().numpy())
                lg = np.concatenate(outs, axis=0)
                if targets is None:
                    targets = np.concatenate(ys, axis=0)
                logit_sum = lg.copy() if logit_sum is None else logit_sum + lg
                individual.append(lg)
                tot_loss, tot_err, tot_n, nmod = tot_loss + ml, tot_err + me, tot_n + mn, nmod + 1
            bma = logit_sum / nmod
            bma_loss = float(self.criterion(torch.tensor(bma), torch.tensor(targets)).item())
            results[name] = {"loss": bma_loss, "error": float(np.mean(np.argmax(bma, 1) != targets)),
                             "num_models": nmod, "targets": targets, "logits": bma,
                             "logits_all": np.stack(individual, axis=2),
                             "individual_avg_loss": tot_loss / (tot_n * nmod),
                             "individual_avg_error": tot_err / (tot_n * nmod)}
            self.logger.info(f"{desc_prefix} BMA {name}: loss = {bma_loss:.4f}, "
                             f"error = {results[name]['error']:.4f} ({nmod} models)")
        with open(os.path.join(args.log_dir, "bma_evaluation_results.pkl"), "wb") as fh:
            pickle.dump(results, fh)
        if "test" in results:
            t = results["test"]
            R.save_logits(args, t["targets"], t["logits"], t["logits_all"], suffix="test_bma")
        return results
