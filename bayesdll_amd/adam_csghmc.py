"""Cyclical Adam-preconditioned SGHMC — drop-in for the reference's
methods/adam_csghmc.py Runner/Model.

Model (methods/adam_csghmc.py:765-863): Adam-SGHMC with grad_U = g/temperature
+ (theta - theta0)/sigma^2/N and p.grad = v_mom (not g + v_mom); the Runner
steps SGD with momentum 0 (:65-75) under the cyclical step size, keeps csgld's
per-cycle running means on sample steps (:345-360), and zeroes v_mom, m, v and
t at the end of every cycle (:372-378, again at :403 via
_reset_optimizer_states), optionally re-initialising the network
(perform_cold_restarts, :102-131, :406-409).

Everything per step is the fused Adam kernel (bayesdll_amd.adam_sghmc.Model
with grad_is_mom); the evaluation (Gaussian mixture over cycles, raw-moment
variance) and checkpoint format are csgld's, as in the reference.
"""
from __future__ import annotations

from .adam_sghmc import Model as _AdamModel
from .csgld import Runner as _CSGLDRunner


class Model(_AdamModel):
    """methods/adam_csghmc.py:733-863."""

    grad_is_mom = True


class Runner(_CSGLDRunner):
    """methods/adam_csghmc.py:17-730."""

    def __init__(self, net, net0, args, logger):
        self.temperature = float(args.hparams.get("temperature", 1.0))
        self.perform_cold_restarts = \
            str(args.hparams.get("perform_cold_restarts", False)).lower() == "true"
        super().__init__(net, net0, args, logger)
        logger.info("Performing cold restarts: re-initializing network parameters at the start "
                    "of each cycle." if self.perform_cold_restarts else
                    "Cold restarts disabled: keeping network parameters across cycles.")

    def _make_model(self, args, hparams):
        return Model(ND=args.ND, prior_sig=float(hparams["prior_sig"]), bias=str(hparams["bias"]),
                     momentum_decay=float(hparams["momentum_decay"]),
                     beta1=float(hparams.get("beta1", 0.9)),
                     beta2=float(hparams.get("beta2", 0.999)),
                     epsilon=float(hparams.get("epsilon", 1e-8)),
                     temperature=self.temperature)

    @staticmethod
    def _momentum(args):
        return 0  # :70 "Force SGD optimizer momentum to 0"

    def _reset_optimizer_states(self):
        """:119-131."""
        self.model.reset_adam()
        self.logger.info("All optimizer states (momentum, m, v, t) reset for new cycle.")

    def _cycle_end(self, cycle_number):
        """:372-378 — every last_in_cycle step."""
        self.logger.info(f"Resetting momentum states for new cycle {cycle_number}")
        self.model.reset_adam()

    def _cycle_completed(self, cycle_number):
        """:402-413."""
        self._reset_optimizer_states()
        if self.perform_cold_restarts and cycle_number >= 1:
            self.logger.info(f"Performing COLD RESTART: fresh random weights for cycle "
                             f"{cycle_number + 1}")
            self._reinitialize_network_fresh()

    def _reinitialize_network_fresh(self):
        """Cold restart: `_runner.reinit_network`, in place in the flat theta."""
        from . import _runner as R
        R.reinit_network(self.net)
        if self.model.flat is not None:
            self.model.flat.check_bound()

    def evaluate_simple(self, test_loader):
        """:544-576: plain forward pass of the current network."""
        from . import _runner as R
        out = R.evaluate_point_estimate(self, test_loader, self.net)
        self.net.train()
        return out
