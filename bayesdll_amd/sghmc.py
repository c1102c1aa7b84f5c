"""SGHMC — drop-in for the reference's methods/sghmc.py Runner/Model.

Reference step (methods/sghmc.py:482-510, then SGD(momentum=0).step at :229):

    grad_U = g + (theta - theta0)/sigma^2/N        (uninformative bias: g)
    v      = v*(1-a) + lr*grad_U + nd*sqrt(2a/(N*lr)) * eps     (note the +)
    p.grad = g + v ;  theta -= lr * p.grad

Fused: one kernel per step, 24 B/element (theta r/w, g r, theta0 r, v r/w),
+16 B on collect steps (running moments as in methods/sghmc.py:236-249).
The Runner loop (burn-in seeding, thinning on the global iteration count,
evaluation by posterior sampling) is shared with SGLD.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from . import kernels as K
from ._base import FusedModelBase
from .sgld import Runner as _SGLDRunner


class Runner(_SGLDRunner):
    """methods/sghmc.py:16-406 (same loop as SGLD; SGD with momentum 0)."""

    def _make_model(self, args, hparams):
        return Model(ND=args.ND, prior_sig=float(hparams["prior_sig"]), bias=str(hparams["bias"]),
                     momentum_decay=float(hparams["momentum_decay"]))

    @staticmethod
    def _momentum(args):
        return 0

    def _extra_ckpt(self):
        """methods/sghmc.py:382: 'momentum_buffer' (name -> v) is saved too."""
        return {"momentum_buffer": {k: v.detach().clone()
                                    for k, v in self.model.momentum_buffer.items()}}

    def _load_extra(self, ckpt):
        """methods/sghmc.py:400-401."""
        mb = ckpt.get("momentum_buffer")
        if mb:
            self._state()  # bind the flat state first
            self.model.load_momentum_buffer(mb)


class Model(FusedModelBase):
    """SGHMC sampler step (methods/sghmc.py:409-512), fused on device."""

    need_prior = True
    need_mom = True

    def __init__(self, ND, prior_sig=1.0, bias="informative", momentum_decay=0.05):
        super().__init__()
        self.ND = ND
        self.prior_sig = prior_sig
        self.bias = bias
        self.momentum_decay = momentum_decay

    def forward(self, x, y, net, net0, criterion, lrs, Ninflate=1.0, nd=1.0, sgd=None,
                collect=None):
        N = self.ND * Ninflate
        lr_body, lr_head = (lrs[0], lrs[0]) if len(lrs) == 1 else (lrs[0], lrs[1])
        st = self.state_for(net, net0)
        loss, out = self.forward_backward(st, net, x, y, criterion)
        nmode = self.draw_noise(st)
        ns = [nd * np.sqrt(2 * self.momentum_decay / (N * lr)) for lr in (lr_body, lr_head)]
        common = dict(lrs=(lr_body, lr_head), noise_scale=ns, noise_mode=nmode,
                      one_minus_alpha=1 - self.momentum_decay, prior_sig=self.prior_sig,
                      sigma2=self.prior_sig ** 2, n_data=N, seed=self.seed, chain=self.chain,
                      step=self.step_count, div_mode=self.div_mode)
        if sgd is None:
            K.sgmcmc_step(st, L.SGHMC_GRAD, **common)  # .grad = g + v', momentum <- v'
        else:
            ckind, m1, m2, ca, cb = (L.COLLECT_NONE, None, None, 1.0, 1.0) if collect is None \
                else collect
            K.sgmcmc_step(st, L.SGHMC, **common, collect=ckind, mom1=m1, mom2=m2, collect_a=ca,
                          collect_b=cb)
        self.step_count += 1
        return self._result(loss, out)
