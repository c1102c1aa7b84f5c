"""Adam-preconditioned SGHMC — drop-in for the reference's methods/adam_sghmc.py.

Reference step (methods/adam_sghmc.py:500-553, then SGD(args.momentum).step at
:229), per tensor, with t incremented once per call:

    grad_U = g + (theta - theta0)/sigma^2/N            (uninformative bias: g)
    m = beta1*m + (1-beta1)*grad_U ;  v = beta2*v + (1-beta2)*grad_U^2
    d = sqrt(v/(1-beta2^t)) + eps ;   pg = (m/(1-beta1^t)) / d
    v_mom = v_mom*(1-a) + lr*pg + nd*sqrt(2a*(1/d)/N) * eps
    p.grad = g + v_mom ;  SGD(momentum mu) steps theta

Fused: one kernel per step over the flat state, 40 B/element (theta, v_mom,
m, v r/w; g, theta0 r), 48 B with the SGD momentum buffer, +16 B on collect
steps.  The Runner loop (burn-in, thinning, posterior-sampling evaluation) is
SGLD's; the checkpoint adds the reference's momentum_buffer / m / v / t keys
(:379-418).
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import kernels as K
from ._base import FusedModelBase
from .sgld import Runner as _SGLDRunner


class Runner(_SGLDRunner):
    """methods/adam_sghmc.py:16-418 (SGLD's loop; SGD with args.momentum)."""

    def _make_model(self, args, hparams):
        return Model(ND=args.ND, prior_sig=float(hparams["prior_sig"]), bias=str(hparams["bias"]),
                     momentum_decay=float(hparams["momentum_decay"]),
                     beta1=float(hparams.get("beta1", 0.9)),
                     beta2=float(hparams.get("beta2", 0.999)),
                     epsilon=float(hparams.get("epsilon", 1e-8)))

    @staticmethod
    def _momentum(args):
        return args.momentum

    def _export_sgd(self):
        self.sgd.export_state(self._state(), buf=self.model.sgd_buffer)

    def _extra_ckpt(self):
        return self.model.adam_state_dict()

    def _load_extra(self, ckpt):
        self._state()
        self.model.load_adam_state(ckpt)
        if self.model.sgd_buffer is not None or self.sgd.momentum != 0:
            self.sgd.import_state(self._state(), buf=self.model.ensure_sgd_buffer())


class Model(FusedModelBase):
    """Adam-SGHMC sampler step (methods/adam_sghmc.py:429-556), fused on device.

    grad_is_mom / temperature select the cyclical variant's rule
    (methods/adam_csghmc.py:834, :860): p.grad = v_mom and g / temperature."""

    need_prior = True
    need_mom = True   # v_mom (the reference's momentum_buffer)
    tune_method = "adam"
    extra_vectors = K.ADAM_EXTRA  # adam_m, adam_v, sgd_buf
    grad_is_mom = False

    def __init__(self, ND, prior_sig=1.0, bias="informative", momentum_decay=0.05, beta1=0.9,
                 beta2=0.999, epsilon=1e-8, temperature=1.0):
        super().__init__()
        self.ND = ND
        self.prior_sig = prior_sig
        self.bias = bias
        self.momentum_decay = momentum_decay
        self.beta1 = beta1
        self.beta2 = beta2
        self.epsilon = epsilon
        self.temperature = temperature
        self.t = 0
        self._adam = None       # (state, m, v)
        self.sgd_buffer = None  # flat torch.optim.SGD momentum buffer (momentum != 0)

    # ------------------------------------------------------------ state
    def adam_buffers(self, st):
        if self._adam is None or self._adam[0] is not st:
            ex = getattr(st, "extra", {})
            m = ex["adam_m"] if "adam_m" in ex else torch.zeros_like(st.theta)
            v = ex["adam_v"] if "adam_v" in ex else torch.zeros_like(st.theta)
            self._adam = (st, m, v)
        return self._adam[1], self._adam[2]

    def ensure_sgd_buffer(self):
        if self.sgd_buffer is None:
            ex = getattr(self._state, "extra", {})
            self.sgd_buffer = ex["sgd_buf"] if "sgd_buf" in ex else \
                torch.zeros_like(self._state.theta)
        return self.sgd_buffer

    def _views(self, flat):
        st = self._state
        return {} if st is None else dict(zip(st.names, st.views(flat)))

    @property
    def m(self):
        """name -> first-moment view (the reference's Model.m dict)."""
        return {} if self._adam is None else self._views(self._adam[1])

    @property
    def v(self):
        """name -> second-moment view (the reference's Model.v dict)."""
        return {} if self._adam is None else self._views(self._adam[2])

    def reset_adam(self):
        """Zero v_mom, m, v and t (methods/adam_csghmc.py:372-378, :119-131)."""
        st = self._state
        if st is not None:
            st.mom.zero_()
            if self._adam is not None:
                self._adam[1].zero_()
                self._adam[2].zero_()
        self.t = 0

    def adam_state_dict(self):
        clone = lambda d: {k: t.detach().clone() for k, t in d.items()}  # noqa: E731
        return {"momentum_buffer": clone(self.momentum_buffer), "m": clone(self.m),
                "v": clone(self.v), "t": self.t}

    def load_adam_state(self, ckpt):
        """methods/adam_sghmc.py:407-418 (copied into the flat buffers)."""
        st = self._state
        m, v = self.adam_buffers(st)
        if ckpt.get("momentum_buffer"):
            self.load_momentum_buffer(ckpt["momentum_buffer"])
        if ckpt.get("m"):
            self.load_momentum_buffer(ckpt["m"], flat=m)
        if ckpt.get("v"):
            self.load_momentum_buffer(ckpt["v"], flat=v)
        if "t" in ckpt:
            self.t = int(ckpt["t"])

    # ---------------------------------------------------------- forward
    def forward(self, x, y, net, net0, criterion, lrs, Ninflate=1.0, nd=1.0, sgd=None,
                collect=None, clip_grad=None):
        N = self.ND * Ninflate
        lr_body, lr_head = (lrs[0], lrs[0]) if len(lrs) == 1 else (lrs[0], lrs[1])
        st = self.state_for(net, net0)
        m, v = self.adam_buffers(st)
        self.t += 1
        loss, out = self.forward_backward(st, net, x, y, criterion)
        nmode = self.draw_noise(st)
        common = dict(adam_m=m, adam_v=v, beta1=self.beta1, beta2=self.beta2, eps=self.epsilon,
                      t=self.t, momentum_decay=self.momentum_decay, nd=nd,
                      temperature=self.temperature, grad_is_mom=self.grad_is_mom,
                      lrs=(lr_body, lr_head), noise_mode=nmode, sigma2=self.prior_sig ** 2,
                      n_data=N, seed=self.seed, chain=self.chain, step=self.step_count,
                      div_mode=self.div_mode)
        if sgd is None:
            # reference contract: .grad (and v_mom, m, v) only; the caller steps
            K.adam_step(st, L.ADAM_SGHMC_GRAD, **common)
        else:
            ckind, m1, m2, ca, cb = (L.COLLECT_NONE, None, None, 1.0, 1.0) if collect is None \
                else collect
            mom = sgd.momentum != 0
            first = mom and not sgd.has_buffer
            buf = self.ensure_sgd_buffer() if mom else None
            sgd_kw = dict(mu=sgd.momentum, first_step=first, momentum=mom, collect=ckind,
                          mom1=m1, mom2=m2, collect_a=ca, collect_b=cb)
            if clip_grad is not None:
                # adam_csghmc.py:319-322: clip_grad_norm_ on p.grad between
                # Model.forward and optimizer.step
                K.adam_step(st, L.ADAM_SGHMC_GRAD, **common)
                torch.nn.utils.clip_grad_norm_(net.parameters(), clip_grad)
                K.sgmcmc_step(st, L.SGLD, lrs=sgd.lrs(), noise_scale=(0.0, 0.0),
                              noise_mode=L.NOISE_NONE, sigma2=1.0, n_data=1.0, grad_ready=True,
                              mom_buf=buf, seed=self.seed, chain=self.chain,
                              step=self.step_count, div_mode=self.div_mode, **sgd_kw)
            else:
                K.adam_step(st, L.ADAM_SGHMC, **dict(common, lrs=sgd.lrs()), sgd_buf=buf,
                            **sgd_kw)
            if mom:
                sgd.has_buffer = True
        self.step_count += 1
        return self._result(loss, out)
