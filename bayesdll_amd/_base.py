"""Shared machinery of the drop-in sampler Models.

Each method module (csghmc, sghmc, csgld, sgld) keeps the reference's
`Model(nn.Module).forward(x, y, net, net0, criterion, lrs, Ninflate, nd, ...)`
signature and return value `(loss.item(), out.detach())`.  What changes is
what happens after `loss.backward()`: instead of the per-tensor Python loop,
one fused HIP kernel updates the chain's flat state.

Noise modes (`Model.noise_mode`, or env BDL_NOISE_MODE):
  "philox"   — N(0,1) generated inside the kernel by Philox4x32-10 keyed by
               (seed, chain, step, element): no noise buffer, no extra HBM
               traffic (the production mode).
  "torch"    — per-tensor `normal_()` draws from torch's generator into a flat
               noise buffer, in named_parameters order, on every step: the
               exact stream the reference's `torch.randn_like(p)` consumes, so
               a chain matches the reference sampler draw-for-draw on the same
               device and seed.
  "external" — `Model.noise_provider(step, flat_noise)` fills the buffer
               (used by the parity tests to replay captured reference noise).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import _lib as L
from .flat import FlatState

NOISE_MODES = ("philox", "torch", "external")


def default_noise_mode():
    m = os.environ.get("BDL_NOISE_MODE", "philox")
    if m not in NOISE_MODES:
        raise ValueError(f"BDL_NOISE_MODE must be one of {NOISE_MODES}, got {m!r}")
    return m


def default_chain():
    """Chain id = process rank when torch.distributed is initialised."""
    from . import chains
    return chains.rank()


class FusedModelBase(nn.Module):
    """Holds the chain's FlatState and the noise configuration."""

    need_prior = False
    need_mom = True
    tune_method = "sgld"  # which production kernel autotune_once times for this sampler
    extra_vectors = ()    # further per-element state placed with the chain (FlatState.extra)

    def __init__(self):
        super().__init__()
        self.noise_mode = default_noise_mode()
        self.noise_provider = None
        self.seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFFFFFF
        self.chain = default_chain()
        self.step_count = 0
        self.div_mode = None
        self._state = None
        self._state_net = None

    # -------------------------------------------------------------- state
    def state_for(self, net, net0=None):
        if self._state is None or self._state_net is not net:
            if self.noise_mode not in NOISE_MODES:
                raise ValueError(f"noise_mode must be one of {NOISE_MODES}")
            self._state = FlatState(net, net0, readout_name=getattr(net, "readout_name", None),
                                    bias=getattr(self, "bias", "informative"),
                                    need_prior=self.need_prior, need_mom=self.need_mom,
                                    need_noise=self.noise_mode != "philox",
                                    placement=self.tune_method, extra=self.extra_vectors)
            self._state_net = net
            # launch geometry for this device and size (speed only: results
            # never depend on it)
            from . import kernels as K
            K.autotune_once(self._state.n, self._state.device, self.tune_method)
        return self._state

    @property
    def flat(self):
        return self._state

    # ----------------------------------------------------------- fwd/bwd
    def forward_backward(self, st, net, x, y, criterion):
        out = net(x)
        loss = criterion(out, y)
        st.zero_grad()          # in place of net.zero_grad(): .grad stays a flat view
        loss.backward()
        st.sync_grads()
        return loss, out

    # -------------------------------------------------------------- noise
    def draw_noise(self, st):
        """Advance the noise source for this step; return the kernel noise mode
        to use when the noise term is applied."""
        if self.noise_mode == "philox":
            return L.NOISE_PHILOX
        if self.noise_mode == "torch":
            st.fill_noise_torch()
        else:
            if self.noise_provider is None:
                raise RuntimeError("noise_mode='external' needs Model.noise_provider")
            self.noise_provider(self.step_count, st.noise)
        return L.NOISE_BUFFER

    # ------------------------------------------------------ reference API
    @property
    def momentum_buffer(self):
        """name -> momentum view (the reference's dict, methods/csghmc.py:727-730)."""
        st = self._state
        if st is None or st.mom is None:
            return {}
        return dict(zip(st.names, st.views(st.mom)))

    def load_momentum_buffer(self, d, flat=None):
        """Copy a saved name -> tensor dict into the flat buffer (st.mom, or
        `flat`), in place, so the kernel's pointers stay valid."""
        st = self._state
        if st is None:
            raise RuntimeError("load the checkpoint after the first step has bound the state")
        dst = st.mom if flat is None else flat
        with torch.no_grad():
            for nm, v in zip(st.names, st.views(dst)):
                if nm in d:
                    v.copy_(d[nm].reshape(v.shape))
