"""Python-side calls into the fused HIP kernels (libbdl_sgmcmc.so).

Every scalar is handed over as the float64 value the reference computes on
the host; ctypes rounds it to fp32 (round-to-nearest), which is exactly the
cast torch applies to a Python/NumPy scalar at an fp32 op.  Launches go on
torch's current HIP stream, so ordering with autograd is implicit and no host
synchronisation happens here.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib as L

# Scalar-division rounding: "recip" = x * fl(1/s), what torch's HIP kernels do
# for a tensor / Python-scalar division (so a chain is bit-compatible with the
# reference sampler running on the same GPU) and ~22 % faster for the SGLD /
# SGHMC sweeps than a correctly rounded divide; "true" = x / s, torch CPU's
# rounding (the golden fixtures were generated on a CPU).
DIV_MODE = os.environ.get("BDL_DIV_MODE", "recip")


def _div_flag(div_mode=None):
    return L.FLAG_RECIP_DIV if (div_mode or DIV_MODE) == "recip" else 0


def _inv(s):
    """fl32(1/s) of the float64 divisor s: torch on a HIP device forms the
    reciprocal of a Python-scalar divisor in double and multiplies by it
    (tools/div_probe.py); ctypes does the final fp32 rounding."""
    s = float(s)
    return 1.0 / s if s != 0.0 else 0.0


def _step_args(state, method, *, lrs, noise_scale, noise_mode, one_minus_alpha=1.0,
               prior_sig=0.0, sigma2=1.0, n_data=1.0, mu=0.0, first_step=False,
               momentum=False, collect=L.COLLECT_NONE, mom1=None, mom2=None, collect_a=1.0,
               collect_b=1.0, seed=0, chain=0, step=0, div_mode=None, noise=None, grad_ready=False,
               mom_buf=None, philox_offset=0):
    a = L.StepArgs()
    a.theta = state.theta.data_ptr()
    g = getattr(state, "grad", None)
    a.grad = None if g is None else g.data_ptr()
    gb = getattr(state, "gbase", None)  # per-tensor gradients ("tensor" grad mode)
    a.grad_base = None if gb is None else gb.data_ptr()
    nf = getattr(state, "nonfinite", None)  # divergence flag (FlatState.nonfinite)
    a.nonfinite = None if nf is None else nf.data_ptr()
    mb = state.mom if mom_buf is None else mom_buf  # mom_buf: a separate SGD buffer
    a.mom = None if mb is None else mb.data_ptr()
    a.prior_mean = None if state.prior is None else state.prior.data_ptr()
    nz = noise if noise is not None else state.noise
    a.noise = None if nz is None else nz.data_ptr()
    a.mom1 = None if mom1 is None else mom1.data_ptr()
    a.mom2 = None if mom2 is None else mom2.data_ptr()
    a.runs = state.runs.data_ptr()
    a.nruns = state.nruns
    a.method = int(method)
    a.noise_mode = int(noise_mode)
    a.collect = int(collect)
    a.flags = ((L.FLAG_FIRST_STEP if first_step else 0) | (L.FLAG_MOMENTUM if momentum else 0)
               | (L.FLAG_GRAD_READY if grad_ready else 0) | _div_flag(div_mode))
    a.n = state.n
    a.lr[0], a.lr[1] = float(lrs[0]), float(lrs[1])
    a.noise_scale[0], a.noise_scale[1] = float(noise_scale[0]), float(noise_scale[1])
    a.one_minus_alpha = float(one_minus_alpha)
    a.prior_sig = float(prior_sig)
    a.sigma2 = float(sigma2)
    a.n_data = float(n_data)
    a.mu = float(mu)
    a.collect_a = float(collect_a)
    a.collect_b = float(collect_b)
    a.inv_sigma2, a.inv_n_data = _inv(sigma2), _inv(n_data)
    a.inv_collect_a, a.inv_collect_b = _inv(collect_a), _inv(collect_b)
    a.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    a.chain = int(chain) & 0xFFFFFFFFFFFFFFFF
    a.step = int(step) & 0xFFFFFFFFFFFFFFFF
    a.philox_offset = int(philox_offset)
    a.chain_groups = int(getattr(state, "chain_groups", 0))  # stacked chains (StackedState)
    return a


def alg_bytes_per_elem(a, adam=None):
    """Algorithmic HBM bytes per element of one step launch: 4 B
    per vector read, 4 B per vector written, from the launch's own arguments."""
    grad_only = a.method in (L.SGHMC_GRAD, L.SGLD_GRAD, L.ADAM_SGHMC_GRAD)
    b = 4 + (0 if grad_only else 4)                      # theta r (+w)
    b += 4 + (4 if grad_only else 0)                     # grad r (+w)
    if a.method in (L.CSGHMC, L.SGHMC, L.SGHMC_GRAD, L.ADAM_SGHMC, L.ADAM_SGHMC_GRAD):
        b += 8                                           # momentum v r+w
    elif a.method == L.SGLD and a.flags & L.FLAG_MOMENTUM:
        b += 4 if a.flags & L.FLAG_FIRST_STEP else 8     # SGD buffer (w | r+w)
    if a.method != L.CSGHMC and a.prior_mean:
        b += 4                                           # theta0 r
    if a.noise_mode == L.NOISE_BUFFER:
        b += 4
    if adam is not None:
        b += 16                                          # Adam m, v r+w
        if adam.sgd_buf:
            b += 4 if a.flags & L.FLAG_FIRST_STEP else 8
    nmom = 2 if a.mom2 else 1
    if a.collect in (L.COLLECT_WELFORD, L.COLLECT_MEAN):
        b += 8 * nmom
    elif a.collect in (L.COLLECT_WELFORD_INIT, L.COLLECT_MEAN_INIT):
        b += 4 * nmom
    return b


class StepTimer:
    """Sampled HIP-event timing of the fused update launches (BDL_STEP_TIMING=k:
    every k-th launch), on the launch stream; summary() once per epoch gives
    launches, mean ms and algorithmic GB/s (expose step counters
    and GB/s).  Off by default; never synchronises per step."""

    def __init__(self, every):
        self.every, self.count, self.recs = max(1, int(every)), 0, []

    def begin(self):
        self.count += 1
        if (self.count - 1) % self.every:
            return None
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        return e0

    def end(self, e0, nbytes):
        if e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.recs.append((e0, e1, nbytes))

    def summary(self, reset=True):
        if not self.recs:
            return {"launches": self.count, "timed": 0}
        self.recs[-1][1].synchronize()
        ms = [a.elapsed_time(b) for a, b, _ in self.recs]
        gbs = [nb / (t * 1e-3) / 1e9 for t, (_, _, nb) in zip(ms, self.recs)]
        out = {"launches": self.count, "timed": len(ms), "avg_ms": sum(ms) / len(ms),
               "gbs": sum(gbs) / len(gbs)}
        if reset:
            self.count, self.recs = 0, []
        return out


def launch_kind(collect):
    """The geometry kind of a launch: "collect" for the steady-state moment
    updates (m1 / m2 read and written), "init" for a cycle's first collect
    (m1 / m2 only written), "step" otherwise; each is tuned on its own."""
    if collect in (L.COLLECT_WELFORD, L.COLLECT_MEAN):
        return "collect"
    if collect in (L.COLLECT_WELFORD_INIT, L.COLLECT_MEAN_INIT):
        return "init"
    return "step"


def _launch(state, fn, a, adam=None, written=None):
    kind = launch_kind(a.collect)
    pend = getattr(state, "_tune_pending", None)
    # a first step (SGD buffer written, not read) is not the steady-state
    # access mix: the kind stays pending until a later launch
    if pend and written is not None and int(a.n) == int(state.n) and kind in pend and \
            not (a.flags & L.FLAG_FIRST_STEP) and \
            not torch.cuda.is_current_stream_capturing():
        _tune_kind(state, fn, kind, written)
    _use_geometry(state, kind)
    t = getattr(state, "timer", None)
    e0 = t.begin() if t is not None else None
    fn()
    if e0 is not None:
        t.end(e0, alg_bytes_per_elem(a, adam) * int(a.n))


def _written(state, method, *, grad_only, mom, extra=(), mom1=None, mom2=None):
    """The vectors a full step launch writes (saved and restored while it is
    tuned on the state's own buffers), or None when they are not all flat
    vectors of the state (per-tensor gradients written by a *_GRAD method)."""
    if grad_only:
        if getattr(state, "grad", None) is None:
            return None
        out = [state.grad]
    else:
        out = [state.theta]
    out += [t for t in (mom,) + tuple(extra) + (mom1, mom2) if t is not None]
    return out


def sgmcmc_step(state, method, **kw):
    """One fused update over `state` (a FlatState). Asynchronous."""
    a = _step_args(state, method, **kw)
    mb = kw.get("mom_buf")
    wr = _written(state, method, grad_only=method in (L.SGHMC_GRAD, L.SGLD_GRAD),
                  mom=state.mom if mb is None else mb,
                  mom1=kw.get("mom1") if kw.get("collect", L.COLLECT_NONE) else None,
                  mom2=kw.get("mom2") if kw.get("collect", L.COLLECT_NONE) else None)
    _launch(state, lambda: L.check(L.lib().bdl_sgmcmc_step(a, L.current_stream_handle(state.device)),
                                   "bdl_sgmcmc_step"), a, written=wr)


def sgmcmc_step_bare(state, **kw):
    """The cSGHMC step of these arguments with its arithmetic removed
    (bdl_sgmcmc_step_bare, include/bdl_measure.h): measurement only — the
    production kernel's own loop, loads and stores, at the launch
    configuration currently installed (set_launch_config; no tuning, no
    geometry switch).  theta / mom / steady-state moments keep their values.
    Asynchronous."""
    a = _step_args(state, L.CSGHMC, **kw)
    L.check(L.lib().bdl_sgmcmc_step_bare(a, L.current_stream_handle(state.device)),
            "bdl_sgmcmc_step_bare")


def adam_step(state, method, *, adam_m, adam_v, sgd_buf=None, beta1, beta2, eps, t,
              momentum_decay, nd, temperature=1.0, grad_is_mom=False, lrs, noise_mode,
              sigma2, n_data, mu=0.0, first_step=False, momentum=False, collect=L.COLLECT_NONE,
              mom1=None, mom2=None, collect_a=1.0, collect_b=1.0, seed=0, chain=0, step=0,
              div_mode=None, noise=None, philox_offset=0):
    """One fused Adam-preconditioned SGHMC step (methods/adam_sghmc.py:500-553,
    adam_csghmc.py:812-860) + SGD step.  The host-side scalars are formed in
    float64 exactly as the reference's Python does (1 - beta1, 1 - beta1**t,
    2 * momentum_decay, 1 - momentum_decay); ctypes rounds them to fp32."""
    a = _step_args(state, method, lrs=lrs, noise_scale=(0.0, 0.0), noise_mode=noise_mode,
                   one_minus_alpha=1 - momentum_decay, sigma2=sigma2, n_data=n_data, mu=mu,
                   first_step=first_step, momentum=momentum, collect=collect, mom1=mom1,
                   mom2=mom2, collect_a=collect_a, collect_b=collect_b, seed=seed, chain=chain,
                   step=step, div_mode=div_mode, noise=noise, philox_offset=philox_offset)
    ad = L.AdamArgs()
    ad.adam_m = adam_m.data_ptr()
    ad.adam_v = adam_v.data_ptr()
    ad.sgd_buf = None if sgd_buf is None else sgd_buf.data_ptr()
    ad.beta1, ad.one_minus_beta1 = float(beta1), 1 - float(beta1)
    ad.beta2, ad.one_minus_beta2 = float(beta2), 1 - float(beta2)
    bc1, bc2 = 1 - float(beta1) ** int(t), 1 - float(beta2) ** int(t)
    ad.bias_corr1, ad.bias_corr2 = bc1, bc2
    ad.eps = float(eps)
    ad.two_alpha = 2 * float(momentum_decay)
    ad.nd = float(nd)
    ad.temperature = float(temperature)
    ad.inv_bias_corr1, ad.inv_bias_corr2 = _inv(bc1), _inv(bc2)
    ad.inv_temperature = _inv(temperature)
    ad.grad_is_mom = 1 if grad_is_mom else 0
    wr = _written(state, method, grad_only=method == L.ADAM_SGHMC_GRAD, mom=state.mom,
                  extra=(adam_m, adam_v) + ((sgd_buf,) if sgd_buf is not None else ()),
                  mom1=mom1 if collect != L.COLLECT_NONE else None,
                  mom2=mom2 if collect != L.COLLECT_NONE else None)
    _launch(state, lambda: L.check(L.lib().bdl_adam_step(a, ad, L.current_stream_handle(state.device)),
                                   "bdl_adam_step"), a, ad, written=wr)


def stream_mix(reads, writes, blocks_per_cu=1, unroll=4, schedule=L.MIX_BARE):
    """The bare access mix of a sweep over these buffers in one issue schedule
    (bdl_stream_mix_schedule, include/bdl_measure.h: L.MIX_BARE, MIX_PIPELINED,
    MIX_PACED): measurement only — the written tensors' contents are
    destroyed.  Asynchronous, on the current stream."""
    n = reads[0].numel()
    dev = reads[0].device
    rp = (C.c_void_p * len(reads))(*[t.data_ptr() for t in reads])
    wp = (C.c_void_p * len(writes))(*[t.data_ptr() for t in writes])
    L.check(L.lib().bdl_stream_mix_schedule(rp, len(reads), wp, len(writes), int(n),
                                            int(blocks_per_cu), int(unroll), int(schedule),
                                            L.current_stream_handle(dev)), "bdl_stream_mix")


def clip_workspace(state):
    """Device scratch for sgld_step_clipped: (total_norm, coef) then per-workgroup
    partial sums.  Cached on the FlatState."""
    ws = getattr(state, "_clip_ws", None)
    if ws is None:
        nbytes = int(L.lib().bdl_clip_workspace_bytes(int(state.n)))
        ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=state.device)
        state._clip_ws = ws
    return ws


def sgld_step_clipped(state, max_norm, **kw):
    """SGLD step with torch.nn.utils.clip_grad_norm_(max_norm) applied to the
    sampler gradient first (methods/csgld.py:250-253), all on device: a norm
    pass, a one-workgroup finalize and the update pass.  Returns the workspace
    whose first two floats are (total_norm, clip_coef)."""
    a = _step_args(state, L.SGLD, **kw)
    _use_geometry(state)
    ws = clip_workspace(state)
    L.check(L.lib().bdl_sgld_step_clipped(a, float(max_norm), ws.data_ptr(),
                                          L.current_stream_handle(state.device)),
            "bdl_sgld_step_clipped")
    return ws


def moments_update(theta, mom1, mom2, collect, collect_a=1.0, collect_b=1.0, div_mode=None):
    """Stand-alone posterior-moment update of flat vectors (no parameter update)."""
    L.require_hip(theta, "theta")
    a = L.MomentsArgs()
    a.theta, a.mom1 = theta.data_ptr(), mom1.data_ptr()
    a.mom2 = None if mom2 is None else mom2.data_ptr()
    a.n = theta.numel()
    a.collect = int(collect)
    a.flags = _div_flag(div_mode)
    a.collect_a, a.collect_b = float(collect_a), float(collect_b)
    a.inv_collect_a, a.inv_collect_b = _inv(collect_a), _inv(collect_b)
    L.check(L.lib().bdl_moments_update(a, L.current_stream_handle(theta.device)),
            "bdl_moments_update")


# (workgroups per CU, float4 groups per lane) tried for a vector's draw
SAMPLE_GEOMETRIES = ((1, 4), (2, 4), (3, 4), (4, 4), (4, 1), (6, 1))
SAMPLE_TUNE_MIN = 1 << 22          # smaller draws keep the default (2 x 4)
_SAMPLE_GEOM = {}                  # (device index, n) -> (workgroups per CU, unroll)


def sample_geometry(n, device):
    """The posterior draw's tuned (workgroups per CU, unroll) for an n-element
    vector on `device` (None until posterior_sample tuned it)."""
    return _SAMPLE_GEOM.get((torch.device(device).index, int(n)))


def _tune_sample(a, out):
    """Time the draw at each SAMPLE_GEOMETRIES entry with its own arguments
    (each launch writes the same values: same keys), keep the fastest.  Why:
    the bare access mix of the draw's buffers ranked 3 workgroups/CU x 4
    first at ViT-L/32 size and 4 x 1 at ResNet-101 size on one box (bench.py
    aux_kernels.posterior_sample.mix_ceiling, profiles/round4/methods/), and
    round 2's probes ranked 2 x 4 first on two others; in round 4's
    same-process A/Bs on ViT-L/32 draws 1 x 4 ran 0.587-0.600 ms against
    0.635-0.653 for the best of the others on three boxes
    (profiles/round4/philox_ab/)."""
    stream = L.current_stream_handle(out.device)
    ts = torch.cuda.current_stream(out.device)  # the stream the draws are launched on
    best = None
    for bpc, u in SAMPLE_GEOMETRIES:
        a.blocks_per_cu, a.unroll = bpc, u
        L.check(L.lib().bdl_posterior_sample(a, stream), "bdl_posterior_sample")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(ts)
        for _ in range(3):
            L.check(L.lib().bdl_posterior_sample(a, stream), "bdl_posterior_sample")
        ev[1].record(ts)
        ev[1].synchronize()
        ms = ev[0].elapsed_time(ev[1])
        if best is None or ms < best[0]:
            best = (ms, (bpc, u))
    return best[1]


def posterior_sample(out, mom1, mom2, *, var_mode, ratio=1.0, var_floor=1e-12, noise=None,
                     seed=0, chain=0, step=0, div_mode=None, chain_groups=0, geometry=None):
    """out = mom1 + sqrt(clamp(var(mom1, mom2), var_floor)) * eps (eps: buffer or Philox;
    chain_groups > 0: stacked chains keyed chain + k, bdl_sample_args.chain_groups).
    geometry: (workgroups per CU, unroll 1 or 4) of the launch; None = tuned
    once per device and size on the first draw of >= SAMPLE_TUNE_MIN elements
    (outside graph capture), 2 x 4 below.  Values never depend on it."""
    L.require_hip(out, "out")
    a = L.SampleArgs()
    a.out, a.mom1 = out.data_ptr(), mom1.data_ptr()
    a.mom2 = None if mom2 is None else mom2.data_ptr()
    a.noise = None if noise is None else noise.data_ptr()
    a.n = out.numel()
    a.var_mode = int(var_mode)
    a.noise_mode = L.NOISE_BUFFER if noise is not None else L.NOISE_PHILOX
    a.ratio = float(ratio)
    a.var_floor = float(var_floor)
    # WELFORD M2 / (n-1): torch-on-GPU multiplies by the reciprocal
    a.inv_ratio = _inv(ratio) if _div_flag(div_mode) else 0.0
    a.seed, a.chain, a.step = int(seed), int(chain), int(step) & 0xFFFFFFFFFFFFFFFF
    a.chain_groups = int(chain_groups)
    if geometry is None:
        key = (out.device.index, int(a.n))
        geometry = _SAMPLE_GEOM.get(key)
        if geometry is None and a.n >= SAMPLE_TUNE_MIN and \
                not torch.cuda.is_current_stream_capturing():
            geometry = _SAMPLE_GEOM[key] = _tune_sample(a, out)
    a.blocks_per_cu, a.unroll = (int(x) for x in (geometry or (0, 0)))
    L.check(L.lib().bdl_posterior_sample(a, L.current_stream_handle(out.device)),
            "bdl_posterior_sample")


def philox_normal(n, seed, chain, step, device="cuda"):
    """The N(0,1) values the step kernel draws in Philox mode, as a tensor."""
    out = torch.empty(n, dtype=torch.float32, device=device)
    L.check(L.lib().bdl_philox_normal(out.data_ptr(), int(n), int(seed), int(chain), int(step),
                                      L.current_stream_handle(out.device)), "bdl_philox_normal")
    return out


_ACTIVE = [None]  # the geometry last installed through set_launch_config (None: defaults)
LIBRARY_DEFAULT = (2, 1, 1)  # what the library launches with before any set_launch_config


def set_launch_config(blocks_per_cu=0, unroll=0, grid_stride=0):
    _ACTIVE[0] = (int(blocks_per_cu), int(unroll), int(grid_stride))
    return L.lib().bdl_set_launch_config(int(blocks_per_cu), int(unroll), int(grid_stride))


def restore_launch_config(packed):
    """Re-install the geometry a set_launch_config call returned (packed as
    (grid_stride << 24) | (blocks_per_cu << 8) | unroll)."""
    return set_launch_config((packed >> 8) & 0xFFFF, packed & 0xFF, (packed >> 24) & 0xFF)


def _use_geometry(state, kind="step"):
    """Install the geometry tuned for this state's size and launch kind
    (state.launch_cfg for plain steps; state.collect_cfg for the steps that
    also read and update the posterior moments, state.init_cfg for a cycle's
    first collect, when tuned; else the plain step's) if another is active:
    the library's launch configuration is process-wide, and a process may hold
    states of very different sizes (e.g. a one-chain sampler and a stacked
    one)."""
    cfg = getattr(state, {"collect": "collect_cfg", "init": "init_cfg"}.get(kind, "launch_cfg"),
                  None)
    if cfg is None:
        cfg = getattr(state, "launch_cfg", None)
    if cfg is not None and cfg != _ACTIVE[0]:
        set_launch_config(*cfg)


# Launch geometries worth trying on gfx950 (workgroups/CU, float4 groups in
# flight per lane, grid-stride): the sweep (profiles/round1/kernel_v1) shows the optimum
# moving between these from one device to the next.  The production kernels
# of every method (cSGHMC; SGLD / SGHMC / Adam with noise) exist at unroll
# depths 1, 2 and 4.
AUTOTUNE_CANDIDATES = ((2, 1, 1), (1, 4, 1), (3, 1, 1), (2, 4, 1), (1, 2, 1), (2, 2, 1))
# per sampler family, the geometries that won somewhere in the interleaved
# 13-geometry probe on a ViT-L/32 state (tools/geom_methods.py,
# profiles/round3/aux/geom_methods.jsonl): SGLD 3 x 4 by 0.5 % over 2 x 4;
# Adam-SGHMC 1 x 1 by 1.5 % and 4 x 4 by 0.3 % over 2 x 4 (seven streams: fewer
# accesses in flight per CU pay); cSGHMC 1 x 4 by >= 1.9 % over every other
AUTOTUNE_BY_METHOD = {
    # + 1 x 1 and 3 x 4: the bare access mix of the SGLD buffers ran 1 x 1 8 %
    # ahead of the tuned 2 x 1 at ResNet-101 size, and of the explore buffers
    # 3 x 4 first at ViT-L/32 size (bench.py mix_ceiling, profiles/round4/methods/)
    # + 1 x 1: the bare mix of the explore buffers ran fastest there on the
    # round-5 box (1.038 ms vs 1.064 for the kernel's tuned 1 x 4)
    "csghmc": AUTOTUNE_CANDIDATES + ((3, 4, 1), (1, 1, 1)),
    "sgld": AUTOTUNE_CANDIDATES + ((3, 4, 1), (4, 4, 1), (1, 1, 1)),
    "adam": AUTOTUNE_CANDIDATES + ((1, 1, 1), (4, 4, 1)),
}
_TUNED = {}
_TUNED_COLLECT = {}
# the collect steps (the step plus the posterior-moment update: cSGHMC Welford
# m1 / M2, SGLD / Adam running m1 / m2 — four to six more streams) are tuned
# separately over the method's candidates plus 1 x 1: the cSGHMC Welford
# collect ran 1.778 ms at 1 x 1 vs 1.800 at the explore's 1 x 4 and >= 1.83 at
# every other geometry (tools/geom_methods.py METHODS=collect,
# profiles/round3/aux/geom_collect.jsonl; round 1's sweep: 1 x 1 best too)
COLLECT_EXTRA = ((1, 1, 1),)


ADAM_EXTRA = ("adam_m", "adam_v", "sgd_buf")  # adam_sghmc.Model.extra_vectors


def _scratch_launcher(n, dev, method):
    """A closure launching `method`'s production kernel over scratch buffers of
    n elements (the buffers live as long as the closure)."""
    return _scratch_launchers(n, dev, method)[0]


def _scratch_launchers(n, dev, method):
    """Closures launching `method`'s production kernel over scratch buffers of
    n elements — (plain step, collect step: the same with the posterior-moment
    update; its m1 / m2 are allocated at its first call, for cSGHMC as the
    Runner allocates a cycle's Welford pair) — the buffers live as long as the
    closures."""
    from .flat import FlatState, moment_pair
    st = FlatState.from_segments([("w", (int(n),))], None, device=dev,
                                 need_prior=method != "csghmc",
                                 extra=ADAM_EXTRA if method == "adam" else ())
    st.theta.zero_()
    if method == "csghmc":
        kw = dict(lrs=(1e-4, 1e-4), noise_scale=(0.0, 0.0), noise_mode=L.NOISE_NONE,
                  one_minus_alpha=0.9, prior_sig=1.0)

        def launch():
            sgmcmc_step(st, L.CSGHMC, **kw)
    elif method == "sgld":
        st.prior.zero_()
        kw = dict(lrs=(1e-4, 1e-4), noise_scale=(1e-3, 1e-3), noise_mode=L.NOISE_PHILOX,
                  sigma2=1.0, n_data=1e6, mu=0.5, momentum=True)

        def launch():
            sgmcmc_step(st, L.SGLD, **kw)
    elif method == "adam":
        st.prior.zero_()
        m, v, buf = (st.extra[k] for k in ADAM_EXTRA)
        kw = dict(adam_m=m, adam_v=v, sgd_buf=buf, beta1=0.9, beta2=0.999, eps=1e-8, t=3,
                  momentum_decay=0.1, nd=0.01, lrs=(1e-4, 1e-4), noise_mode=L.NOISE_PHILOX,
                  sigma2=1.0, n_data=1e6, mu=0.5, momentum=True)

        def launch():
            adam_step(st, L.ADAM_SGHMC, **kw)
    else:
        raise ValueError(f"unknown method {method!r}")
    moms = []

    def launch_collect():
        if not moms:
            moms.extend(moment_pair(int(n), dev) if method == "csghmc" else
                        (torch.zeros_like(st.theta), torch.zeros_like(st.theta)))
            moms[0].copy_(st.theta)
            moms[1].zero_()
        if method == "csghmc":
            sgmcmc_step(st, L.CSGHMC, lrs=(1e-4, 1e-4), noise_scale=(1e-7, 1e-7),
                        noise_mode=L.NOISE_PHILOX, one_minus_alpha=0.9, prior_sig=1.0,
                        collect=L.COLLECT_WELFORD, mom1=moms[0], mom2=moms[1], collect_a=3.0)
        elif method == "sgld":
            sgmcmc_step(st, L.SGLD, collect=L.COLLECT_MEAN, mom1=moms[0], mom2=moms[1],
                        collect_a=2.0, collect_b=3.0, **kw)
        else:
            adam_step(st, L.ADAM_SGHMC, collect=L.COLLECT_MEAN, mom1=moms[0], mom2=moms[1],
                      collect_a=2.0, collect_b=3.0, **kw)
    return launch, launch_collect


def _device(device):
    return torch.device(device) if device is not None else torch.device(
        "cuda", torch.cuda.current_device())


def autotune(n, device=None, reps=6, candidates=None, method="csghmc", collect=False):
    """Pick the fastest launch geometry for an n-element sweep on this device.

    The update of every element is independent of the launch geometry (noise
    is keyed by element index), so the choice changes speed only, never
    results.  Times the method's production kernel (cSGHMC exploration; SGLD
    + SGD momentum with Philox noise; Adam-SGHMC + SGD momentum) on scratch
    buffers (freed afterwards) and installs the winner process-wide.  Returns
    (config, {config: ms}); with collect=True, (config, {config: ms},
    collect config, {config: ms}) — the collect step tuned on the same
    scratch state over the candidates plus COLLECT_EXTRA (not installed)."""
    import numpy as np
    dev = _device(device)
    if candidates is None:
        candidates = AUTOTUNE_BY_METHOD.get(method, AUTOTUNE_CANDIDATES)
    launch, launch_collect = _scratch_launchers(n, dev, method)

    def pick(fn, cands):
        # round 1: every candidate; round 2: the three fastest again with twice
        # the repetitions, averaged with round 1 (damps the +-1-2 % burst-to-burst noise)
        times = measure(fn, cands, reps)
        top = sorted(times, key=times.get)[:3]
        again = measure(fn, top, 2 * reps)
        for cfg in top:
            times[cfg] = 0.5 * (times[cfg] + again[cfg])
        return min(top, key=times.get), times

    def measure(fn, cfgs, k):
        out = {}
        for cfg in cfgs:
            set_launch_config(*cfg)
            for _ in range(2):
                fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(k)]
            for e0, e1 in ev:
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize(dev)
            out[cfg] = float(np.median([a.elapsed_time(b) for a, b in ev]))
        return out

    best, times = pick(launch, candidates)
    res = (best, times)
    if collect:
        cbest, ctimes = pick(launch_collect, tuple(candidates) + tuple(
            c for c in COLLECT_EXTRA if c not in candidates))
        res = (best, times, cbest, ctimes)
    set_launch_config(*best)
    del launch, launch_collect
    torch.cuda.empty_cache()
    return res


TUNE_ON_STATE_MIN = 1 << 16  # smaller states keep the default geometry
TUNE_SNAPSHOT_FRACTION = 0.25  # the tuning's snapshot of the written vectors, at most this share of free HBM


def request_state_tuning(state, method):
    """Tune `state`'s launch geometry on its OWN buffers at the first full
    launch of each kind (the plain step; the collect step), with that launch's
    own arguments, restoring every vector it writes after each candidate (so
    the chain is unchanged; the update never depends on geometry anyway).
    Why not scratch vectors (autotune): which geometry is fastest depends on
    where the vectors sit in HBM — on one box the SGLD sweep over ResNet-101
    ran 2 x 4 fastest on scratch vectors while the bare access mix of the
    chain's own buffers ran 1 x 1 8 % ahead of it, and the Adam sweep's best
    moved from 2 x 4 to 1 x 4 (bench.py mix_ceiling, profiles/round4/methods_b/).
    BDL_AUTOTUNE=0: the defaults."""
    if os.environ.get("BDL_AUTOTUNE", "1") == "0" or int(state.n) < TUNE_ON_STATE_MIN:
        return
    state._tune_pending = {"step", "collect", "init"}
    state._tune_method = method
    state.tuned = {}


def _tune_kind(state, fn, kind, written):
    state._tune_pending.discard(kind)
    cands = tuple(AUTOTUNE_BY_METHOD.get(state._tune_method, AUTOTUNE_CANDIDATES))
    if kind != "step":
        cands += tuple(c for c in COLLECT_EXTRA if c not in cands)
    nf = getattr(state, "nonfinite", None)
    written = list(written) + ([nf] if nf is not None else [])
    # the snapshot of what the launch writes must fit comfortably: otherwise
    # keep the current geometry (a model this large is tuned on nothing)
    need = sum(w.numel() * w.element_size() for w in written)
    free, _ = torch.cuda.mem_get_info(state.device)
    if need > TUNE_SNAPSHOT_FRACTION * free:
        state.tuned[kind] = {"skipped": f"snapshot {need >> 20} MiB > "
                                        f"{TUNE_SNAPSHOT_FRACTION:g} x free {free >> 20} MiB"}
        return
    best, times = tune_on_state(fn, written, cands, state.device)
    setattr(state, {"collect": "collect_cfg", "init": "init_cfg"}.get(kind, "launch_cfg"), best)
    state.tuned[kind] = {"best": best, "ms": {f"{c[0]}wg/cu x{c[1]}": round(t, 4)
                                              for c, t in times.items()}}


def tune_on_state(launch, written, candidates, device, reps=4):
    """Time `launch` (a zero-argument launch over a state's own buffers) at
    each candidate geometry — round 1 every candidate, round 2 the three
    fastest again with twice the repetitions, averaged — restoring the
    `written` tensors after every candidate.  Returns (best, {cfg: ms}); the
    previous geometry is re-installed."""
    import numpy as np
    saved = [w.clone() for w in written]
    prev = _ACTIVE[0]
    ts = torch.cuda.current_stream(device)  # the stream `launch` enqueues on

    def measure(cfgs, k):
        out = {}
        for cfg in cfgs:
            set_launch_config(*cfg)
            launch()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(k)]
            for e0, e1 in ev:
                e0.record(ts)
                launch()
                e1.record(ts)
            torch.cuda.synchronize(device)
            out[cfg] = float(np.median([x.elapsed_time(y) for x, y in ev]))
            for w, s in zip(written, saved):
                w.copy_(s)
        return out

    try:
        times = measure(candidates, reps)
        top = sorted(times, key=times.get)[:3]
        again = measure(top, 2 * reps)
        for cfg in top:
            times[cfg] = 0.5 * (times[cfg] + again[cfg])
        best = min(top, key=times.get)
    finally:
        for w, s in zip(written, saved):
            w.copy_(s)
        del saved
        if prev is not None:
            set_launch_config(*prev)
    return best, times


def prewarm(n, device=None, method="csghmc", seconds=2.5):
    """Run the method's kernel back to back on scratch buffers for `seconds`
    (untimed setup before a measurement): the GPU's clocks ramp over the first
    ~0.8 s of sustained load (tools/drift.py, round 5: 1.058 ms per ViT-L/32
    explore sweep in the first 0.25 s, 1.032-1.035 from ~0.8 s on), so a
    short measurement from idle would read the ramp, not the steady state.
    Returns the number of launches."""
    import time
    dev = _device(device)
    launch = _scratch_launcher(n, dev, method)
    t_end, k = time.perf_counter() + float(seconds), 0
    while time.perf_counter() < t_end:
        for _ in range(20):
            launch()
        k += 20
        torch.cuda.synchronize(dev)
    del launch
    torch.cuda.empty_cache()
    return k


def autotune_once(n, device, method):
    """autotune() (plain and collect steps) once per (n, device, method) in this
    process; later calls only re-install the cached winner.  Returns the plain
    step's geometry (collect_config: the collect step's).  BDL_AUTOTUNE=0
    keeps the defaults."""
    if os.environ.get("BDL_AUTOTUNE", "1") == "0":
        return None
    key = (int(n), str(device), method)
    if key not in _TUNED:
        best, _, cbest, _ = autotune(n, device, method=method, collect=True)
        _TUNED[key], _TUNED_COLLECT[key] = best, cbest
    else:
        set_launch_config(*_TUNED[key])
    return _TUNED[key]


def collect_config(n, device, method):
    """The collect step's geometry autotune_once found for (n, device, method),
    or None (not tuned: the plain step's geometry is used)."""
    return _TUNED_COLLECT.get((int(n), str(device), method))
