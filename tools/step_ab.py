"""Same-process A/B of library builds on the fused ViT-L/32 cSGHMC step
(tooling).  One FlatState, then for every build in argv and every launch
geometry, the explore step (theta rw, grad r, mom rw) and the Welford collect
step, HIP-event mean over 20 launches, builds alternating A, B, C, ... for
ROUNDS rounds — so a build's number is never a different allocation's number.

  python tools/step_ab.py LIB [LIB ...]     (ROUNDS=4, GEOMS="1,4,1;2,1,1;1,2,1;1,4,0")
  GRAD=tensor: the gradient read per tensor through the run / base table from
  separate allocations (the Runners' default); GRAD=views: the same table over
  views of the one flat gradient allocation; GRAD=ab: flat and per-tensor
  gradients alternating in the same process (reported as lib name + "/flat"
  and "/tensor").  COLLECT_ALL=1: the collect step at every geometry (default:
  the first only).
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import FlatState  # noqa: E402
from bayesdll_amd.shapes import segments  # noqa: E402

libs = [os.path.abspath(p) for p in sys.argv[1:]]
rounds = int(os.environ.get("ROUNDS", "4"))
geoms = [tuple(int(x) for x in g.split(",")) for g in
         os.environ.get("GEOMS", "1,4,1;2,1,1;1,2,1;1,4,0").split(";")]
dev = torch.device("cuda", 0)


def use(path):
    """Load one build; an older build (the A/B baseline) may lack entry points
    added since, which this tool never calls: they are left unbound."""
    import ctypes
    L._lib = None
    L.LIB_PATH = path
    h = ctypes.CDLL(path)
    saved = dict(L.EXPORTS)
    for name in list(L.EXPORTS):
        if not hasattr(h, name):
            del L.EXPORTS[name]
    try:
        L.lib()
    finally:
        L.EXPORTS.clear()
        L.EXPORTS.update(saved)


METHOD = os.environ.get("METHOD", "csghmc")  # or "adam" (Adam-SGHMC + SGD), "sgld" (+ SGD),
# "sghmc" (+ SGD(0)), "draw" (the Welford posterior draw; GEOMS entries = workgroups/CU, unroll)
use(libs[0])
segs, readout = segments(os.environ.get("BACKBONE", "vit_l_32"), 1000)
adam = METHOD == "adam"
sgld = METHOD == "sgld"
sghmc = METHOD == "sghmc"
st = FlatState.from_segments(segs, readout, device=dev, need_prior=adam or sgld or sghmc,
                             extra=("adam_m", "adam_v", "sgd_buf") if adam else ())
gen = torch.Generator(device=dev).manual_seed(1)
st.theta.normal_(0.0, 0.02, generator=gen)
st.grad.normal_(0.0, 1e-3, generator=gen)
m1 = st.theta.clone()
m2 = torch.zeros_like(st.theta)
n = st.n
GRAD = os.environ.get("GRAD", "flat")
COLLECT_ALL = os.environ.get("COLLECT_ALL", "0") == "1"  # the collect at every geometry
_flat = st.grad
_grads = [st.grad[o:o + k].clone() for o, k in zip(st.offsets, st.numels)] \
    if GRAD in ("tensor", "ab") else None


def grad_mode(mode):
    """Switch the state between the flat gradient and the per-tensor copies."""
    if mode == "tensor":
        st.use_tensor_grads(_grads)
    else:
        st.grad_mode, st.grad, st.gbase, st._untouched = "flat", _flat, None, ()
        st.runs, st.nruns = st._base_runs


if GRAD == "tensor":
    grad_mode("tensor")
elif GRAD == "views":
    st.use_tensor_grads([st.grad[o:o + k] for o, k in zip(st.offsets, st.numels)])
print(json.dumps({"grad": GRAD, "runs": st.nruns}), flush=True)
lrs, alpha, N = (1e-4, 1e-2), 0.18, 1840.0


def explore(i):
    if METHOD == "draw":  # methods/csghmc.py:466-468 (mom1 = mean, mom2 = M2)
        K.posterior_sample(st.mom, m1, m2, var_mode=L.VAR_WELFORD, ratio=1.0 / 7.0, seed=3,
                           step=i, geometry=geoms_now[0][:2])
        return
    if sghmc:  # methods/sghmc.py:482-510 + SGD(momentum 0), Philox
        K.sgmcmc_step(st, L.SGHMC, lrs=lrs, noise_scale=(1e-3, 1e-3), noise_mode=L.NOISE_PHILOX,
                      one_minus_alpha=1 - alpha, sigma2=1.0, n_data=N * 1e3, seed=3, chain=0,
                      step=i)
        return
    if sgld:  # methods/sgld.py:469-484 + SGD(momentum 0.5), Philox
        K.sgmcmc_step(st, L.SGLD, lrs=lrs, noise_scale=(1e-3, 1e-3), noise_mode=L.NOISE_PHILOX,
                      prior_sig=1.0, sigma2=1.0, n_data=N * 1e3, mu=0.5, momentum=True,
                      seed=3, chain=0, step=i)
        return
    if adam:  # methods/adam_sghmc.py:458-553 + SGD(momentum 0.5), Philox
        K.adam_step(st, L.ADAM_SGHMC, adam_m=st.extra["adam_m"], adam_v=st.extra["adam_v"],
                    sgd_buf=st.extra["sgd_buf"], beta1=0.9, beta2=0.999, eps=1e-8, t=i + 2,
                    momentum_decay=alpha, nd=0.01, lrs=lrs, noise_mode=L.NOISE_PHILOX,
                    sigma2=1.0, n_data=N * 1e3, mu=0.5, momentum=True, seed=3, chain=0, step=i)
        return
    K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=(0.0, 0.0), noise_mode=L.NOISE_NONE,
                  one_minus_alpha=1 - alpha, prior_sig=1.0)


def collect(i):
    if sghmc:  # running mean / second moment on the sample steps (sghmc.py:242-245)
        K.sgmcmc_step(st, L.SGHMC, lrs=lrs, noise_scale=(1e-3, 1e-3), noise_mode=L.NOISE_PHILOX,
                      one_minus_alpha=1 - alpha, sigma2=1.0, n_data=N * 1e3,
                      collect=L.COLLECT_MEAN, mom1=m1, mom2=m2, collect_a=float(i + 1),
                      collect_b=float(i + 2), seed=3, chain=0, step=i)
        return
    if sgld:
        K.sgmcmc_step(st, L.SGLD, lrs=lrs, noise_scale=(1e-3, 1e-3), noise_mode=L.NOISE_PHILOX,
                      prior_sig=1.0, sigma2=1.0, n_data=N * 1e3, mu=0.5, momentum=True,
                      collect=L.COLLECT_MEAN, mom1=m1, mom2=m2, collect_a=float(i + 1),
                      collect_b=float(i + 2), seed=3, chain=0, step=i)
        return
    ns = [0.01 * np.sqrt(2 * alpha * x) / N for x in lrs]
    K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                  one_minus_alpha=1 - alpha, prior_sig=1.0, collect=L.COLLECT_WELFORD, mom1=m1,
                  mom2=m2, collect_a=float(i + 3), seed=3, chain=0, step=i)


def init(i):  # the cycle-init Welford collect (csghmc.py:333-337): m1 = theta, m2 = 0
    ns = [0.01 * np.sqrt(2 * alpha * x) / N for x in lrs]
    K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                  one_minus_alpha=1 - alpha, prior_sig=1.0, collect=L.COLLECT_WELFORD_INIT,
                  mom1=m1, mom2=m2, collect_a=1.0, seed=3, chain=0, step=i)


INIT = os.environ.get("INIT", "0") == "1" and METHOD == "csghmc"  # also time the init collect


def t(fn, reps=20):
    for i in range(3):
        fn(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res, geoms_now = {}, []
m2.normal_(0.0, 1e-2, generator=gen).square_()
for r in range(rounds):
    for path, gm in [(p, m) for p in libs for m in (("flat", "tensor") if GRAD == "ab" else (None,))]:
        use(path)
        if gm is not None:
            grad_mode(gm)
        tag = os.path.basename(path) + ("" if gm is None else "/" + gm)
        for g in geoms:
            geoms_now[:] = [g]
            K.set_launch_config(*g)
            for name, fn, bpe in ((METHOD if METHOD in ("adam", "sgld", "sghmc", "draw")
                                   else "explore", explore,
                                   {"adam": 48, "sgld": 24, "sghmc": 24, "draw": 12}.get(METHOD, 20)),
                                  ("collect", collect, 40 if sgld or sghmc else 36)) + \
                    ((("init", init, 28),) if INIT else ()):
                if name in ("collect", "init") and (adam or METHOD == "draw" or
                                          (g != geoms[0] and not COLLECT_ALL)):
                    continue
                ms = t(fn)
                res.setdefault((tag, g, name), []).append(ms)
                print(json.dumps({"round": r, "lib": tag, "geom": g,
                                  "kernel": name, "ms": round(ms, 4),
                                  "frac": round(bpe * n / ms / 1e6 / 8000.0, 4)}), flush=True)
for (lib, g, name), v in sorted(res.items(), key=lambda kv: (kv[0][2], np.median(kv[1]))):
    print(json.dumps({"summary": name, "lib": lib, "geom": g, "median_ms": round(float(np.median(v)), 4),
                      "min_ms": round(min(v), 4)}))
