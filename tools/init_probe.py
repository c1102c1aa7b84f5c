"""Where does the cSGHMC cycle-init collect (Philox + Welford init: theta rw,
grad r, mom rw, m1 w, m2 w = 28 B/elem) lose to its bare 3-read / 4-write
mix?  One ViT-L/32 state and ONE moment pair; at each geometry, alternating
for ROUNDS rounds: the init step with Philox noise (the product's), the same
step without noise, the Philox sample step without a collect, the explore
step, and the bare mixes 3r/4w and 3r/2w on the same buffers.  HIP-event mean
over REPS launches.

  python tools/init_probe.py        (ROUNDS=3, REPS=10, GEOMS="1,1,1;1,4,1;2,1,1;2,4,1")
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import FlatState, moment_pair  # noqa: E402
from bayesdll_amd.shapes import segments  # noqa: E402

rounds = int(os.environ.get("ROUNDS", "3"))
reps = int(os.environ.get("REPS", "10"))
geoms = [tuple(int(x) for x in g.split(",")) for g in
         os.environ.get("GEOMS", "1,1,1;1,4,1;2,1,1;2,4,1").split(";")]
dev = torch.device("cuda", 0)
segs, ro = segments("vit_l_32")
st = FlatState.from_segments(segs, ro, device=dev)
gen = torch.Generator(device=dev).manual_seed(1)
st.theta.normal_(0.0, 0.02, generator=gen)
st.grad.normal_(0.0, 1e-3, generator=gen)
m1, m2 = moment_pair(st.n, dev)
lrs, alpha, N = (1e-5, 1e-3), 0.18, 1840.0
ns = [0.01 * np.sqrt(2 * alpha * x) / N for x in lrs]
base = dict(lrs=lrs, one_minus_alpha=1 - alpha, prior_sig=1.0, seed=3, chain=0)


def init_philox(i):
    K.sgmcmc_step(st, L.CSGHMC, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                  collect=L.COLLECT_WELFORD_INIT, mom1=m1, mom2=m2, collect_a=1.0, step=i, **base)


def init_none(i):
    K.sgmcmc_step(st, L.CSGHMC, noise_scale=(0.0, 0.0), noise_mode=L.NOISE_NONE,
                  collect=L.COLLECT_WELFORD_INIT, mom1=m1, mom2=m2, collect_a=1.0, step=i, **base)


def sample(i):
    K.sgmcmc_step(st, L.CSGHMC, noise_scale=ns, noise_mode=L.NOISE_PHILOX, step=i, **base)


def explore(i):
    K.sgmcmc_step(st, L.CSGHMC, noise_scale=(0.0, 0.0), noise_mode=L.NOISE_NONE, step=i, **base)


def mix(reads, writes):
    def f(i):
        K.stream_mix(reads, writes, *_geo[0][:2])
    return f


_geo = [None]
cases = [("init_philox", init_philox, 28), ("init_none", init_none, 28),
         ("mix_3r4w", mix([st.theta, st.grad, st.mom], [st.theta, st.mom, m1, m2]), 28),
         ("sample", sample, 20), ("explore", explore, 20),
         ("mix_3r2w", mix([st.theta, st.grad, st.mom], [st.theta, st.mom]), 20)]


def timed(fn):
    for i in range(2):
        fn(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
for r in range(rounds):
    for g in geoms:
        _geo[0] = g
        K.set_launch_config(*g)
        for name, fn, bpe in cases:
            ms = timed(fn)
            res.setdefault((name, g), []).append(ms)
            print(json.dumps({"round": r, "geom": g, "case": name, "ms": round(ms, 4),
                              "frac": round(bpe * st.n / ms / 1e6 / 8000.0, 4)}), flush=True)
for (name, g), v in sorted(res.items()):
    print(json.dumps({"summary": name, "geom": g, "median_ms": round(float(np.median(v)), 4)}))
