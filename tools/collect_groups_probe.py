"""Placement groups for the Welford collect step (tooling).

Times the (theta, mom) explore step on every pair of NV torch allocations,
clusters them into groups by their pair-time profile (two allocations are in
the same group when their rows of the pair matrix agree), then, with theta
and mom on the fastest cross-group pair, times the cSGHMC Welford collect
step (theta rw, g r, mom rw, m1 rw, m2 rw) for m1 / m2 in every combination
of groups.  One JSON line per timing (median of 5 launches)."""
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from types import SimpleNamespace  # noqa: E402

from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import _time_launch, build_runs  # noqa: E402

n = 306535400
NV = int(os.environ.get("NV", "16"))
dev = torch.device("cuda", 0)
runs = build_runs([0], [n], [L.ATTR_PRIOR], n).to(dev)
K.set_launch_config(1, 4, 1)
g = torch.empty(n, device=dev).normal_(0, 1e-3)
V = [torch.empty(n, device=dev).normal_(0, 0.02).abs_() for _ in range(NV)]


def step(theta, mom, m1=None, m2=None, collect=L.COLLECT_NONE):
    st = SimpleNamespace(theta=theta, grad=g, mom=mom, prior=None, noise=None, runs=runs, nruns=1,
                         n=n, device=dev)
    return lambda: K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-9, 1e-9), noise_scale=(1e-9, 1e-9),
                                 noise_mode=L.NOISE_PHILOX if collect else L.NOISE_NONE,
                                 one_minus_alpha=0.5, prior_sig=0.0, collect=collect, mom1=m1,
                                 mom2=m2, collect_a=3.0, seed=1, chain=0, step=5)


M = np.zeros((NV, NV))
for i, j in itertools.combinations(range(NV), 2):
    M[i, j] = M[j, i] = _time_launch(step(V[i], V[j]), dev)
print(json.dumps({"pairs": np.round(M, 4).tolist()}), flush=True)
# group: same row profile (within 1.5 %) over the other allocations
groups = []
for i in range(NV):
    for gr in groups:
        k = gr[0]
        others = [x for x in range(NV) if x not in (i, k)]
        if np.all(np.abs(M[i, others] - M[k, others]) < 0.015 * M[k, others]) and \
                M[i, k] > 0.97 * M.max():
            gr.append(i)
            break
    else:
        groups.append([i])
print(json.dumps({"groups": groups}), flush=True)
# theta / mom: the fastest pair
i0, j0 = np.unravel_index(np.argmin(np.where(M > 0, M, np.inf)), M.shape)
used = {int(i0), int(j0)}
gid = {x: q for q, gr in enumerate(groups) for x in gr}
print(json.dumps({"theta": int(i0), "mom": int(j0), "pair_ms": round(float(M[i0, j0]), 4),
                  "theta_group": gid[int(i0)], "mom_group": gid[int(j0)]}), flush=True)
for rep in range(2):
    for ga, gb in itertools.product(range(len(groups)), repeat=2):
        pa = [x for x in groups[ga] if x not in used]
        pb = [x for x in groups[gb] if x not in used and (ga != gb or x != (pa[0] if pa else -1))]
        if not pa or not pb:
            continue
        a, b = pa[0], pb[0]
        if a == b:
            continue
        t = _time_launch(step(V[i0], V[j0], V[a], V[b], L.COLLECT_WELFORD), dev)
        print(json.dumps({"kernel": "collect_welford", "m1_group": ga, "m2_group": gb,
                          "m1": a, "m2": b, "ms": round(t, 4)}), flush=True)
