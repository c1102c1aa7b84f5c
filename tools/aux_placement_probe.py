"""Do the posterior-sample and moments sweeps have the same placement classes
as the step (tooling, not product)?  K separately allocated ViT-L/32-sized
vectors; every ordered role assignment of three distinct vectors is timed for
  explore  (theta rw, grad r, mom rw)       — the classes (fast iff theta/mom cross-class)
  sample   (out w, m1 r, m2 r)              bdl_posterior_sample, Philox, Welford variance
  moments  (theta r, m1 rw, m2 rw)          bdl_moments_update, running mean
HIP events, median of 5 launches.  One JSON line per (kernel, roles)."""
import itertools
import json
import sys

import torch

sys.path.insert(0, ".")
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import build_runs, _time_launch  # noqa: E402
from types import SimpleNamespace  # noqa: E402

n = 306535400
nv = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = torch.device("cuda", 0)
V = [torch.empty(n, device=dev).normal_(0, 0.02) for _ in range(nv)]
for v in V[1:]:
    v.abs_().mul_(1e-3)  # usable as a positive second moment
runs = build_runs([0], [n], [L.ATTR_PRIOR], n).to(dev)
K.set_launch_config(1, 4, 1)

for i, j, k in itertools.permutations(range(nv), 3):
    st = SimpleNamespace(theta=V[i], grad=V[j], mom=V[k], prior=None, noise=None, runs=runs,
                         nruns=1, n=n, device=dev)
    t = _time_launch(lambda: K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-9, 1e-9), noise_scale=(0, 0),
                                           noise_mode=L.NOISE_NONE, one_minus_alpha=0.5,
                                           prior_sig=0.0), dev)
    print(json.dumps({"kernel": "explore", "roles": [i, j, k], "ms": round(t, 4)}), flush=True)
for o, a, b in itertools.permutations(range(nv), 3):
    t = _time_launch(lambda: K.posterior_sample(V[o], V[a], V[b], var_mode=L.VAR_WELFORD,
                                                ratio=4.0, seed=7, chain=0, step=1), dev)
    print(json.dumps({"kernel": "sample", "roles": [o, a, b], "ms": round(t, 4)}), flush=True)
for th, a, b in itertools.permutations(range(nv), 3):
    t = _time_launch(lambda: K.moments_update(V[th], V[a], V[b], L.COLLECT_MEAN, collect_a=3.0,
                                              collect_b=4.0), dev)
    print(json.dumps({"kernel": "moments", "roles": [th, a, b], "ms": round(t, 4)}), flush=True)
