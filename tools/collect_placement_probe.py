"""Placement classes for the collect step and the posterior draw (tooling).

Allocates up to MAXV ViT-L/32-sized vectors with torch, sorts them into the
two physical classes by the explore step (theta = V0, mom = Vk: fast iff Vk is
in the other class), then times, with theta / mom already
split across the classes:
  collect  cSGHMC + Philox + Welford (theta rw, g r, mom rw, m1 rw, m2 rw)
           for m1 / m2 in each of the four class combinations;
  sample   bdl_posterior_sample (out w, m1 r, m2 r) for all eight.
One JSON line per timing (median of 5 launches)."""
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from types import SimpleNamespace  # noqa: E402

from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import _time_launch, build_runs  # noqa: E402

n = 306535400
MAXV = int(os.environ.get("MAXV", "20"))
dev = torch.device("cuda", 0)
runs = build_runs([0], [n], [L.ATTR_PRIOR], n).to(dev)
K.set_launch_config(1, 4, 1)
g = torch.empty(n, device=dev).normal_(0, 1e-3)
V = [torch.empty(n, device=dev).normal_(0, 0.02)]


def step(theta, mom, m1=None, m2=None, collect=L.COLLECT_NONE):
    st = SimpleNamespace(theta=theta, grad=g, mom=mom, prior=None, noise=None, runs=runs, nruns=1,
                         n=n, device=dev)
    return lambda: K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-9, 1e-9), noise_scale=(1e-9, 1e-9),
                                 noise_mode=L.NOISE_PHILOX if collect else L.NOISE_NONE,
                                 one_minus_alpha=0.5, prior_sig=0.0, collect=collect, mom1=m1,
                                 mom2=m2, collect_a=3.0, seed=1, chain=0, step=5)


cls = {0: "A"}
times = {}
while len(V) < MAXV:
    V.append(torch.empty(n, device=dev).normal_(0, 0.02).abs_())
    k = len(V) - 1
    times[k] = _time_launch(step(V[0], V[k]), dev)
    print(json.dumps({"classify": k, "ms": round(times[k], 4)}), flush=True)
    ms = sorted(times.values())
    nA = sum(1 for t in times.values() if t > 0.95 * ms[-1])
    if ms[0] < 0.95 * ms[-1] and len(times) >= 4 and nA >= 4 and len(times) - nA >= 3:
        break
ms = sorted(times.values())
if not ms[0] < 0.95 * ms[-1]:
    print(json.dumps({"error": "one class only among the allocations", "ms": ms}))
    sys.exit(0)
cut = 0.5 * (ms[0] + ms[-1])
for k, t in times.items():
    cls[k] = "B" if t < cut else "A"
A = [k for k in sorted(cls) if cls[k] == "A"]
B = [k for k in sorted(cls) if cls[k] == "B"]
print(json.dumps({"classes": cls}), flush=True)
if len(A) < 3 or len(B) < 3:
    print(json.dumps({"error": "not enough vectors per class", "A": A, "B": B}))
    sys.exit(0)
th, mo = A[0], B[0]
pool = {"A": A[1:], "B": B[1:]}
for rep in range(2):
    for c1, c2 in itertools.product("AB", repeat=2):
        a, b = pool[c1][0], (pool[c2][1] if c1 == c2 else pool[c2][0])
        for kind in (L.COLLECT_WELFORD, L.COLLECT_MEAN):
            t = _time_launch(step(V[th], V[mo], V[a], V[b], kind), dev)
            print(json.dumps({"kernel": "collect_welford" if kind == L.COLLECT_WELFORD else
                              "collect_mean", "m1": c1, "m2": c2, "ms": round(t, 4)}), flush=True)
    for co, c1, c2 in itertools.product("AB", repeat=3):
        used = {}

        def pick(c):
            used[c] = used.get(c, -1) + 1
            return pool[c][used[c]]
        try:
            o, a, b = pick(co), pick(c1), pick(c2)
        except IndexError:  # not enough vectors of that class for three distinct roles
            continue
        t = _time_launch(lambda: K.posterior_sample(V[o], V[a], V[b], var_mode=L.VAR_WELFORD,
                                                    ratio=4.0, seed=7, chain=0, step=1), dev)
        print(json.dumps({"kernel": "sample", "out": co, "m1": c1, "m2": c2, "ms": round(t, 4)}),
              flush=True)
