"""Placement classes for the Adam-SGHMC step (tooling).  Five vectors are
rewritten per step (theta, v_mom, Adam m, Adam v, the SGD buffer); the chain
placement pairs only theta / v_mom across the two physical classes
(DESIGN.md §4).  This sorts torch allocations into the two classes by the
explore step (theta = V0, mom = Vk: fast iff Vk is in the other class), then
times bdl_adam_step (Philox, SGD momentum, ViT-L/32 size) with theta in class
A, v_mom in class B and Adam m / Adam v / SGD buffer in each of the eight
class combinations.  One JSON line per timing (median of 5 launches)."""
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
dev = torch.device("cuda", 0)
runs = build_runs([0], [n], [L.ATTR_PRIOR], n).to(dev)
K.set_launch_config(1, 4, 1)
g = torch.empty(n, device=dev).normal_(0, 1e-3)
prior = torch.empty(n, device=dev).normal_(0, 0.02)
V = [torch.empty(n, device=dev).normal_(0, 0.02)]


def ns(theta, mom):
    return SimpleNamespace(theta=theta, grad=g, mom=mom, prior=prior, noise=None, runs=runs,
                           nruns=1, n=n, device=dev)


def explore(theta, mom):
    st = ns(theta, mom)
    return lambda: K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-9, 1e-9), noise_scale=(0, 0),
                                 noise_mode=L.NOISE_NONE, one_minus_alpha=0.5, prior_sig=0.0)


NV = int(os.environ.get("NV", "12"))
while len(V) < NV:
    V.append(torch.empty(n, device=dev).normal_(0, 1e-3).abs_())
pair = {}
for i, j in itertools.combinations(range(NV), 2):
    pair[(i, j)] = _time_launch(explore(V[i], V[j]), dev)
ms = sorted(pair.values())
print(json.dumps({"pairs": {f"{i},{j}": round(t, 4) for (i, j), t in pair.items()}}), flush=True)
if not ms[0] < 0.95 * ms[-1]:
    print(json.dumps({"error": "no fast pair among the allocations", "min": ms[0], "max": ms[-1]}))
    sys.exit(0)
cut = 0.5 * (ms[0] + ms[-1])
# two classes = a 2-colouring of the "fast" graph (a fast pair sits across the classes)
cls = {}
for root in range(NV):
    if root in cls:
        continue
    cls[root] = "A"
    stack = [root]
    while stack:
        u = stack.pop()
        for (i, j), t in pair.items():
            if t < cut and u in (i, j):
                w = j if u == i else i
                want = "B" if cls[u] == "A" else "A"
                if w not in cls:
                    cls[w] = want
                    stack.append(w)
print(json.dumps({"classes": cls}), flush=True)
A = [k for k in sorted(cls) if cls[k] == "A"]
B = [k for k in sorted(cls) if cls[k] == "B"]
if len(A) < 4 or len(B) < 4:
    A, B = (B, A) if len(B) > len(A) else (A, B)
if len(A) < 4 or len(B) < 4:
    print(json.dumps({"error": "not enough vectors per class", "A": A, "B": B}))
    sys.exit(0)
th, mo = A[0], B[0]
pool = {"A": A[1:], "B": B[1:]}
for rep in range(2):
    for combo in itertools.product("AB", repeat=3):
        used = {"A": 0, "B": 0}
        ids = []
        for c in combo:
            ids.append(pool[c][used[c]])
            used[c] += 1
        st = ns(V[th], V[mo])
        kw = dict(adam_m=V[ids[0]], adam_v=V[ids[1]], sgd_buf=V[ids[2]], beta1=0.9, beta2=0.999,
                  eps=1e-8, t=3, momentum_decay=0.1, nd=0.01, lrs=(1e-9, 1e-9),
                  noise_mode=L.NOISE_PHILOX, sigma2=1.0, n_data=1e6, mu=0.5, momentum=True)
        t = _time_launch(lambda: K.adam_step(st, L.ADAM_SGHMC, **kw), dev)
        print(json.dumps({"kernel": "adam", "m": combo[0], "v": combo[1], "buf": combo[2],
                          "ms": round(t, 4), "frac": round(48 * n / t / 1e6 / 8000, 4)}),
              flush=True)
