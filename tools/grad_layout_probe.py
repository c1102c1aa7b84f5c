"""Which property of the per-tensor gradient layout costs the explore sweep
its last 1-2 % against the flat gradient (tooling)?

One ViT-L/32 FlatState (theta, momentum, flat gradient from torch's caching
allocator), the explore step (csghmc, no noise) at geometries 1 x 4 and 1 x 1,
HIP-event mean of 20 launches, every layout below timed in turn for ROUNDS
rounds (so a layout's number is never a different moment's):

  flat        the flat gradient vector (the headline)
  views       296 views of the flat gradient through the per-tensor table
  copy0       one new allocation, tensor t at 4*offset_t (same layout as flat)
  gapP        one new allocation, tensor t at 4*offset_t + t*P bytes (P in
              GAPS: a gap of P bytes after every tensor — keeps each tensor's
              address phase against theta modulo P, breaks it modulo larger)
  rev         one new allocation, tensors in reverse order, packed
  revalign    reverse order, each tensor placed at its flat offset's phase
              modulo 2 MiB
  caching     296 clones from torch's default pool (backward order)
  arena       296 clones from the gradient arena's pool (backward order)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import arena as A  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import FlatState  # noqa: E402
from bayesdll_amd.shapes import segments  # noqa: E402

ROUNDS = int(os.environ.get("ROUNDS", "3"))
GEOMS = [(1, 4, 1), (1, 1, 1)]
GAPS = [int(x) for x in os.environ.get("GAPS", "4096,2097152,1048832").split(",")]
dev = torch.device("cuda", 0)
segs, readout = segments("vit_l_32", 1000)
st = FlatState.from_segments(segs, readout, device=dev)
gen = torch.Generator(device=dev).manual_seed(1)
st.theta.normal_(0.0, 0.02, generator=gen)
st.grad.normal_(0.0, 1e-3, generator=gen)
flat = st.grad
offs, nums = st.offsets, st.numels
nt = len(nums)


def placed(starts_bytes, total_bytes):
    """One allocation; tensor t's gradient at byte starts_bytes[t] of it."""
    buf = torch.empty(total_bytes // 4 + 1024, dtype=torch.float32, device=dev)
    out = []
    for t in range(nt):
        s = starts_bytes[t] // 4
        v = buf[s:s + nums[t]]
        v.copy_(flat[offs[t]:offs[t] + nums[t]])
        out.append(v)
    return buf, out


layouts = {}
layouts["views"] = (None, [flat[o:o + k] for o, k in zip(offs, nums)])
layouts["copy0"] = placed([4 * o for o in offs], 4 * st.n)
for P in GAPS:
    layouts[f"gap{P}"] = placed([4 * o + t * P for t, o in enumerate(offs)], 4 * st.n + nt * P)
pos, starts = 0, [0] * nt
for t in reversed(range(nt)):
    starts[t] = pos
    pos += 4 * nums[t]
    pos = (pos + 255) // 256 * 256
layouts["rev"] = placed(starts, pos)
M = 2 << 20
pos, starts = 0, [0] * nt
for t in reversed(range(nt)):
    want = (4 * offs[t]) % M
    cand = pos - pos % M + want
    if cand < pos:
        cand += M
    starts[t] = cand
    pos = cand + 4 * nums[t]
layouts["revalign"] = placed(starts, pos)
M2 = 2 << 20
pos, starts = 0, [0] * nt
for t in range(nt):
    starts[t] = pos
    pos = (pos + 4 * nums[t] + M2 - 1) // M2 * M2
layouts["fwd2M"] = placed(starts, pos)
pos, starts = 0, [0] * nt
for t in reversed(range(nt)):
    starts[t] = pos
    pos = (pos + 4 * nums[t] + M2 - 1) // M2 * M2
layouts["rev2M"] = placed(starts, pos)
g = [None] * nt
for t in reversed(range(nt)):
    g[t] = flat[offs[t]:offs[t] + nums[t]].clone()
layouts["caching"] = (None, g)
layouts["cachingfwd"] = (None, [flat[offs[t]:offs[t] + nums[t]].clone() for t in range(nt)])
ar = A.GradArena(dev, 4 * st.n)
with ar.routing():
    g = [None] * nt
    for t in reversed(range(nt)):
        g[t] = flat[offs[t]:offs[t] + nums[t]].clone()
layouts["arena"] = (None, g)
with ar.routing():
    layouts["arenafwd"] = (None, [flat[offs[t]:offs[t] + nums[t]].clone() for t in range(nt)])


def use(name):
    st.grad_mode, st.grad, st.gbase, st._untouched = "flat", flat, None, ()
    st.runs, st.nruns = st._base_runs
    if name != "flat":
        st.use_tensor_grads(layouts[name][1])


def explore(i):
    K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-5, 1e-3), noise_scale=(0.0, 0.0),
                  noise_mode=L.NOISE_NONE, one_minus_alpha=0.82, prior_sig=1.0,
                  seed=0, chain=0, step=i)


def timed(reps=20):
    for i in range(2):
        explore(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        explore(i)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


names = ["flat"] + list(layouts)
res = {(nm, g): [] for nm in names for g in GEOMS}
for r in range(ROUNDS):
    for g in GEOMS:
        K.set_launch_config(*g)
        for nm in names:
            use(nm)
            res[(nm, g)].append(timed())
    print(json.dumps({"round": r}), flush=True)
for g in GEOMS:
    base = np.mean(res[("flat", g)])
    for nm in names:
        v = np.mean(res[(nm, g)])
        print(json.dumps({"geometry": f"{g[0]}x{g[1]}", "layout": nm, "ms": round(float(v), 4),
                          "vs_flat": round(float(v / base), 4),
                          "rounds": [round(x, 4) for x in res[(nm, g)]]}), flush=True)
