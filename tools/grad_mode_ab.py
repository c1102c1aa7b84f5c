"""What does reading the gradient per tensor cost the fused step (tooling)?

One placed ViT-L/32 cSGHMC state; the explore step timed with the flat
gradient vector ("flat" mode: 2 runs), then with the gradient read from 296
separate tensors through the per-run base table ("tensor" mode, what the
Runners use), on the same theta / mom; then, for every further library build
given, tensor mode again (same process, same buffers, alternating builds).

  python tools/grad_mode_ab.py [LIB ...]     (ROUNDS=4)
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

libs = [os.path.abspath(p) for p in sys.argv[1:]] or [L.LIB_PATH]
rounds = int(os.environ.get("ROUNDS", "4"))
dev = torch.device("cuda", 0)


def use(path):
    L._lib = None
    L.LIB_PATH = path
    L.lib()
    K.set_launch_config(1, 4, 1)


use(libs[0])
segs, readout = segments("vit_l_32", 1000)
st = FlatState.from_segments(segs, readout, device=dev, placement="csghmc")
gen = torch.Generator(device=dev).manual_seed(1)
st.theta.normal_(0.0, 0.02, generator=gen)
st.grad.normal_(0.0, 1e-3, generator=gen)
print(json.dumps({"placement_chosen_ms": st.placement_info.get("chosen_ms"),
                  "nruns_flat": int(st.nruns)}), flush=True)


def explore(i):
    K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-4, 1e-2), noise_scale=(0.0, 0.0), noise_mode=L.NOISE_NONE,
                  one_minus_alpha=0.82, prior_sig=1.0)


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


res = {}
for r in range(rounds):
    res.setdefault(("flat", os.path.basename(libs[0])), []).append(t(explore))
grads = [st.grad[o:o + k].clone() for o, k in zip(st.offsets, st.numels)]
st.use_tensor_grads(grads)
print(json.dumps({"nruns_tensor": int(st.nruns)}), flush=True)
for r in range(rounds):
    for path in libs:
        use(path)
        res.setdefault(("tensor", os.path.basename(path)), []).append(t(explore))
for (mode, lib), v in res.items():
    print(json.dumps({"mode": mode, "lib": lib, "median_ms": round(float(np.median(v)), 4),
                      "all_ms": [round(x, 4) for x in v]}), flush=True)
