"""Launch-geometry sweep of the fused cSGHMC kernel on a ViT-L/32-sized chain.

For each (blocks_per_cu, unroll) it times, with HIP events on torch's stream,
the three kernel kinds of the benchmark schedule: explore (no noise, 20 B/el),
sample+collect (Philox + Welford, 36 B/el) and a pure Philox sample step
(20 B/el, not produced by the reference schedule with thin > 1 but the
noise-bearing variant of the same sweep).  Prints one JSON line per config.
"""
import itertools
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


def time_kind(st, kind, reps, m1, m2):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    kw = dict(lrs=(1e-4, 1e-2), noise_scale=(1e-7, 1e-6), one_minus_alpha=0.82, prior_sig=1.0,
              seed=42, chain=0)
    for i in range(reps + 3):
        if kind == "explore":
            args = dict(noise_mode=L.NOISE_NONE)
        elif kind == "sample":
            args = dict(noise_mode=L.NOISE_PHILOX)
        else:
            args = dict(noise_mode=L.NOISE_PHILOX, collect=L.COLLECT_WELFORD, mom1=m1, mom2=m2,
                        collect_a=3.0)
        if i >= 3:
            ev[i - 3][0].record()
        K.sgmcmc_step(st, L.CSGHMC, step=i, **kw, **args)
        if i >= 3:
            ev[i - 3][1].record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    reps = int(os.environ.get("REPS", "30"))
    segs, ro = segments("vit_l_32")
    st = FlatState.from_segments(segs, ro, device="cuda")
    st.theta.normal_(0, 0.02)
    st.grad.normal_(0, 1e-3)
    m1 = torch.zeros_like(st.theta)
    m2 = torch.zeros_like(st.theta)
    n = st.n
    bpcs = [int(x) for x in os.environ.get("BPC", "1,2,4,8").split(",")]
    unrolls = [int(x) for x in os.environ.get("UNROLL", "1,2,4").split(",")]
    strides = [int(x) for x in os.environ.get("GRID_STRIDE", "0,1").split(",")]
    for gs, bpc, un in itertools.product(strides, bpcs, unrolls):
        K.set_launch_config(bpc, un, gs)
        res = {"lib": os.path.basename(L.LIB_PATH), "grid_stride": gs, "blocks_per_cu": bpc,
               "unroll": un}
        kinds = os.environ.get("KINDS", "explore,sample,collect").split(",")
        for kind, bpe in (("explore", 20), ("sample", 20), ("collect", 36)):
            if kind not in kinds:
                continue
            ms = time_kind(st, kind, reps, m1, m2)
            res[kind] = {"ms": round(ms, 4), "gbs": round(bpe * n / ms / 1e6, 1)}
        print(json.dumps(res), flush=True)
    # plain device copy for reference (torch's own kernel): 8 B/el
    dst = torch.empty_like(st.theta)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        dst.copy_(st.theta)
    e0.record()
    for _ in range(reps):
        dst.copy_(st.theta)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"torch_copy": {"ms": round(ms, 4), "gbs": round(8 * n / ms / 1e6, 1)}}))


if __name__ == "__main__":
    main()
