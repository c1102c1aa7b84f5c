"""Does the sweep time depend on how the chain's vectors are allocated?
Alternates (a) separate torch allocations per vector (theta, grad, mom) and
(b) one allocation carved into the three vectors, re-allocating every round
(torch.cuda.empty_cache in between, so physical pages change), and times the
cSGHMC explore sweep (ViT-L/32 size) under two launch geometries."""
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


def sweep_ms(st, reps=40):
    kw = dict(lrs=(1e-4, 1e-2), noise_scale=(0.0, 0.0), one_minus_alpha=0.82, prior_sig=1.0,
              noise_mode=L.NOISE_NONE)
    out = {}
    for cfg in ((1, 4, 1), (3, 1, 1)):
        K.set_launch_config(*cfg)
        for _ in range(3):
            K.sgmcmc_step(st, L.CSGHMC, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            K.sgmcmc_step(st, L.CSGHMC, **kw)
        e1.record()
        e1.synchronize()
        out[f"{cfg[0]}x{cfg[1]}"] = round(e0.elapsed_time(e1) / reps, 4)
    return out


def main():
    segs, ro = segments("vit_l_32")
    n = sum(int(np.prod(s)) for _, s in segs)
    for rnd in range(int(os.environ.get("ROUNDS", "4"))):
        for layout in ("separate", "single"):
            torch.cuda.empty_cache()
            if layout == "separate":
                st = FlatState.from_segments(segs, ro, device="cuda")
                big = None
            else:
                big = torch.empty(3 * n + 64, dtype=torch.float32, device="cuda")
                st = FlatState.from_segments(segs, ro, device="cuda", need_mom=False,
                                             init=big[0:n])
                st.grad = big[n + 4:2 * n + 4]
                st.mom = big[2 * n + 8:3 * n + 8]
            st.theta.normal_(0, 0.02)
            st.grad.normal_(0, 1e-3)
            st.mom.zero_()
            print(json.dumps({"round": rnd, "layout": layout, **sweep_ms(st),
                              "theta_addr_mod_2MB": st.theta.data_ptr() % (2 << 20)}), flush=True)
            del st, big


if __name__ == "__main__":
    main()
