"""Does the explore kernel's duration drift with sustained load (clock /
power-state ramp) right after the chain state is built?  Runs the ViT-L/32
explore sweep back to back for DURATION seconds (geometry GEOM, default the
tuned 1 x 4) and prints the mean per-launch time of every WINDOW launches,
with the wall time since the state existed — what a short bench (the driver's
--steps 20) would read at that moment.

  DURATION=8 WINDOW=20 python tools/drift.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import FlatState  # noqa: E402
from bayesdll_amd.shapes import segments  # noqa: E402


def main():
    dur = float(os.environ.get("DURATION", "8"))
    win = int(os.environ.get("WINDOW", "20"))
    geom = tuple(int(x) for x in os.environ.get("GEOM", "1,4,1").split(","))
    segs, ro = segments("vit_l_32")
    st = FlatState.from_segments(segs, ro, device="cuda")
    st.theta.normal_(0, 0.02)
    st.grad.normal_(0, 1e-3)
    torch.cuda.synchronize()
    K.set_launch_config(*geom)
    kw = dict(lrs=(1e-4, 1e-2), noise_scale=(0.0, 0.0), one_minus_alpha=0.82, prior_sig=1.0,
              noise_mode=L.NOISE_NONE)
    t0 = time.time()
    i = 0
    while time.time() - t0 < dur:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(win):
            K.sgmcmc_step(st, L.CSGHMC, step=i, **kw)
            i += 1
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / win
        print(json.dumps({"t_s": round(time.time() - t0, 3), "launches": i, "ms": round(ms, 4),
                          "frac": round(20 * st.n / ms / 1e6 / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
