"""Does the fused kernel's duration drift with sustained load (clock / power
state ramp)?  Runs the explore kernel back to back for DURATION seconds and
prints the mean per-launch time of every ~1 s window."""
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
    dur = float(os.environ.get("DURATION", "30"))
    segs, ro = segments("vit_l_32")
    st = FlatState.from_segments(segs, ro, device="cuda")
    st.theta.normal_(0, 0.02)
    st.grad.normal_(0, 1e-3)
    kw = dict(lrs=(1e-4, 1e-2), noise_scale=(1e-7, 1e-6), one_minus_alpha=0.82, prior_sig=1.0,
              noise_mode=L.NOISE_NONE)
    t_end = time.time() + dur
    i = 0
    while time.time() < t_end:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(500):
            K.sgmcmc_step(st, L.CSGHMC, step=i, **kw)
            i += 1
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 500
        print(json.dumps({"t": round(dur - (t_end - time.time()), 1), "ms": round(ms, 4),
                          "gbs": round(20 * st.n / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
