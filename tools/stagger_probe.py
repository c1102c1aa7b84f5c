"""Does the relative placement of the swept vectors matter (HBM channel /
bank camping)?  Carves theta, grad and mom out of ONE allocation at offsets
0, n + d, 2n + 2d (floats) for several strides d and times the cSGHMC explore
sweep (ViT-L/32 size) on each layout, alternating layouts to cancel drift."""
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


def main():
    segs, ro = segments("vit_l_32")
    st = FlatState.from_segments(segs, ro, device="cuda", need_mom=True)
    n = st.n
    del st
    strides_b = [int(x) for x in os.environ.get("STRIDES", "0,256,4096,65536,1048576,3145728").split(",")]
    pad = max(strides_b) // 4 + 64
    big = torch.zeros(3 * (n + pad) + 64, dtype=torch.float32, device="cuda")
    K.set_launch_config(1, 4, 1)
    kw = dict(lrs=(1e-4, 1e-2), noise_scale=(0.0, 0.0), one_minus_alpha=0.82, prior_sig=1.0,
              noise_mode=L.NOISE_NONE)
    res = {d: [] for d in strides_b}
    for rep in range(int(os.environ.get("REPS", "4"))):
        for d in strides_b:
            df = d // 4
            st = FlatState.from_segments(segs, ro, device="cuda", need_mom=True,
                                         init=big[0:n])
            st.grad = big[n + df:2 * n + df]
            st.mom = big[2 * (n + df):2 * (n + df) + n]
            for _ in range(3):
                K.sgmcmc_step(st, L.CSGHMC, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                K.sgmcmc_step(st, L.CSGHMC, **kw)
            e1.record()
            e1.synchronize()
            res[d].append(e0.elapsed_time(e1) / 50)
    for d in strides_b:
        ms = float(np.mean(res[d]))
        print(json.dumps({"stride_bytes": d, "ms": round(ms, 4), "all": [round(x, 4) for x in res[d]],
                          "gbs": round(20 * n / ms / 1e6, 1)}))
    print(json.dumps({"base_addr_mod_2MB": big.data_ptr() % (2 << 20)}))


if __name__ == "__main__":
    main()
