"""Is a fast physical placement a stable property of an allocation?  Allocates
K candidate (theta, grad, mom) sets at once, times the explore sweep on each
(interleaved, 3 passes), and reports per-set means — if the ranking holds
across passes, choosing the fastest set is meaningful."""
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
    k = int(os.environ.get("K", "6"))
    sets = []
    for i in range(k):
        st = FlatState.from_segments(segs, ro, device="cuda")
        st.theta.normal_(0, 0.02)
        st.grad.normal_(0, 1e-3)
        st.mom.zero_()
        sets.append(st)
    K.set_launch_config(1, 4, 1)
    kw = dict(lrs=(1e-4, 1e-2), noise_scale=(0.0, 0.0), one_minus_alpha=0.82, prior_sig=1.0,
              noise_mode=L.NOISE_NONE)
    res = [[] for _ in range(k)]
    for p in range(int(os.environ.get("PASSES", "3"))):
        for i, st in enumerate(sets):
            for _ in range(2):
                K.sgmcmc_step(st, L.CSGHMC, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                K.sgmcmc_step(st, L.CSGHMC, **kw)
            e1.record()
            e1.synchronize()
            res[i].append(round(e0.elapsed_time(e1) / 20, 4))
    for i in range(k):
        print(json.dumps({"set": i, "ms": res[i], "mean": round(float(np.mean(res[i])), 4)}))


if __name__ == "__main__":
    main()
