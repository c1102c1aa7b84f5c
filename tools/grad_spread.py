"""Does the GRADIENT's physical memory move the explore step on this box?
Builds the chain state as bench.py does (autotune on placed scratch vectors,
whose parked set the chain state takes), then times the cSGHMC explore step
with the state's theta / mom and each of NGRAD gradient vectors allocated by
torch (interleaved ROUNDS rounds, median of REPS launches each).  One JSON
line to stdout."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import FlatState, _time_launch  # noqa: E402
from bayesdll_amd.shapes import segments  # noqa: E402


def main():
    ngrad, rounds, reps = (int(os.environ.get(k, d)) for k, d in
                           (("NGRAD", "8"), ("ROUNDS", "3"), ("REPS", "10")))
    segs, readout = segments("vit_l_32", 1000)
    n = sum(int(np.prod(s)) for _, s in segs)
    best, _ = K.autotune(n, device=0, method="csghmc", placed=True)
    st = FlatState.from_segments(segs, readout, device=torch.device("cuda", 0), placement="csghmc")
    st.theta.normal_(0, 0.02)
    st.grad.normal_(0, 1e-3)
    grads = [st.grad] + [torch.empty(n, device="cuda").normal_(0, 1e-3) for _ in range(ngrad - 1)]
    own = st.grad
    kw = dict(lrs=(1e-4, 1e-2), noise_scale=(0.0, 0.0), noise_mode=L.NOISE_NONE,
              one_minus_alpha=0.82, prior_sig=1.0)
    times = [[] for _ in grads]
    for r in range(rounds):
        for k, g in enumerate(grads):
            st.grad = g
            times[k].append(_time_launch(lambda: K.sgmcmc_step(st, L.CSGHMC, **kw), 0, reps))
    st.grad = own
    ms = [float(np.mean(t)) for t in times]
    print(json.dumps({"geometry": best, "placement_chosen_ms": st.placement_info.get("chosen_ms"),
                      "grad_ms": [round(x, 4) for x in ms],
                      "spread": round(max(ms) / min(ms) - 1, 4),
                      "rounds": [[round(x, 4) for x in t] for t in times]}))


if __name__ == "__main__":
    main()
