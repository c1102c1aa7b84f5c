"""What does in-register Philox noise cost on the SGLD sweep (config 3 shape
and ViT-L/32)?  Times the SGLD + SGD-momentum kernel with no noise, Philox
noise and a noise buffer (+4 B/elem) under a few launch geometries."""
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


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    for bb in os.environ.get("BACKBONES", "resnet101,vit_l_32").split(","):
        segs, ro = segments(bb)
        st = FlatState.from_segments(segs, ro, device="cuda", need_prior=True, need_noise=True)
        st.theta.normal_(0, 0.02)
        st.grad.normal_(0, 1e-3)
        st.noise.normal_()
        kw = dict(lrs=(1e-4, 1e-2), noise_scale=(1e-3, 1e-2), sigma2=1.0, n_data=1.84e6, mu=0.5,
                  momentum=True)
        for cfg in ((1, 4, 1), (2, 1, 1), (3, 1, 1), (2, 2, 1)):
            K.set_launch_config(*cfg)
            row = {"backbone": bb, "cfg": cfg}
            for name, mode in (("none", L.NOISE_NONE), ("philox", L.NOISE_PHILOX),
                               ("buffer", L.NOISE_BUFFER)):
                ms = timeit(lambda: K.sgmcmc_step(st, L.SGLD, noise_mode=mode, **kw))
                b = 24 + (4 if mode == L.NOISE_BUFFER else 0)
                row[name] = {"ms": round(ms, 4), "gbs": round(b * st.n / ms / 1e6, 1)}
            print(json.dumps(row), flush=True)
        del st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
