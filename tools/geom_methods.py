"""Launch geometry per sampler family on a placed ViT-L/32-sized state.

For each method (cSGHMC explore, SGLD + SGD momentum with Philox, Adam-SGHMC +
SGD momentum) builds the autotuner's own scratch state (kernels._scratch_launcher:
placed like a chain's vectors) and times the production kernel at a grid of
(workgroups/CU, unroll) geometries — the autotuner's six plus the deeper
occupancy ones — in ROUNDS interleaved passes (median of REPS launches each),
so box drift hits every geometry alike.  One JSON line per (method, geometry)
with the per-round medians and their mean.  Results never depend on geometry
(tests/test_gpu_geometry.py)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.shapes import segments  # noqa: E402

GEOMS = [(1, 1), (2, 1), (3, 1), (4, 1), (1, 2), (2, 2), (3, 2), (4, 2), (5, 2),
         (1, 4), (2, 4), (3, 4), (4, 4)]


def time_geom(launch, cfg, reps):
    K.set_launch_config(cfg[0], cfg[1], 1)
    for _ in range(2):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        launch()
        e1.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def collect_launcher(n):
    from bayesdll_amd import _lib as L
    from bayesdll_amd.flat import FlatState, moment_pair
    st = FlatState.from_segments([("w", (int(n),))], None, device="cuda", placement="csghmc")
    st.theta.normal_(0, 0.02)
    st.grad.normal_(0, 1e-3)
    m1, m2 = moment_pair(n, st.device)
    m1.copy_(st.theta)
    m2.zero_()

    def launch():
        K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-4, 1e-2), noise_scale=(1e-7, 1e-6),
                      noise_mode=L.NOISE_PHILOX, one_minus_alpha=0.82, prior_sig=1.0,
                      collect=L.COLLECT_WELFORD, mom1=m1, mom2=m2, collect_a=3.0, seed=42,
                      chain=0, step=1)
    return launch


def main():
    reps = int(os.environ.get("REPS", "10"))
    rounds = int(os.environ.get("ROUNDS", "3"))
    methods = os.environ.get("METHODS", "csghmc,sgld,adam").split(",")
    # "collect": the cSGHMC Welford collect step (Philox + m1 / m2 of one
    # flat.moment_pair) on the explore's placed scratch state
    segs, _ = segments("vit_l_32")
    n = sum(int(np.prod(s)) for _, s in segs)
    for method in methods:
        if method == "collect":
            launch = collect_launcher(n)
        else:
            launch = K._scratch_launcher(n, torch.device("cuda", 0), method, placed=True)
        per = {g: [] for g in GEOMS}
        for r in range(rounds):
            order = GEOMS if r % 2 == 0 else GEOMS[::-1]
            for g in order:
                per[g].append(time_geom(launch, g, reps))
        best = min(per, key=lambda g: np.mean(per[g]))
        for g in GEOMS:
            print(json.dumps({"method": method, "blocks_per_cu": g[0], "unroll": g[1],
                              "ms_rounds": [round(t, 4) for t in per[g]],
                              "ms_mean": round(float(np.mean(per[g])), 4),
                              "vs_best": round(float(np.mean(per[g]) / np.mean(per[best])), 4),
                              "autotune_candidate": (g[0], g[1], 1) in K.AUTOTUNE_CANDIDATES}),
                  flush=True)
        del launch
        import gc
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
