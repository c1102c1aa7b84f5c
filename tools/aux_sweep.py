"""Launch-geometry sweep for the stand-alone sweeps (posterior sample, moments)
at ViT-L/32 size: workgroups per CU via bdl_set_launch_config, HIP events.
Tooling; prints one JSON line per (kernel, blocks/CU)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402

N = 306535400
dev = "cuda"
m1 = torch.randn(N, device=dev)
m2 = torch.rand(N, device=dev)
out = torch.empty(N, device=dev)
th = torch.randn(N, device=dev)


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


kernels = {
    "sample_welford_philox": (12, lambda i: K.posterior_sample(
        out, m1, m2, var_mode=L.VAR_WELFORD, ratio=4.0, seed=7, step=i)),
    "sample_raw_philox": (12, lambda i: K.posterior_sample(
        out, m1, m2, var_mode=L.VAR_RAW_MOMENTS, ratio=1.25, seed=7, step=i)),
    "moments_mean": (20, lambda i: K.moments_update(th, m1, m2, L.COLLECT_MEAN, float(i + 1),
                                                    float(i + 2))),
    "moments_welford": (20, lambda i: K.moments_update(th, m1, m2, L.COLLECT_WELFORD,
                                                       float(i + 2))),
    "philox_normal": (4, lambda i: L.check(L.lib().bdl_philox_normal(
        out.data_ptr(), N, 7, 0, i, L.current_stream_handle(out.device)), "philox")),
}
for bpc in [int(b) for b in os.environ.get("BPCS", "1,2,3,4,6,8,12,16").split(",")]:
    K.set_launch_config(bpc, 1, 1)
    for name, (bpe, fn) in kernels.items():
        ms = t(fn)
        print(json.dumps({"lib": os.environ.get("BDL_SGMCMC_LIB", "prod"), "kernel": name, "blocks_per_cu": bpc, "ms": round(ms, 4),
                          "gbs": round(bpe * N / ms / 1e6, 1)}), flush=True)
