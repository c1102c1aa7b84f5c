"""Same-process A/B of two builds of libbdl_sgmcmc.so on the SAME buffers
(tooling).  Separate processes get different physical placements of their
vectors, which moves these sweeps by up to ~10 % (placement) and
hides a kernel change of a few percent; here both builds sweep one set of
allocations, alternating A, B, A, B, ...

  python tools/lib_ab.py LIB_A LIB_B [ROUNDS]

Prints one JSON line per (round, lib, kernel): HIP-event mean over 20 launches.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402

N = int(os.environ.get("AB_N", 306535400))
libs = [os.path.abspath(p) for p in sys.argv[1:3]]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = "cuda"
m1 = torch.randn(N, device=dev)
m2 = torch.rand(N, device=dev)
out = torch.empty(N, device=dev)
th = torch.randn(N, device=dev)


def use(path):
    L._lib = None
    L.LIB_PATH = path
    L.lib()
    K.set_launch_config(1, 4, 1)


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
    "moments_mean": (20, lambda i: K.moments_update(th, m1, m2, L.COLLECT_MEAN, float(i + 1),
                                                    float(i + 2))),
    "moments_welford": (20, lambda i: K.moments_update(th, m1, m2, L.COLLECT_WELFORD,
                                                       float(i + 2))),
}
results = {}
for r in range(rounds):
    for path in libs:
        use(path)
        for name, (bpe, fn) in kernels.items():
            ms = t(fn)
            results.setdefault((path, name), []).append(ms)
            print(json.dumps({"round": r, "lib": os.path.basename(path), "kernel": name,
                              "ms": round(ms, 4), "gbs": round(bpe * N / ms / 1e6, 1)}),
                  flush=True)
# the two builds must agree bit for bit on the same inputs
outs = []
for path in libs:
    use(path)
    K.posterior_sample(out, m1, m2, var_mode=L.VAR_WELFORD, ratio=4.0, seed=7, step=123)
    outs.append(out.clone())
print(json.dumps({"sample_outputs_identical": bool(torch.equal(outs[0].view(torch.int32),
                                                                 outs[1].view(torch.int32)))}))
for name in kernels:
    a = sorted(results[(libs[0], name)])
    b = sorted(results[(libs[1], name)])
    print(json.dumps({"kernel": name, "median_ms": {os.path.basename(libs[0]): a[len(a) // 2],
                                                    os.path.basename(libs[1]): b[len(b) // 2]}}))
