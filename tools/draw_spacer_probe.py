"""Can the posterior draw's output buffer be steered into the other physical
class than its m1 / m2 reads by allocating it farther away (tooling, not
product)?  After a bench-like state (theta / grad / mom, four per-cycle
moment pairs and the draw's m1 / m2 pair from flat.moment_pair, ViT-L/32
size), output candidates are allocated behind spacer allocations of growing
size (kept alive while the probe runs) and the draw is timed into each (HIP
events, median of 5).  One JSON line per candidate."""
import json
import sys

import torch

sys.path.insert(0, ".")
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import _time_launch, moment_pair  # noqa: E402

n = 306535400
dev = torch.device("cuda", 0)
K.set_launch_config(2, 4, 1)
state = [torch.zeros(n, device=dev) for _ in range(3)]
cycles = [moment_pair(n, dev) for _ in range(4)]
m1, m2 = cycles[-1]
m1.normal_(0, 0.02)
m2.uniform_(1e-6, 1e-4)


def draw_ms(out):
    return _time_launch(lambda: K.posterior_sample(out, m1, m2, var_mode=L.VAR_WELFORD, ratio=4.0,
                                                   seed=7, chain=0, step=1), dev)


keep = []
for gb in [0, 0, 0, 1, 1, 2, 2, 4, 4, 8, 8, 16]:
    if gb:
        keep.append(torch.empty(gb << 28, device=dev))  # gb GiB of fp32
    out = torch.empty(n, device=dev)
    keep.append(out)
    print(json.dumps({"spacer_gib": gb, "allocated_gib": round(torch.cuda.memory_allocated(dev) / 2**30, 1),
                      "ms": round(draw_ms(out), 4)}), flush=True)
# the same candidates again (is a candidate's time stable?)
for k, t in enumerate(x for x in keep if x.numel() == n):
    print(json.dumps({"again": k, "ms": round(draw_ms(t), 4)}), flush=True)
