"""A/B of the overlapped update (Model.overlap: per-bucket launches from
post-accumulate hooks on a side stream) against the single launch after
backward, on one box: alternating blocks of STEPS full cSGHMC steps
(eager forward/backward), BACKBONE (vit_l_32 | resnet101), batch 16.
Tooling; one JSON line per block."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesdll_amd.csghmc as csghmc  # noqa: E402
from bayesdll_amd.backbones import backbone  # noqa: E402

name = os.environ.get("BACKBONE", "vit_l_32")
steps = int(os.environ.get("STEPS", "20"))
dev = "cuda"
torch.manual_seed(0)
net = backbone(name, 1000).to(dev)
x = torch.randn(16, 3, 224, 224, device=dev)
y = torch.randint(0, 1000, (16,), device=dev)
crit = torch.nn.CrossEntropyLoss()
model = csghmc.Model(ND=1840, prior_sig=1.0, momentum_decay=0.18)
model.noise_mode = "philox"
for k in range(3):
    model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=True)
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for ovl in (False, True):
        model.overlap = ovl
        for k in range(2):
            model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=k == 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=k % 10 == 0)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        print(json.dumps({"backbone": name, "round": rnd, "overlap": ovl,
                          "ms_per_step": round(ms, 3)}), flush=True)
