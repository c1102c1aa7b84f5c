"""mlp_mnist (or BACKBONE=...) cSGHMC steps through Model.forward (config 2 shape, batch 128),
eager or graph mode (GRAPH=1), for a kernel-trace profile: wall ms/step vs
the GPU kernel time per step from rocprofv3 --kernel-trace --stats. Tooling."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesdll_amd.csghmc as csghmc  # noqa: E402
from bayesdll_amd.backbones import backbone  # noqa: E402

steps = int(os.environ.get("STEPS", "500"))
dev = "cuda"
torch.manual_seed(0)
name = os.environ.get("BACKBONE", "mlp_mnist")
classes = 10 if name == "mlp_mnist" else 1000
net = backbone(name, classes).to(dev)
model = csghmc.Model(ND=30000, prior_sig=1.0, momentum_decay=0.18)
model.graph = os.environ.get("GRAPH", "1") == "1"
crit = torch.nn.CrossEntropyLoss()
batch = int(os.environ.get("BATCH", "128" if name == "mlp_mnist" else "16"))
x = torch.randn(*((batch, 1, 28, 28) if name == "mlp_mnist" else (batch, 3, 224, 224)), device=dev)
y = torch.randint(0, classes, (batch,), device=dev)
for k in range(int(os.environ.get("WARM", "20"))):
    model(x, y, net, None, crit, [1e-2, 1e-2], 1.0, 0.01, should_sample=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(steps):
    model(x, y, net, None, crit, [1e-2, 1e-2], 1.0, 0.01, should_sample=(k % 2 == 0))
torch.cuda.synchronize()
print(f"graph={model.graph} steps={steps} wall {((time.perf_counter() - t0) / steps) * 1e3:.4f} ms/step")
