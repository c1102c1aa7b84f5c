"""Is ViT-L/32 forward/backward bitwise repeatable on this GPU (tooling)?

Runs the config-5 worker's chain 7 first (the process's first ViT-L/32
forward / backward), then the same batch through the random-init ViT-L/32 several times (with the
config-5 test's deterministic settings) and reports, per parameter, whether
its gradient came out bit-identical every time; then the config-5 worker's
single chain twice in this process.  Prints JSON lines."""
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
from bayesdll_amd.backbones import backbone  # noqa: E402
from config5_worker import deterministic_autograd, run_chain  # noqa: E402

dev = "cuda"
first = run_chain(chain=7)  # this process's first ViT-L/32 forward / backward
with deterministic_autograd():
    torch.manual_seed(0)
    net = backbone("vit_l_32", 1000).to(dev)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 3, 224, 224, generator=g).to(dev)
    y = torch.randint(0, 1000, (4,), generator=g).to(dev)
    crit = torch.nn.CrossEntropyLoss()
    runs = []
    for r in range(int(os.environ.get("REPS", "4"))):
        net.zero_grad(set_to_none=True)
        out = net(x)
        loss = crit(out, y)
        loss.backward()
        torch.cuda.synchronize()
        runs.append(([p.grad.clone() for p in net.parameters()], out.detach().clone()))
    names = [n for n, _ in net.named_parameters()]
    diff = [names[i] for i in range(len(names))
            if not all(torch.equal(runs[0][0][i], r[0][i]) for r in runs[1:])]
    print(json.dumps({"forward_identical": all(torch.equal(runs[0][1], r[1]) for r in runs[1:]),
                      "grads_differing": len(diff), "of": len(names), "first": diff[:12]}),
          flush=True)
a = run_chain(chain=7)
b = run_chain(chain=7)
print(json.dumps({"later_runs_identical": int(a["theta_bits"]) == int(b["theta_bits"]),
                  "first_run_equals_later": int(first["theta_bits"]) == int(a["theta_bits"]),
                  "bits": [int(first["theta_bits"]), int(a["theta_bits"]), int(b["theta_bits"])]}),
      flush=True)
