"""Does the read-only gradient's placement matter for the explore step?  (tooling)

One process, one box, ViT-L/32 size.  Builds the cSGHMC placement two ways:
  old: theta, grad, mom all placed (grad = a chunk composite, the round-2 set)
  new: theta, mom placed; grad a plain torch allocation (the round-3 set)
and times the explore step (HIP events, median of 20) on
  old set with its own grad / old theta+mom with a torch grad /
  new set with a torch grad / new theta+mom with the old set's grad,
alternating, 3 rounds.  One JSON line per measurement."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd import placement as P  # noqa: E402
from bayesdll_amd.flat import _placement_launcher, _time_launch, build_runs  # noqa: E402

n = 306535400
dev = torch.device("cuda", 0)
runs_by_n = {}


def launcher(roles, m):
    if m not in runs_by_n:
        runs_by_n[m] = build_runs([0], [m], [L.ATTR_PRIOR], m).to(dev)
    return _placement_launcher("csghmc", roles, m, dev, runs_by_n[m])


K.set_launch_config(1, 4, 1)
free, _ = torch.cuda.mem_get_info(dev)
per, cb = P.chunk_geometry(n)
gscratch = torch.zeros(max(n, cb // 4), device=dev)
old, old_info = P.place(n, dev, ["theta", "grad", "mom"], launcher,
                        lambda f: _time_launch(f, dev, 5), budget_bytes=int(0.25 * free))
new, new_info = P.place(n, dev, ["theta", "mom"],
                        lambda r, m: launcher(dict(r, grad=gscratch[:m]), m),
                        lambda f: _time_launch(f, dev, 5), budget_bytes=int(0.25 * free))
tgrad = torch.zeros(n, device=dev)
print(json.dumps({"old_chosen_ms": old_info["chosen_ms"], "old_kept": old_info["kept"],
                  "new_chosen_ms": new_info["chosen_ms"], "new_kept": new_info["kept"]}), flush=True)
combos = {
    "old_set_own_grad": dict(theta=old["theta"], grad=old["grad"], mom=old["mom"]),
    "old_set_torch_grad": dict(theta=old["theta"], grad=tgrad, mom=old["mom"]),
    "new_set_torch_grad": dict(theta=new["theta"], grad=tgrad, mom=new["mom"]),
    "new_set_old_grad": dict(theta=new["theta"], grad=old["grad"], mom=new["mom"]),
}
for r in range(3):
    for name, roles in combos.items():
        f = launcher(roles, n)
        for _ in range(3):
            f()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(20)]
        for e0, e1 in ev:
            e0.record()
            f()
            e1.record()
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        print(json.dumps({"round": r, "combo": name, "ms": round(ms, 4)}), flush=True)
