"""Do chunk composites alias, and are their timings real?  (tooling, not product)

Replays bayesdll_amd.placement's candidate construction on ViT-L/32-sized
vectors: K physical chunks, each mapped alone (the per-chunk views), and a
series of composites mapped, timed and dropped one after another (so virtual
ranges get reused).  For every composite:
  * each role is filled with its own constant through the composite, then
    every chunk's own view is read back: the chunk must hold the constant of
    the role that maps it (no aliasing, no stale translation);
  * the explore kernel is timed per launch (HIP events), every launch printed.
One JSON line per composite."""
import json
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import placement as P  # noqa: E402
from bayesdll_amd.flat import _placement_launcher, build_runs  # noqa: E402

n = 306535400
dev = torch.device("cuda", 0)
names = ["theta", "grad", "mom"]
per, cb = P.chunk_geometry(n)
K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
ncand = int(sys.argv[2]) if len(sys.argv) > 2 else 12
ch = P._Chunks(0, cb)
ch.add(K)
runs = build_runs([0], [n], [L.ATTR_PRIOR], n).to(dev)
rng = random.Random(5)
tail = n - (per - 1) * (cb // 4)  # elements of the last chunk a composite covers
for c in range(ncand):
    ids = rng.sample(range(K), 3 * per)
    assign = {nm: ids[q * per:(q + 1) * per] for q, nm in enumerate(names)}
    vec = {nm: P.Mapping(0, [ch.handles[k] for k in a], cb, n).tensor() for nm, a in assign.items()}
    for q, nm in enumerate(names):
        vec[nm].fill_(float(q + 1))
    torch.cuda.synchronize()
    bad = []
    for q, nm in enumerate(names):
        for k in assign[nm]:
            v = ch.views[k][:tail] if k == assign[nm][-1] else ch.views[k]
            lo, hi = float(v.min()), float(v.max())
            if lo != q + 1 or hi != q + 1:
                bad.append([nm, k, lo, hi])
    for v in vec.values():
        v.zero_()
    launch = _placement_launcher("csghmc", vec, n, dev, runs)
    launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(8)]
    for e0, e1 in ev:
        e0.record()
        launch()
        e1.record()
    torch.cuda.synchronize()
    ms = [round(a.elapsed_time(b), 4) for a, b in ev]
    print(json.dumps({"cand": c, "assign": assign,
                      "va": {nm: hex(t.data_ptr()) for nm, t in vec.items()},
                      "alias_errors": bad, "ms": ms}), flush=True)
    del vec, launch
ch.release()
