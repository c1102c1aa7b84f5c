"""The full (theta, mom) pair-time matrix of NCHUNK physical chunks of a
ViT-L/32 vector's chunk size (586 MB), timed with the cSGHMC placement probe
(bayesdll_amd.placement / flat._placement_launcher, 1 workgroup/CU x 4), plus
full-size composites drawn from the pair levels it shows — to calibrate the
search's thresholds (chunk-level contrast vs full-size contrast).

Prints one JSON line: {"pairs": {"i,j": ms}, "composites": [...]} into
gpurun_out/chunk_matrix.jsonl (append)."""
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


def main():
    nchunk = int(os.environ.get("NCHUNK", "40"))
    n = 306535400
    dev = torch.device("cuda", 0)
    per, cb = P.chunk_geometry(n)
    m = cb // 4
    K.set_launch_config(1, 4, 1)
    runs_m = build_runs([0], [m], [L.ATTR_PRIOR], m).to(dev)
    runs_n = build_runs([0], [n], [L.ATTR_PRIOR], n).to(dev)
    grad = torch.zeros(n, device=dev)
    ch = P._Chunks(0, cb)
    ch.add(nchunk)
    gm = grad[:m] if m <= n else torch.zeros(m, device=dev)
    pairs = {}
    for i in range(nchunk):
        for j in range(nchunk):
            if i != j:
                f = _placement_launcher("csghmc", {"theta": ch.views[i], "mom": ch.views[j],
                                                   "grad": gm}, m, dev, runs_m)
                pairs[f"{i},{j}"] = round(_time_launch(f, dev, 3), 4)
        print(f"row {i} done", file=sys.stderr, flush=True)
    # full-size composites: theta = (a, b), mom = (c, d) for a few choices
    mat = np.full((nchunk, nchunk), np.nan)
    for k, v in pairs.items():
        i, j = map(int, k.split(","))
        mat[i, j] = v
    sym = np.nanmean(np.stack([mat, mat.T]), axis=0)
    order = np.argsort(np.nanmin(sym, axis=1))
    comps = []
    rng = np.random.default_rng(0)
    picks = []
    for _ in range(int(os.environ.get("NCOMP", "16"))):
        a, b, c, d = rng.choice(nchunk, 4, replace=False)
        picks.append((int(a), int(b), int(c), int(d)))
    for a, b, c, d in picks:
        mt = P.Mapping(0, [ch.handles[a], ch.handles[b]], cb, n).tensor()
        mm = P.Mapping(0, [ch.handles[c], ch.handles[d]], cb, n).tensor()
        f = _placement_launcher("csghmc", {"theta": mt, "mom": mm, "grad": grad}, n, dev, runs_n)
        ms = _time_launch(f, dev, 5)
        comps.append({"theta": [a, b], "mom": [c, d], "ms": round(ms, 4),
                      "pair_ms": [pairs[f"{a},{c}"], pairs[f"{b},{d}"]]})
        del mt, mm
    ch.release()
    with open("gpurun_out/chunk_matrix.jsonl", "a") as fh:
        fh.write(json.dumps({"nchunk": nchunk, "chunk_mb": cb >> 20, "pairs": pairs,
                             "composites": comps}) + "\n")
    print(json.dumps({"composites": comps})[:2000])


if __name__ == "__main__":
    main()
