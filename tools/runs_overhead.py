"""Cost of a per-tensor run table on the fused sweep (tooling).

Same buffers, same kernel, two run tables: the merged flat-mode table (ViT-L/32
cSGHMC: 2 runs) and the per-tensor table of "tensor" gradient mode (296 runs),
here pointing at views of the same flat gradient vector — so the only
difference is the run table (more iterations on the guarded slow path at
tensor boundaries).  Alternating HIP-event timings, one JSON line per round."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import FlatState  # noqa: E402
from bayesdll_amd.shapes import segments  # noqa: E402

backbone = os.environ.get("BACKBONE", "vit_l_32")
segs, readout = segments(backbone, 1000)
st = FlatState.from_segments(segs, readout, device="cuda", placement="csghmc")
st.theta.normal_(0, 0.02)
st.grad.normal_(0, 1e-3)
K.autotune_once(st.n, st.device, "csghmc")
flat_tab = st.grad_table()
grad = st.grad
st.use_tensor_grads([grad[o:o + k] for o, k in zip(st.offsets, st.numels)])
st.grad = grad  # keep the flat vector alive for the flat-table launches
tensor_tab = st.grad_table()
# isolating variants: the 296-run table without bases (flat gradient vector),
# and the 2-run merged table with a base per run (the flat vector's address)
runs296 = tensor_tab[0].clone()
runs296[:, 1] &= ~L.ATTR_GUNALIGNED
many_flat = (runs296, tensor_tab[1], None, ())
gb2 = torch.full((flat_tab[1],), grad.data_ptr(), dtype=torch.int64, device=st.device)
two_based = (flat_tab[0], flat_tab[1], gb2, ())


def launch():
    K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-4, 1e-2), noise_scale=(0.0, 0.0),
                  noise_mode=L.NOISE_NONE, one_minus_alpha=0.82, prior_sig=1.0)


def timed(tab, reps=50):
    st.use_grad_table(tab)
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for rnd in range(int(os.environ.get("ROUNDS", "4"))):
    a = timed(flat_tab)
    b = timed(tensor_tab)
    c = timed(many_flat)
    d = timed(two_based)
    print(json.dumps({"round": rnd, "runs_flat": int(flat_tab[1]), "runs_tensor": int(tensor_tab[1]),
                      "flat_2runs_ms": round(a, 4), "tensor_296runs_bases_ms": round(b, 4),
                      "flat_296runs_ms": round(c, 4), "bases_2runs_ms": round(d, 4),
                      "tensor_vs_flat_pct": round(100 * (b / a - 1), 2)}), flush=True)
