"""Adam-SGHMC + SGD step on ViT-L/32 (306,535,400 params, plain torch
allocations) with its state streams as separate vectors vs interleaved in a
flat.TiledState (tooling).  Every trial allocates a fresh set of state buffers
for every layout (earlier trials' buffers stay alive, so each trial lands on
other physical memory); within a trial the layouts alternate for ROUNDS
rounds, HIP-event mean of 10 launches each, at every geometry in GEOMS.
Also checks that each tiled layout produces the separate layout's bits.

  python tools/adam_tile_ab.py          (TRIALS=3 ROUNDS=2 GEOMS="1,1;2,1;4,1;2,2;4,2;1,4")
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("BDL_PLACEMENT", "0")
from bayesdll_amd import _lib as L  # noqa: E402
from bayesdll_amd import kernels as K  # noqa: E402
from bayesdll_amd.flat import FlatState, TiledState  # noqa: E402
from bayesdll_amd.shapes import segments  # noqa: E402

SLOTS = ("mom", "adam_m", "adam_v", "sgd_buf")
LAYOUTS = {"separate": (), "mvb": ("adam_m", "adam_v", "sgd_buf"),
           "all4": ("mom", "adam_m", "adam_v", "sgd_buf"), "mv": ("adam_m", "adam_v")}
trials = int(os.environ.get("TRIALS", "3"))
rounds = int(os.environ.get("ROUNDS", "2"))
geoms = [tuple(int(x) for x in g.split(",")) for g in os.environ.get("GEOMS", "1,1;2,1;4,1;2,2;4,2;1,4").split(";")]
dev = torch.device("cuda", 0)
segs, readout = segments("vit_l_32", 1000)
st = FlatState.from_segments(segs, readout, device=dev, placement=None, need_prior=True,
                             extra=("adam_m", "adam_v", "sgd_buf"))
n = st.n
gen = torch.Generator(device=dev).manual_seed(1)
st.theta.normal_(0.0, 0.02, generator=gen)
st.grad.normal_(0.0, 1e-3, generator=gen)
st.prior.normal_(0.0, 0.02, generator=gen)
theta0 = st.theta.clone()


def make(layout):
    """(tensors per slot, tile tuple or None, keep-alive)."""
    if not LAYOUTS[layout]:
        vecs = {nm: torch.zeros(n, dtype=torch.float32, device=dev) for nm in SLOTS}
        return vecs, None, vecs
    ts = TiledState(n, LAYOUTS[layout], dev)
    vecs = {nm: (ts.stream(nm) if nm in LAYOUTS[layout] else
                 torch.zeros(n, dtype=torch.float32, device=dev)) for nm in SLOTS}
    return vecs, ts.abi(SLOTS), (ts, vecs)


def launcher(vecs, tile):
    mom_saved = st.mom

    def go(i):
        st.mom = vecs["mom"]
        try:
            K.adam_step(st, L.ADAM_SGHMC, adam_m=vecs["adam_m"], adam_v=vecs["adam_v"],
                        sgd_buf=vecs["sgd_buf"], beta1=0.9, beta2=0.999, eps=1e-8, t=i + 2,
                        momentum_decay=0.18, nd=0.01, lrs=(1e-4, 1e-2),
                        noise_mode=L.NOISE_PHILOX, sigma2=1.0, n_data=1.84e6, mu=0.5,
                        momentum=True, first_step=False, seed=3, chain=0, step=i, tile=tile)
        finally:
            st.mom = mom_saved
    return go


def flat(v):
    return v if v.dim() == 1 else v.reshape(-1)[:n]


def bits_check(sets):
    """Three steps from the same start in every layout: identical theta and state."""
    out = {}
    for layout, (vecs, tile, _) in sets.items():
        st.theta.copy_(theta0)
        for nm in SLOTS:
            vecs[nm].zero_()
        go = launcher(vecs, tile)
        for i in range(3):
            go(i)
        torch.cuda.synchronize()
        out[layout] = [st.theta.clone()] + [flat(vecs[nm]).clone() for nm in SLOTS]
    ref = out["separate"]
    return {k: all(torch.equal(a, b) for a, b in zip(ref, v)) for k, v in out.items()}


def timeit(go, reps=10):
    for i in range(2):
        go(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        go(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


keep = []
for trial in range(trials):
    sets = {lay: make(lay) for lay in LAYOUTS}
    keep.append(sets)
    if trial == 0:
        print(json.dumps({"bit_identical": bits_check(sets)}), flush=True)
    for bpc, unroll in geoms:
        K.set_launch_config(bpc, unroll, 1)
        res = {lay: [] for lay in LAYOUTS}
        res["bare_mix_separate"] = []
        sv = sets["separate"][0]
        reads = [st.theta, st.grad, st.prior, sv["mom"], sv["adam_m"], sv["adam_v"], sv["sgd_buf"]]
        writes = [st.theta, sv["mom"], sv["adam_m"], sv["adam_v"], sv["sgd_buf"]]
        for _ in range(rounds):
            for lay, (vecs, tile, _) in sets.items():
                st.theta.copy_(theta0)
                for nm in SLOTS:  # the bare mix below overwrites the separate layout's state
                    vecs[nm].zero_()
                res[lay].append(round(timeit(launcher(vecs, tile)), 4))
            # the same access mix with no arithmetic, on the separate layout's buffers
            res["bare_mix_separate"].append(round(timeit(
                lambda i: K.stream_mix(reads, writes, bpc, unroll)), 4))
        print(json.dumps({"trial": trial, "geom": f"{bpc}x{unroll}", "ms": res,
                          "frac": {k: round(48 * n / (min(v) * 1e-3) / 8e12, 4)
                                   for k, v in res.items()}}), flush=True)
