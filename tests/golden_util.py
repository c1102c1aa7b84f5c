"""Helpers to load the golden fixtures (tests/golden/*.npz) and replay them."""
import json
import os

import numpy as np

from fakenet import grads_for_step

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = ["csghmc_k20", "csghmc_k21", "csghmc_fs_k20", "csgld_k20", "csgld_clip", "sgld_inf", "sgld_uninf_nomom",
            "sghmc_inf", "sghmc_uninf", "adam_sghmc_inf", "adam_sghmc_uninf_nomom",
            "adam_csghmc_k20", "adam_csghmc_clip"]


def load(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {k: d[k] for k in d.files}
    out["config"] = json.loads(str(out["config"]))
    if "segments" in out:
        out["segments"] = [(nm, tuple(s)) for nm, s in json.loads(str(out["segments"]))]
        out["readout"] = str(out["readout"])
    return out


def grad_fn(fx):
    cfg = fx["config"]
    n = fx["theta"].shape[1]
    return lambda t: grads_for_step(cfg["grad_seed"], t, n, cfg["grad_scale"])


def noise_fn(fx):
    return lambda t: fx["noise"][t]
