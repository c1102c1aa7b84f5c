"""Checkpoint interop, product -> reference direction (tooling, two halves).

  GPU box:   python tools/ckpt_interop.py write gpurun_out/interop
      trains the PRODUCT Runner (bayesdll_amd.csghmc / .sgld) with the
      CKPT_CONFIGS of tests/golden/gen_golden.py (same data, init, noise
      stream), copies the checkpoint its save_ckpt wrote, and records what a
      fresh product Runner predicts from that file (eval noise restarted).
  container: PYTHONDONTWRITEBYTECODE=1 python tools/ckpt_interop.py check gpurun_out/interop
      loads each product checkpoint into a fresh REFERENCE Runner (imported
      read-only from /root/reference, as gen_golden.py does), evaluates with
      the same noise stream, and compares with the product's prediction.

The other direction (reference-written checkpoint -> product) is a test:
tests/test_gpu_runner_e2e.py::test_reference_written_checkpoint_loads_and_predicts_alike.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import shutil
import sys
import tempfile
from types import SimpleNamespace

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

from fakenet import MLP, det_normal, init_vector, synthetic_mnist  # noqa: E402


def configs():
    import gen_golden
    return copy.deepcopy(gen_golden.CKPT_CONFIGS)


class Det:
    """det_normal draws, one per tensor, counter k (the gen_golden stream)."""

    def __init__(self, seed, numels):
        self.seed, self.numels, self.k = seed, numels, 0

    def __call__(self, step, buf):
        parts = []
        for n in self.numels:
            parts.append(det_normal(self.seed, self.k, n))
            self.k += 1
        buf.copy_(torch.from_numpy(np.concatenate(parts)))


def make_args(cfg, dev, tmp, noise_mode=None):
    kw = dict(device=dev, ND=cfg["ND"], pretrained=None, lr=cfg["lr"], lr_head=cfg["lr_head"],
              momentum=cfg.get("momentum", 0.0), epochs=cfg["epochs"],
              num_cycles=cfg.get("num_cycles", 2), proportion_exploration=cfg.get("beta", 0.5),
              full_sample=False, test_eval_freq=1, ece_num_bins=15, log_dir=tmp, num_classes=10,
              hparams={k: str(v) for k, v in cfg["hparams"].items()})
    if noise_mode:
        kw["noise_mode"] = noise_mode
    return SimpleNamespace(**kw)


def fresh_net(cfg, init_seed, width_net):
    torch.manual_seed(0)
    net = width_net()
    n = sum(p.numel() for p in net.parameters())
    with torch.no_grad():
        torch.nn.utils.vector_to_parameters(torch.tensor(init_vector(init_seed, n, 0.03)),
                                            net.parameters())
    return net


def write(outdir):
    import bayesdll_amd.csghmc as csghmc
    import bayesdll_amd.sgld as sgld
    os.makedirs(outdir, exist_ok=True)
    dev = "cuda"
    rec = {}
    for method, cfg in configs().items():
        mod = {"csghmc": csghmc, "sgld": sgld}[method]
        train = synthetic_mnist(cfg["data_seed"], cfg["ntrain"], cfg["batch"], device=dev)
        test = synthetic_mnist(cfg["data_seed"] + 100, cfg["ntest"], cfg["batch"], device=dev)
        tmp = tempfile.mkdtemp()
        net = fresh_net(cfg, cfg["init_seed"], lambda: MLP(width=cfg["width"])).to(dev)
        runner = mod.Runner(net, None, make_args(cfg, dev, tmp, "external"), logging.getLogger("w"))
        numels = [p.numel() for p in runner.net.parameters()]
        runner.model.noise_provider = Det(cfg["noise_seed"], numels)
        runner.train(train, None, test)
        dst = os.path.join(outdir, f"ckpt_product_{method}.pt")
        shutil.copyfile(os.path.join(tmp, cfg["ckpt"]), dst)
        # what a fresh product Runner predicts from the file
        net = fresh_net(cfg, cfg["init_seed"] + 1000, lambda: MLP(width=cfg["width"])).to(dev)
        fresh = mod.Runner(net, None, make_args(cfg, dev, tempfile.mkdtemp(), "external"),
                           logging.getLogger("w"))
        prov = Det(cfg["eval_noise_seed"], numels)
        fresh.model.noise_provider = prov
        epoch = fresh.load_ckpt(dst)
        loss, err, targets, logits, logits_all = fresh.evaluate(test)
        rec.update({f"{method}_epoch": np.int64(epoch), f"{method}_loss": np.float64(loss),
                    f"{method}_err": np.float64(err), f"{method}_logits": logits,
                    f"{method}_logits_all": logits_all, f"{method}_draws": np.int64(prov.k)})
        print(f"{method}: wrote {dst} epoch={epoch} loss={loss:.6f} draws={prov.k}", flush=True)
    np.savez(os.path.join(outdir, "product_eval.npz"), **rec)


def check(outdir):
    import gen_golden
    methods = gen_golden.import_reference()
    from networks import small_nets
    logging.basicConfig(level=logging.WARNING)
    got = dict(np.load(os.path.join(outdir, "product_eval.npz")))
    orig = torch.randn_like
    ok = True
    for method, cfg in configs().items():
        mod = getattr(methods, method)
        test = synthetic_mnist(cfg["data_seed"] + 100, cfg["ntest"], cfg["batch"])
        counter = [0]

        def det_randn_like(t, *a, **k):
            out = torch.from_numpy(det_normal(cfg["eval_noise_seed"], counter[0], t.numel()))
            counter[0] += 1
            return out.reshape(t.shape).to(t.dtype)

        def width_net():
            m = small_nets.MLP(input_dim=784, output_dim=10, width=cfg["width"], depth=3)
            m.readout_name = "classifier"
            return m

        net = fresh_net(cfg, cfg["init_seed"] + 1000, width_net)
        runner = mod.Runner(net, None, make_args(cfg, "cpu", tempfile.mkdtemp()),
                            logging.getLogger("c"))
        torch.randn_like = det_randn_like
        try:
            epoch = runner.load_ckpt(os.path.join(outdir, f"ckpt_product_{method}.pt"))
            loss, err, targets, logits, logits_all = runner.evaluate(test)
        finally:
            torch.randn_like = orig
        rel = float(np.max(np.abs(logits - got[f"{method}_logits"])) /
                    np.max(np.abs(got[f"{method}_logits"])))
        row = {"method": method, "epoch_ref": int(epoch), "epoch_product": int(got[f"{method}_epoch"]),
               "draws_ref": counter[0], "draws_product": int(got[f"{method}_draws"]),
               "loss_ref": loss, "loss_product": float(got[f"{method}_loss"]),
               "err_ref": err, "err_product": float(got[f"{method}_err"]), "logits_max_rel": rel}
        good = (row["epoch_ref"] == row["epoch_product"] and row["draws_ref"] == row["draws_product"]
                and rel < 1e-4 and err == row["err_product"])
        ok &= good
        print(json.dumps(dict(row, ok=good)))
    return 0 if ok else 1


if __name__ == "__main__":
    mode, outdir = sys.argv[1], sys.argv[2]
    if mode == "write":
        write(outdir)
    else:
        sys.exit(check(outdir))
