"""Locate CPU-vs-GPU divergence on the mlp_mnist cSGHMC chain (diagnostic).

Runs the reference's csghmc training loop restated with the oracle's
per-tensor rules + real autograd (i) on CPU, (ii) on the GPU with torch ops,
and (iii) the product Runner on the GPU; prints each one's distance to the
golden fixture and to each other, per step."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from fakenet import MLP, det_normal, init_vector, synthetic_mnist  # noqa: E402
from golden_util import load  # noqa: E402
from oracle import sgmcmc_oracle as O  # noqa: E402


def oracle_loop(fx, dev, steps=None):
    cfg = fx["config"]
    hp = {k: str(v) for k, v in cfg["hparams"].items()}
    net = MLP()
    n = sum(p.numel() for p in net.parameters())
    with torch.no_grad():
        torch.nn.utils.vector_to_parameters(torch.tensor(init_vector(cfg["init_seed"], n, 0.03)),
                                            net.parameters())
    net = net.to(dev)
    names = [nm for nm, _ in net.named_parameters()]
    train = synthetic_mnist(cfg["data_seed"], cfg["ntrain"], cfg["batch"], device=dev)
    sched = O.CyclicalSchedule(cfg["lr"], cfg["num_cycles"], cfg["epochs"], cfg["beta"])
    crit = torch.nn.CrossEntropyLoss()
    moms = [torch.zeros_like(p) for p in net.parameters()]
    k = 0
    bpe = len(train)
    traj = []
    for ep in range(cfg["epochs"]):
        for b, (x, y) in enumerate(train):
            lr = sched.calculate_lr(ep, b, bpe)
            ss = sched.should_sample(ep, b, bpe) and b % int(hp["thin"]) == 0
            out = net(x)
            loss = crit(out, y)
            net.zero_grad()
            loss.backward()
            params = list(net.parameters())
            noise = []
            for p in params:
                noise.append(torch.from_numpy(det_normal(cfg["noise_seed"], k, p.numel()))
                             .reshape(p.shape).to(dev))
                k += 1
            with torch.no_grad():
                moms = O.csghmc_update(params, [p.grad for p in params], moms, names, "classifier",
                                       [lr, lr * (cfg["lr_head"] / cfg["lr"])],
                                       float(hp["prior_sig"]), float(hp["momentum_decay"]),
                                       cfg["ND"] * float(hp["Ninflate"]), float(hp["nd"]), ss,
                                       noise)
            traj.append(torch.nn.utils.parameters_to_vector(net.parameters()).detach().cpu()
                        .numpy().copy())
    return traj


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def main():
    fx = load("mlp_csghmc_c2")
    idx = fx["idx"]
    cpu = oracle_loop(fx, "cpu")
    print("oracle-CPU final vs golden:", rel(cpu[-1][idx], fx["theta_sub"]))
    out = os.environ.get("DIAG_OUT")
    if out:
        np.savez_compressed(out, cpu=np.stack(cpu)[:, idx])
    if torch.cuda.is_available():
        gpu = oracle_loop(fx, "cuda")
        print("oracle-GPU final vs golden:", rel(gpu[-1][idx], fx["theta_sub"]))
        for t in range(len(cpu)):
            print(f"step {t}: oracle GPU vs CPU rel {rel(gpu[t], cpu[t]):.3e}")


if __name__ == "__main__":
    main()
