"""Chain-steps/s of K stacked cSGHMC chains on one GPU (bayesdll_amd.stacked)
vs one chain per step (the fused Runner Model, eager and HIP-graph).

Synthetic MNIST-shaped batch, shared by the chains; every 10th step a noise
(sample) step, as in e2e_compare.py.  Informational; not the bench metric.

    BACKBONE=mlp_mnist BATCH=128 STEPS=50 KS=1,4,16,64,256 python tools/stacked_throughput.py
"""
import os
import sys
import time
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesdll_amd.csghmc as csghmc  # noqa: E402
from bayesdll_amd import stacked  # noqa: E402
from bayesdll_amd.backbones import backbone  # noqa: E402


def main():
    name = os.environ.get("BACKBONE", "mlp_mnist")
    batch = int(os.environ.get("BATCH", "128"))
    steps = int(os.environ.get("STEPS", "50"))
    ks = [int(k) for k in os.environ.get("KS", "1,4,16,64,256").split(",")]
    dev = "cuda"
    x = torch.randn(batch, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (batch,), device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def timed(fn):
        for k in range(3):
            fn(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            fn(3 + k)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    for graph in (False, True):
        torch.manual_seed(0)
        net = backbone(name, 10).to(dev)
        model = csghmc.Model(ND=60000, prior_sig=1.0, momentum_decay=0.1)
        model.graph = graph
        ms = timed(lambda k: model(x, y, net, None, crit, [1e-4, 1e-4], 1.0, 1.0,
                                   should_sample=k % 10 == 0))
        print(f"{name} batch {batch}: one chain, fused{' + graph' if graph else ''}: "
              f"{ms:.3f} ms/step, {1e3 / ms:.0f} chain-steps/s", flush=True)

    args = SimpleNamespace(lr=1e-4, lr_head=1e-4, epochs=1, num_cycles=1,
                           proportion_exploration=0.5, ND=60000, device=dev, seed=0,
                           hparams={"prior_sig": 1.0, "momentum_decay": 0.1, "Ninflate": 1.0,
                                    "nd": 1.0, "thin": 1, "nst": 0, "bias": "informative"})
    for K_, graph in [(k, g) for k in ks for g in (False, True)]:
        torch.manual_seed(0)
        S = stacked.StackedCSGHMC(backbone(name, 10).to(dev), K_, args, init="reinit",
                                  graph=graph)
        ms = timed(lambda k: S.step(x, y, 1e-4, should_sample=k % 10 == 0))
        # the fused update alone, over K * n elements (20 B/element, explore)
        grads, _, _ = S.gradients(x, y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            S.update(grads, 1e-4)
        e0.record()
        for _ in range(20):
            S.update(grads, 1e-4)
        e1.record()
        torch.cuda.synchronize()
        ums = e0.elapsed_time(e1) / 20
        gbs = 20 * S.state.n / (ums * 1e-3) / 1e9
        print(f"{name} batch {batch}: {K_} stacked chains{' + graph' if graph else ''} "
              f"({S.state.grad_mode} grads, "
              f"{S.state.nruns} runs): {ms:.3f} ms/step, {K_ * 1e3 / ms:.0f} chain-steps/s; "
              f"update {ums:.4f} ms ({gbs:.0f} GB/s over {S.state.n} elements)", flush=True)
        del S, grads
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
