"""K chains on one GPU two ways: the reference's recipe (K processes, one
chain each — here the fused one-chain step with HIP-graph replay) vs
bayesdll_amd.stacked (one process, K stacked chains, graph replay).
Aggregate chain-steps/s; mlp_mnist, batch 128, synthetic data.

    KS=4,8 STEPS=400 python tools/stacked_vs_processes.py

The parent never touches the GPU (children are spawned, not exec'd)."""
import os
import sys
import time

import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _one_chain(rank, steps, barrier, q):
    import torch
    import bayesdll_amd.csghmc as csghmc
    from bayesdll_amd.backbones import backbone
    torch.manual_seed(rank)
    dev = "cuda"
    net = backbone("mlp_mnist", 10).to(dev)
    model = csghmc.Model(ND=60000, prior_sig=1.0, momentum_decay=0.1)
    model.graph, model.chain = True, rank
    model.defer_loss = True  # as under the Runner: no per-step host sync
    crit = torch.nn.CrossEntropyLoss()
    x = torch.randn(128, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (128,), device=dev)
    for k in range(10):
        model(x, y, net, None, crit, [1e-4, 1e-4], 1.0, 1.0, should_sample=k % 10 == 0)
    torch.cuda.synchronize()
    barrier.wait()
    t0 = time.perf_counter()
    for k in range(steps):
        model(x, y, net, None, crit, [1e-4, 1e-4], 1.0, 1.0, should_sample=k % 10 == 0)
    torch.cuda.synchronize()
    q.put((t0, time.perf_counter()))


def _stacked(K, steps, q):
    from types import SimpleNamespace

    import torch
    from bayesdll_amd import stacked
    from bayesdll_amd.backbones import backbone
    dev = "cuda"
    args = SimpleNamespace(lr=1e-4, lr_head=1e-4, epochs=1, num_cycles=1,
                           proportion_exploration=0.5, ND=60000, device=dev, seed=0,
                           hparams={"prior_sig": 1.0, "momentum_decay": 0.1, "Ninflate": 1.0,
                                    "nd": 1.0, "thin": 1, "nst": 0, "bias": "informative"})
    S = stacked.StackedCSGHMC(backbone("mlp_mnist", 10).to(dev), K, args, init="reinit",
                              graph=True)
    x = torch.randn(128, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (128,), device=dev)
    for k in range(10):
        S.step(x, y, 1e-4, should_sample=k % 10 == 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        S.step(x, y, 1e-4, should_sample=k % 10 == 0)
    torch.cuda.synchronize()
    q.put((t0, time.perf_counter()))


def main():
    ks = [int(k) for k in os.environ.get("KS", "4,8").split(",")]
    steps = int(os.environ.get("STEPS", "400"))
    ctx = mp.get_context("spawn")
    for K in ks:
        q, barrier = ctx.Queue(), ctx.Barrier(K)
        ps = [ctx.Process(target=_one_chain, args=(r, steps, barrier, q)) for r in range(K)]
        for p in ps:
            p.start()
        spans = [q.get(timeout=300) for _ in range(K)]
        for p in ps:
            p.join(timeout=60)
        wall = max(b for _, b in spans) - min(a for a, _ in spans)
        print(f"mlp_mnist batch 128: {K} processes x 1 chain (fused + graph): "
              f"{K * steps / wall:.0f} chain-steps/s aggregate", flush=True)
        q = ctx.Queue()
        p = ctx.Process(target=_stacked, args=(K, steps, q))
        p.start()
        a, b = q.get(timeout=300)
        p.join(timeout=60)
        print(f"mlp_mnist batch 128: 1 process x {K} stacked chains (graph): "
              f"{K * steps / (b - a):.0f} chain-steps/s", flush=True)


if __name__ == "__main__":
    main()
