"""Wall time per step of a whole Runner epoch (mlp_mnist, synthetic MNIST
batches on the device): per-step loss.item() (the reference's host sync,
BDL_SYNC_LOSS=1) vs losses summed on the device, eager and HIP-graph.

    METHOD=csghmc STEPS=200 python tools/runner_epoch_time.py
"""
import importlib
import logging
import os
import sys
import time
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bayesdll_amd.backbones import backbone  # noqa: E402
from bayesdll_amd.run import DEFAULT_HPARAMS, SyntheticLoader, parse_hparams  # noqa: E402


def main():
    method = os.environ.get("METHOD", "csghmc")
    steps = int(os.environ.get("STEPS", "200"))
    bs = 128
    dev = torch.device("cuda", 0)
    log = logging.getLogger("epoch_time")
    log.addHandler(logging.NullHandler())
    loader = SyntheticLoader(steps * bs, (1, 28, 28), 10, bs, dev, 0)
    modes = [(g, s) for g in (False, True) for s in ("1", "0")]
    if os.environ.get("PROFILE"):  # cProfile of one graph-mode epoch (host hot spots)
        modes = [(True, "0")]
    for graph, sync in modes:
        if True:
            os.environ["BDL_SYNC_LOSS"] = sync
            torch.manual_seed(0)
            hp, _ = parse_hparams(DEFAULT_HPARAMS[method])
            args = SimpleNamespace(
                lr=1e-3, lr_head=1e-3, epochs=100, num_cycles=50, proportion_exploration=0.5,
                ND=steps * bs, device=dev, seed=0, hparams=hp, pretrained=None, graph=graph,
                log_dir=os.path.join("gpurun_out", "epoch_time"), num_classes=10,
                ece_num_bins=15, momentum=0.5, clip_grad=None, test_eval_freq=1000)
            os.makedirs(args.log_dir, exist_ok=True)
            net = backbone("mlp_mnist", 10).to(dev)
            R = importlib.import_module(f"bayesdll_amd.{method}").Runner(net, None, args, log)
            one = (lambda: R.train_one_epoch(loader)) if method in ("csghmc", "csgld") else \
                (lambda: R.train_one_epoch(loader, False, 0))
            one()  # placement, capture, warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if os.environ.get("PROFILE"):
                import cProfile
                import pstats
                pr = cProfile.Profile()
                pr.enable()
                res = one()
                torch.cuda.synchronize()
                pr.disable()
                pstats.Stats(pr).sort_stats("tottime").print_stats(30)
            else:
                res = one()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            print(f"{method} mlp_mnist batch {bs}: graph={int(graph)} per-step loss sync={sync}: "
                  f"{ms:.3f} ms/step (epoch loss {res[0]:.6f})", flush=True)


if __name__ == "__main__":
    main()
