"""Command-line driver for the fused SG-MCMC samplers with the reference's flag
and hparams surface (demo_mnist.py / demo_vision.py: --method, --hparams
"k=v,k=v", --epochs, --batch_size, --lr, --lr_head, --momentum, --num_cycles,
--proportion_exploration, --val_heldout, --seed, --log_dir, ...).

    python -m bayesdll_amd.run --method sgld --dataset mnist --backbone mlp_mnist \
        --hparams prior_sig=1.0,Ninflate=1e3,nd=1.0,burnin=5,thin=10,bias=informative,nst=5 \
        --lr 1e-2 --momentum 0.5
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m bayesdll_amd.run --method csghmc --dataset pets --backbone vit_l_32 ...

Differences, all forced by the environment rather than chosen: the datasets
are synthetic tensors of the real datasets' shapes and split sizes (there is
no network for downloads, datasets.py:26-43); --pretrained takes a local
state_dict file loaded with weights_only=True (no URL fetch,
networks/__init__.py:66-130); wandb is not available.  Only the SG-MCMC
methods exist here (the VI / MC-dropout / Laplace / vanilla families are not
part of this framework).  With several processes (torch.distributed.run),
each rank samples its own chain (seed + rank) and evaluation averages the
posterior predictive across chains.
"""
from __future__ import annotations

import argparse
import importlib
import logging
import os
import sys
from datetime import datetime

import numpy as np
import torch

METHODS = ("sgld", "csgld", "sghmc", "csghmc", "csghmc_fs", "adam_sghmc", "adam_csghmc")

# (input shape, classes, train-set size, test-set size) of the reference's datasets
DATASETS = {
    "mnist": ((1, 28, 28), 10, 60000, 10000),
    "pets": ((3, 224, 224), 37, 3680, 3669),
    "imagenet": ((3, 224, 224), 1000, 1281167, 50000),
    "cifar100": ((3, 32, 32), 100, 50000, 10000),
    "cifar10": ((3, 32, 32), 10, 50000, 10000),
}


# pretrain_resnet101.py:122-134 defaults, used when --hparams is empty
DEFAULT_HPARAMS = {
    "csgld": "prior_sig=1.0,Ninflate=1.0,nd=0.01,burnin=50,thin=10,bias=informative,nst=5,temp=1.0",
    "sgld": "prior_sig=1.0,Ninflate=1e3,nd=1.0,burnin=50,thin=10,bias=informative,nst=5,temp=1.0",
    "csghmc": "prior_sig=1.0,Ninflate=1.0,nd=0.01,burnin=50,momentum_decay=0.18,thin=10,"
              "bias=informative,nst=5,temp=1.0",
    "sghmc": "prior_sig=1.0,Ninflate=1e3,nd=1.0,burnin=5,momentum_decay=0.18,thin=1,"
             "bias=informative,nst=5,temp=1.0",
    "adam_sghmc": "prior_sig=1.0,Ninflate=1e3,nd=1.0,momentum_decay=0.05,burnin=50,thin=10,"
                  "bias=informative,nst=5,temp=1.0,beta1=0.9,beta2=0.999",
}
DEFAULT_HPARAMS["csghmc_fs"] = DEFAULT_HPARAMS["csghmc"]
DEFAULT_HPARAMS["adam_csghmc"] = DEFAULT_HPARAMS["adam_sghmc"]


def parse_hparams(s):
    """demo_mnist.py:77-86: strip quotes, split on ',', keep 'k=v' items, values
    stay strings; also returns the directory tag (',' -> '_')."""
    s = s.replace('"', "")
    tag = s.replace(",", "_")
    out = {}
    for opt in s.split(","):
        if "=" in opt:
            k, v = opt.split("=")
            out[k] = v
    return out, tag


def build_parser():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--method", type=str, default="csghmc", choices=METHODS)
    ap.add_argument("--hparams", type=str, default="")
    ap.add_argument("--pretrained", type=str, default=None,
                    help="local state_dict file of the backbone (prior mean net0)")
    ap.add_argument("--dataset", type=str, default="mnist", choices=sorted(DATASETS))
    ap.add_argument("--backbone", type=str, default="mlp_mnist",
                    choices=["mlp_mnist", "resnet101", "vit_l_32"])
    ap.add_argument("--val_heldout", type=float, default=0.1)
    ap.add_argument("--ece_num_bins", type=int, default=15)
    ap.add_argument("--num_cycles", type=int, default=1)
    ap.add_argument("--proportion_exploration", type=float, default=0.5)
    ap.add_argument("--full_sample", type=bool, default=False)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--lr_head", type=float, default=None)
    ap.add_argument("--momentum", type=float, default=0.5)
    ap.add_argument("--clip_grad", type=float, default=None)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--log_dir", type=str, default="results")
    ap.add_argument("--test_eval_freq", type=int, default=1)
    # synthetic data (the reference downloads the real sets)
    ap.add_argument("--train_size", type=int, default=None,
                    help="synthetic training examples (default: the dataset's size)")
    ap.add_argument("--test_size", type=int, default=None)
    # MI355X path options
    ap.add_argument("--noise_mode", type=str, default="philox", choices=["philox", "torch"])
    ap.add_argument("--graph", action="store_true", help="replay forward/backward from a HIP graph")
    ap.add_argument("--overlap", action="store_true",
                    help="overlap the fused update with backward, bucket by bucket (cSGHMC)")
    ap.add_argument("--resume_state", action="store_true",
                    help="checkpoints carry what an exact resume needs")
    ap.add_argument("--stacked_chains", type=int, default=0,
                    help="csghmc / sghmc / sgld / csgld: K > 0 chains per device stepped together "
                         "(bayesdll_amd.stacked; no BatchNorm statistics)")
    return ap


class SyntheticLoader:
    """Batches of N(0,1) inputs and uniform labels of a dataset's shape,
    generated on the device from a fixed seed (the same batches every epoch,
    like iterating a fixed dataset without shuffling)."""

    def __init__(self, n, shape, classes, batch_size, device, seed):
        self.n, self.shape, self.classes, self.bs = int(n), tuple(shape), classes, batch_size
        self.device, self.seed = device, seed

    def __len__(self):
        return (self.n + self.bs - 1) // self.bs

    def __iter__(self):
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        for i in range(0, self.n, self.bs):
            b = min(self.bs, self.n - i)
            x = torch.randn((b,) + self.shape, device=self.device, generator=g)
            y = torch.randint(0, self.classes, (b,), device=self.device, generator=g)
            yield x, y


def prepare(args, device):
    """datasets.prepare's split arithmetic (val_heldout carved from train)
    over synthetic tensors; returns loaders and ND = train-set size."""
    shape, classes, ntrain, ntest = DATASETS[args.dataset]
    ntrain = args.train_size if args.train_size is not None else ntrain
    ntest = args.test_size if args.test_size is not None else ntest
    nval = int(args.val_heldout * ntrain) if args.val_heldout > 0 else 0
    ntr = ntrain - nval
    args.num_classes = classes
    mk = lambda n, s: SyntheticLoader(n, shape, classes, args.batch_size, device, s)  # noqa: E731
    return mk(ntr, args.seed), (mk(nval, args.seed + 1) if nval else None), \
        mk(ntest, args.seed + 2), ntr


def main(argv=None):
    args = build_parser().parse_args(argv)
    from . import chains
    rank, world, device = chains.init_chains()
    if device.type != "cuda":
        raise RuntimeError("bayesdll_amd.run needs a HIP device (the samplers have no CPU path)")
    args.device = device
    seed = chains.chain_seed(args.seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    np.random.seed(seed)
    args.hparams, hpstr = parse_hparams(args.hparams or DEFAULT_HPARAMS[args.method])
    if args.lr_head is None:
        args.lr_head = args.lr
    args.seed = seed
    pretr = 1 if args.pretrained is not None else 0
    main_dir = (f"{args.dataset}_val_heldout{args.val_heldout}/{args.backbone}/"
                f"{args.method}_{hpstr}_pretr{pretr}/ep{args.epochs}_bs{args.batch_size}_"
                f"lr{args.lr}_lrh{args.lr_head}_mo{args.momentum}/seed{args.seed}_"
                + datetime.now().strftime("%Y_%m%d_%H%M%S"))
    args.log_dir = os.path.join(args.log_dir, main_dir)
    os.makedirs(args.log_dir, exist_ok=True)
    logging.basicConfig(handlers=[logging.FileHandler(os.path.join(args.log_dir, "logs.txt")),
                                  logging.StreamHandler()],
                        format="[%(asctime)s,%(msecs)03d %(levelname)s] %(message)s",
                        datefmt="%H:%M:%S", level=logging.INFO, force=True)
    logger = logging.getLogger()
    logger.info(f"Command :: {' '.join(sys.argv)}  (chain {rank} of {world})\n")

    train_loader, val_loader, test_loader, args.ND = prepare(args, device)
    from .backbones import create_backbone
    net = create_backbone(args)
    logger.info("Total params in the backbone: %.2fM"
                % (sum(p.numel() for p in net.parameters()) / 1e6))
    net0 = None
    if args.pretrained is not None:
        # feat-ext params = pretrained; net0 with a zero head, net with a random head
        state = torch.load(args.pretrained, map_location="cpu", weights_only=True)
        net0 = create_backbone(args)
        for m in (net, net0):
            own = m.state_dict()
            # networks/__init__.py:66-130: feature extractor from the file; the
            # readout stays as created (random in net, zeroed in net0 below)
            m.load_state_dict({k: v for k, v in state.items()
                               if k in own and own[k].shape == v.shape
                               and not k.startswith(m.readout_name + ".")}, strict=False)
        with torch.no_grad():
            for nm, p in net0.named_parameters():
                if net0.readout_name in nm:
                    p.zero_()
        net0 = net0.to(device)
    net = net.to(device)

    if args.stacked_chains > 0:
        from . import stacked
        cls = {"csghmc": stacked.StackedCSGHMC, "sgld": stacked.StackedSGLD,
               "csgld": stacked.StackedCSGLD, "sghmc": stacked.StackedSGHMC}.get(args.method)
        if cls is None:
            raise ValueError("--stacked_chains: csghmc, sghmc, sgld or csgld")
        S = cls(net, args.stacked_chains, args, logger=logger, init="reinit", graph=args.graph,
                net0=net0)
        logger.info(f"{args.stacked_chains} stacked chains on this device "
                    f"(chain ids {S.chain0}..{S.chain0 + S.K - 1})")
        return S.train(train_loader, test_loader)
    runner_cls = importlib.import_module(f"bayesdll_amd.{args.method}").Runner
    runner = runner_cls(net, net0, args, logger)
    return runner.train(train_loader, val_loader, test_loader)


if __name__ == "__main__":
    main()
