"""One chain of the multi-chain ensemble (config 5's logic at mlp size) —
TEST INFRASTRUCTURE for tests/test_gpu_chains.py.

`run_chain(method, chain)` trains one chain with the product Runner
(bayesdll_amd.csghmc / .sgld, Philox noise, fused HIP step) on synthetic
MNIST-shaped data and evaluates it.  Run as a script under a torch.distributed
environment (RANK / WORLD_SIZE / MASTER_*), every process is one chain and
`Runner.evaluate` averages the posterior predictive across chains with the
one all_reduce of bayesdll_amd.chains; run in a single process with an
explicit chain id it gives that chain alone, so the test can rebuild the
ensemble by hand.  Results go to an .npz.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
import tempfile
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.dirname(HERE), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

from fakenet import MLP, synthetic_mnist  # noqa: E402

HPARAMS = {
    # config 2 (cSGHMC, pretrain_resnet101.py:127) with a short run
    "csghmc": dict(prior_sig=1.0, bias="informative", momentum_decay=0.18, Ninflate=1.0,
                   nd=0.01, burnin=0, thin=1, nst=3),
    # config 1 (SGLD, README.md:83) with a short burn-in
    "sgld": dict(prior_sig=1.0, bias="informative", Ninflate=1e3, nd=1.0, burnin=1, thin=2,
                 nst=3),
}
BASE_SEED = 77  # the same Philox seed on every chain: chains differ by chain id only


def run_chain(method, chain=None, replica=False):
    """Train + evaluate one chain on cuda (the current device).  chain=None:
    the chain id is the process rank (bayesdll_amd.chains).  replica=True
    (cyclical methods, under torch.distributed): every rank runs the SAME
    chain (chain id 0), then the cycle-end likelihood pass is run sharded
    over the ranks and locally, the sharded pass is refused for ranks whose
    moments differ, and evaluate() runs with GMM weights over chains."""
    import bayesdll_amd.csghmc as csghmc
    import bayesdll_amd.sgld as sgld
    dev = "cuda"
    torch.manual_seed(0)
    net = MLP(width=128).to(dev)
    train = synthetic_mnist(11, 384, 64, device=dev)
    test = synthetic_mnist(12, 128, 64, device=dev)
    args = SimpleNamespace(device=dev, ND=384, pretrained=None, lr=1e-2, lr_head=1e-2,
                           momentum=0.5, epochs=4, num_cycles=2, proportion_exploration=0.5,
                           full_sample=False, test_eval_freq=100, ece_num_bins=15,
                           log_dir=tempfile.mkdtemp(), num_classes=10, noise_mode="philox",
                           seed=BASE_SEED,
                           hparams={k: str(v) for k, v in HPARAMS[method].items()})
    mod = {"csghmc": csghmc, "sgld": sgld}[method]
    runner = mod.Runner(net, None, args, logging.getLogger("chain"))
    if chain is not None:
        runner.model.chain = int(chain)
    if replica:
        runner.model.chain = 0
    runner.model.seed = BASE_SEED
    runner.train(train, None, test)
    extra = {}
    if method == "csghmc":
        extra["lik_local"] = np.array(runner.full_batch_likelihoods(train))
    if replica:
        import torch.distributed as dist
        from bayesdll_amd import chains
        extra["lik_shard"] = np.array(runner.full_batch_likelihoods(train,
                                                                    group=dist.group.WORLD))
        c = runner.current_cycle
        saved = runner.cycle_theta_mom1[c]
        runner.cycle_theta_mom1[c] = saved + (1e-3 if chains.rank() == 1 else 0.0)
        try:
            runner.full_batch_likelihoods(train, group=dist.group.WORLD)
            extra["mismatch_refused"] = np.bool_(False)
        except ValueError:
            extra["mismatch_refused"] = np.bool_(True)
        runner.cycle_theta_mom1[c] = saved
        runner.gmm_over_chains = True
        extra["logits_gmm_over_chains"] = runner.evaluate(test)[3]
        runner.gmm_over_chains = False
    loss, err, targets, logits, logits_all = runner.evaluate(test)
    torch.cuda.synchronize()
    return {**extra, "log_dir": np.array(runner.args.log_dir),
            "theta": runner.model.flat.theta.detach().cpu().numpy(),
            "chain": np.int64(runner.model.chain), "loss": np.float64(loss),
            "err": np.float64(err), "targets": targets, "logits": logits,
            "logits_all": logits_all}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", required=True, choices=sorted(HPARAMS))
    ap.add_argument("--out", required=True)
    ap.add_argument("--replica", action="store_true")
    ap.add_argument("--chain", type=int, default=None,
                    help="one process alone with this chain id (no torch.distributed)")
    a = ap.parse_args()
    if a.chain is not None:
        np.savez(a.out, **run_chain(a.method, chain=a.chain))
        return
    from bayesdll_amd import chains
    chains.init_chains(backend="gloo")  # ranks share one GPU here; RCCL needs one GPU per rank
    try:
        res = run_chain(a.method, replica=a.replica)
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    np.savez(a.out, **res)


if __name__ == "__main__":
    main()
