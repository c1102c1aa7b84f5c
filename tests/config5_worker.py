"""One chain of config 5 (ViT-L/32 cSGHMC, independent chains, cross-chain
posterior-predictive all-reduce) at full model size — TEST INFRASTRUCTURE for
tests/test_gpu_config5.py.

`run_chain(chain)` trains one cSGHMC chain with the product Runner
(bayesdll_amd.csghmc: fused HIP step, Philox noise, per-cycle Welford,
cycle-end likelihoods, mixture evaluation with posterior draws) on the
random-init ViT-L/32 (306,535,400 parameters, 296 tensors) and synthetic
224 x 224 batches.  Run as a script under a torch.distributed environment
every process is one chain (chain id = rank) and Runner.evaluate averages the
predictive across the chains with bayesdll_amd.chains; the ranks share the
box's one GPU over gloo (RCCL needs one GPU per rank); with --chain K the
process samples chain K alone.  The full theta does not travel: the worker returns exact checksums of it (float64 sum, the int64 sum of
its bit patterns) and a strided subsample.
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

BASE_SEED = 5
NUM_CLASSES = 1000
HPARAMS = dict(prior_sig=1.0, bias="informative", momentum_decay=0.1, Ninflate=1.0,
               nd=1.0, burnin=0, thin=1, nst=2)


def _images(seed, n, batch, device):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, 224, 224, generator=g)
    y = torch.randint(0, NUM_CLASSES, (n,), generator=g)
    return [(x[i:i + batch].to(device), y[i:i + batch].to(device)) for i in range(0, n, batch)]


def theta_digest(theta):
    """Exact, order-independent checksums of a flat fp32 vector on its device."""
    bits = theta.view(torch.int32).to(torch.int64)
    return (np.float64(theta.double().sum().item()), np.int64(bits.sum().item()),
            theta[::4099].detach().cpu().numpy())


class deterministic_autograd:
    """The reference demos' determinism (demo_mnist.py:74 sets
    cudnn.deterministic) plus the math attention backend, and MIOpen off for
    the one convolution (ViT-L/32's 32x32 / stride-32 patch embedding): with
    cudnn.deterministic MIOpen still picks its solver per process — the lone
    chain-7 process ran the patch conv as `naive_conv_ab_nonpacked_fwd_nchw` /
    `_wrw_nchw`, ensemble rank 7 as `Im2d2Col_v2` + Tensile GEMMs
    (profiles/round4/config5_trace/diff.json, tools/config5_trace.py) — so
    the gradients' low bits depended on the process, which would hide whether
    the SAMPLER couples chains.  torch's own convolution (im2col + GEMM) picks
    its kernels from the shapes alone.  Restores the previous settings on exit
    (the test process runs others)."""

    def __enter__(self):
        b = torch.backends
        self.saved = (b.cudnn.deterministic, b.cudnn.benchmark, b.cuda.flash_sdp_enabled(),
                      b.cuda.mem_efficient_sdp_enabled(), b.cudnn.enabled)
        b.cudnn.deterministic, b.cudnn.benchmark = True, False
        b.cudnn.enabled = False
        b.cuda.enable_flash_sdp(False)
        b.cuda.enable_mem_efficient_sdp(False)
        return self

    def __exit__(self, *exc):
        b = torch.backends
        b.cudnn.deterministic, b.cudnn.benchmark = self.saved[0], self.saved[1]
        b.cuda.enable_flash_sdp(self.saved[2])
        b.cuda.enable_mem_efficient_sdp(self.saved[3])
        b.cudnn.enabled = self.saved[4]


def run_chain(chain=None):
    with deterministic_autograd():
        return _run_chain(chain)


def _run_chain(chain=None):
    import bayesdll_amd.csghmc as csghmc
    from bayesdll_amd.backbones import backbone
    dev = "cuda"
    torch.manual_seed(0)  # the same random-init network on every chain
    net = backbone("vit_l_32", NUM_CLASSES).to(dev)
    train = _images(11, 8, 4, dev)
    test = _images(12, 4, 4, dev)
    args = SimpleNamespace(device=dev, ND=8, pretrained=None, lr=1e-6, lr_head=1e-6,
                           momentum=0.5, epochs=2, num_cycles=1, proportion_exploration=0.5,
                           full_sample=False, test_eval_freq=100, ece_num_bins=15,
                           log_dir=tempfile.mkdtemp(), num_classes=NUM_CLASSES,
                           noise_mode="philox", seed=BASE_SEED, calibration=False,
                           hparams={k: str(v) for k, v in HPARAMS.items()})
    runner = csghmc.Runner(net, None, args, logging.getLogger("config5"))
    runner.save_ckpt = lambda epoch: None  # ViT-L/32 checkpoints: GBs per chain, not under test
    if chain is not None:
        runner.model.chain = int(chain)
    runner.model.seed = BASE_SEED
    runner.train(train, None, test)
    loss, err, targets, logits, logits_all = runner.evaluate(test)
    torch.cuda.synchronize()
    s, b, sub = theta_digest(runner.model.flat.theta.detach())
    return {"chain": np.int64(runner.model.chain), "theta_sum": s, "theta_bits": b,
            "theta_sub": sub, "n": np.int64(runner.model.flat.theta.numel()),
            "loss": np.float64(loss), "err": np.float64(err), "targets": targets,
            "logits": logits, "logits_all": logits_all,
            "weights": np.array(list(runner.calculate_gmm_weights().values()), np.float64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--chain", type=int, default=None,
                    help="one process alone with this chain id (no torch.distributed)")
    a = ap.parse_args()
    if a.chain is not None:
        np.savez(a.out, **run_chain(chain=a.chain))
        return
    from bayesdll_amd import chains
    chains.init_chains(backend="gloo")
    try:
        res = run_chain()
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    np.savez(a.out, **res)


if __name__ == "__main__":
    main()
