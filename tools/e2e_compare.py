"""End-to-end cSGHMC step (BACKBONE = mlp_mnist: BASELINE config 2,
vit_l_32: config 4, resnet101): the fused kernel vs the reference's
per-tensor torch-op update (methods/csghmc.py:747-778 as written, running on
the same GPU), whole steps (forward + backward + update + loss.item()) and
the update alone.  Informational; not the bench metric.  One JSON line.
Restored in round 6 from d6fb22c (round 1) to refresh those numbers."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesdll_amd.csghmc as csghmc  # noqa: E402
from bayesdll_amd.backbones import backbone  # noqa: E402


def reference_update(net, moms, lrs, prior_sig, alpha, N, nd, should_sample):
    """methods/csghmc.py:747-778, per tensor, torch ops (the reference on a GPU)."""
    with torch.no_grad():
        for (pname, p) in net.named_parameters():
            lr = lrs[1] if net.readout_name in pname else lrs[0]
            v = moms[pname]
            grad_u = p.grad + prior_sig * p.data
            noise = nd * np.sqrt((2 * alpha * lr)) / N * torch.randn_like(p)
            v = v * (1 - alpha) - lr * grad_u + (noise if should_sample else 0)
            moms[pname] = v
            p.data.add_(v)


def main():
    name = os.environ.get("BACKBONE", "vit_l_32")
    batch = int(os.environ.get("BATCH", "16"))
    steps = int(os.environ.get("STEPS", "10"))
    dev = "cuda"
    classes = 10 if name == "mlp_mnist" else 1000
    shape = (batch, 1, 28, 28) if name == "mlp_mnist" else (batch, 3, 224, 224)
    x = torch.randn(*shape, device=dev)
    y = torch.randint(0, classes, (batch,), device=dev)
    crit = torch.nn.CrossEntropyLoss()
    lrs = [1e-4, 1e-2]
    res = {}
    for mode in ("reference_torch_ops", "fused", "fused_graph"):
        torch.manual_seed(0)
        net = backbone(name, classes).to(dev)
        model = csghmc.Model(ND=1840, prior_sig=1.0, momentum_decay=0.18)
        model.noise_mode = "philox"
        model.graph = mode == "fused_graph"  # forward + backward from a captured HIP graph
        model.overlap = mode == "fused_overlap"  # update per bucket, overlapping backward
        moms = {n: torch.zeros_like(p) for n, p in net.named_parameters()}
        fwdbwd = upd = 0.0
        for k in range(steps + 3):
            if k == 3:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            ss = k % 10 == 0
            if mode.startswith("fused"):
                model(x, y, net, None, crit, lrs, 1.0, 0.01, should_sample=ss)
            else:
                out = net(x)
                loss = crit(out, y)
                net.zero_grad()
                loss.backward()
                reference_update(net, moms, lrs, 1.0, 0.18, 1840.0, 0.01, ss)
                loss.item()
        torch.cuda.synchronize()
        res[mode] = (time.perf_counter() - t0) / steps * 1e3
        # update-only timing
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if mode in ("fused_graph", "fused_overlap"):
            pass
        elif mode == "fused":
            from bayesdll_amd import _lib as L
            from bayesdll_amd import kernels as K
            st = model.flat
            e0.record()
            h0 = time.perf_counter()
            for _ in range(steps):
                K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=(1e-7, 1e-6),
                              noise_mode=L.NOISE_PHILOX, one_minus_alpha=0.82, prior_sig=1.0)
            res["fused_host_ms_per_call"] = (time.perf_counter() - h0) / steps * 1e6 * 1e-3
            e1.record()
        else:
            e0.record()
            for _ in range(steps):
                reference_update(net, moms, lrs, 1.0, 0.18, 1840.0, 0.01, True)
            e1.record()
        torch.cuda.synchronize()
        if mode not in ("fused_graph", "fused_overlap"):
            res[mode + "_update_only"] = e0.elapsed_time(e1) / steps
        del net, model, moms
        torch.cuda.empty_cache()
    res = {k: round(v, 4) for k, v in res.items()}
    res["speedup_step"] = round(res["reference_torch_ops"] / res["fused"], 2)
    res["speedup_update"] = round(res["reference_torch_ops_update_only"] /
                                  res["fused_update_only"], 1)
    print(json.dumps({"backbone": name, "batch": batch, "steps": steps, "ms": res,
                      "device": torch.cuda.get_device_name(0)}))


if __name__ == "__main__":
    main()
