"""What physical-chunk placement costs and buys on the Runner path (ViT-L/32
cSGHMC, random init, synthetic [16,3,224,224] batch), with and without it
(BDL_PLACEMENT=search vs 0), each mode in its own fresh process:

  * first-step seconds: the first Model.forward builds the flat state, runs the
    autotuner and the placement search (eager and graph models separately);
  * peak transient HBM over that first step (device free memory sampled every
    ~2 ms from a thread), and the steady footprint after it;
  * e2e ms/step, eager and HIP-graph (fwd + bwd + fused update, per-step
    loss.item() as in the reference), and the fused update's sampled kernel
    time (BDL_STEP_TIMING).

    python tools/placement_cost.py          # both modes, one JSON line each
"""
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FreeSampler:
    def __init__(self, dev):
        import torch
        self.torch, self.dev, self.low, self.stop = torch, dev, None, False
        self.t = threading.Thread(target=self.run, daemon=True)

    def run(self):
        while not self.stop:
            f, _ = self.torch.cuda.mem_get_info(self.dev)
            self.low = f if self.low is None else min(self.low, f)
            time.sleep(0.002)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *a):
        self.stop = True
        self.t.join()


def one_mode(steps):
    import torch
    sys.path.insert(0, ROOT)
    import bayesdll_amd.csghmc as csghmc
    from bayesdll_amd.backbones import backbone
    dev = torch.device("cuda", 0)
    out = {"placement": os.environ.get("BDL_PLACEMENT", "search")}
    crit = torch.nn.CrossEntropyLoss()
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(16, 3, 224, 224, device=dev, generator=g)
    y = torch.randint(0, 1000, (16,), device=dev, generator=g)
    for graph in (False, True):
        tag = "graph" if graph else "eager"
        torch.manual_seed(0)
        net = backbone("vit_l_32", 1000).to(dev)
        model = csghmc.Model(ND=1840, prior_sig=1.0, momentum_decay=0.18)
        model.noise_mode = "philox"
        model.graph = graph
        torch.cuda.synchronize()
        free0, total = torch.cuda.mem_get_info(dev)
        with FreeSampler(dev) as fs:
            t0 = time.perf_counter()
            model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=True)
            torch.cuda.synchronize()
            first = time.perf_counter() - t0
        free1, _ = torch.cuda.mem_get_info(dev)
        for k in range(3):
            model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=(k % 2 == 0))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=(k % 10 == 0))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        st = model.flat
        timer = getattr(st, "timer", None)
        pinfo = dict(st.placement_info or {})
        out[tag] = {"first_step_s": round(first, 3),
                    "peak_transient_gb": round((free0 - fs.low) / 2**30, 2),
                    "footprint_after_gb": round((free0 - free1) / 2**30, 2),
                    "ms_per_step": round(ms, 3),
                    "update": timer.summary() if timer is not None else None,
                    "placement_kept": pinfo.get("kept"), "placement_s": pinfo.get("seconds"),
                    "placement_chosen_ms": pinfo.get("chosen_ms"),
                    "placement_transient_gb": pinfo.get("transient_gb")}
        del net, model, st
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    out["device"] = torch.cuda.get_device_name(0)
    print(json.dumps(out), flush=True)


def main():
    if os.environ.get("_PC_CHILD"):
        one_mode(int(os.environ.get("STEPS", "30")))
        return
    order = os.environ.get("MODES", "search,0,search,0").split(",")
    for m in order:
        env = dict(os.environ, _PC_CHILD="1", BDL_PLACEMENT=m, BDL_STEP_TIMING="1")
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, timeout=600)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
