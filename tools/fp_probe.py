"""Which fp32 torch ops are correctly rounded on this device/CPU?  Compares
torch results with IEEE round-to-nearest references (float64 computation
rounded once to fp32 -- exact for sqrt/div/reciprocal of fp32 inputs)."""
import torch


def check(dev):
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(1 << 20, generator=g) * 4 + 1e-6).float()
    y = (torch.rand(1 << 20, generator=g) * 3 + 1e-3).float()
    xd, yd = x.double(), y.double()
    ref = {"sqrt": xd.sqrt().float(), "div": (xd / yd).float(), "recip": (1.0 / xd).float()}
    xs, ys = x.to(dev), y.to(dev)
    got = {"sqrt": xs.sqrt(), "div": xs / ys, "recip": 1.0 / xs}
    for k in ref:
        bad = (got[k].cpu() != ref[k]).sum().item()
        print(f"{dev:5s} {k:6s} mismatches vs IEEE: {bad} / {x.numel()}")


check("cpu")
if torch.cuda.is_available():
    check("cuda")
    from bayesdll_amd import kernels as K  # noqa: F401
