"""How does torch on this device divide an fp32 tensor by a Python float?
Compares x / s with x * fl32(1/fl32(s)), x * fl32(1/s) (reciprocal in double)
and the correctly rounded quotient."""
import numpy as np
import torch

for dev in (["cpu", "cuda"] if torch.cuda.is_available() else ["cpu"]):
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(1 << 20, generator=g) * 2 - 1).to(dev)
    for s in (1 - 0.9 ** 5, 1 - 0.999 ** 7, 0.64, 1840000.0, 3.3):
        q = x / s
        inv32 = float(np.float32(1.0) / np.float32(s))
        inv64 = float(np.float32(1.0 / s))
        a = x * inv32
        c = x * inv64
        exact = (x.double() / s).float()
        print(f"{dev:4s} s={s:.17g} inv32==inv64:{inv32 == inv64} "
              f"match recip32 {(q == a).float().mean().item():.4f} "
              f"recip64 {(q == c).float().mean().item():.4f} "
              f"true {(q == exact).float().mean().item():.4f}")
