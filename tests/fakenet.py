"""Fake backbone with prescribed gradients — TEST INFRASTRUCTURE ONLY.

A `FakeNet` carries parameters with exactly the names and shapes of a segment
list (including `'bias'` names and a `readout_name`, the two things the
reference's per-tensor loop keys on: methods/csghmc.py:750-762,
methods/sgld.py:471-484).  Its forward is a custom autograd Function whose
backward returns a *prescribed* gradient for every parameter, so the sampler
update can be pinned independently of any forward/backward numerics.

The gradient for training step t is `grads_for_step(seed, t, n, scale)`: a
numpy PCG64 stream, deterministic across platforms, so the golden generator
(which runs the reference) and the tests (which run the oracle and the HIP
kernels) see bit-identical gradients without storing them.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

# Segment list used by the golden fixtures: odd sizes so that flat offsets
# are not multiples of 4 (exercises run boundaries inside float4 groups), a
# tail that is not a multiple of 4, a size-1 tensor, biases, and a readout.
TOY_SEGMENTS = [
    ("layer0.weight", (10, 25)),     # 250
    ("layer0.bias", (7,)),           # 7
    ("layer1.weight", (1027,)),      # 1027
    ("layer1.bias", (1,)),           # 1
    ("layer2.weight", (8, 8)),       # 64
    ("classifier.weight", (10, 13)), # 130
    ("classifier.bias", (10,)),      # 10
]
TOY_READOUT = "classifier"
TOY_CLASSES = 10


def numel_of(segments):
    return int(sum(int(np.prod(s)) for _, s in segments))


def grads_for_step(seed: int, step: int, n: int, scale: float) -> np.ndarray:
    rng = np.random.default_rng([int(seed), int(step)])
    return (rng.standard_normal(n, dtype=np.float32) * np.float32(scale)).astype(np.float32)


def init_vector(seed: int, n: int, scale: float) -> np.ndarray:
    rng = np.random.default_rng([int(seed), 0xA11CE])
    return (rng.standard_normal(n, dtype=np.float32) * np.float32(scale)).astype(np.float32)


class _PrescribedGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, grads, *params):
        ctx.grads = grads
        return torch.zeros(x.shape[0], TOY_CLASSES, dtype=torch.float32, device=x.device) + 0.0 * x.sum()

    @staticmethod
    def backward(ctx, gout):
        return (None, None, *[g.clone() for g in ctx.grads])


class FakeNet(nn.Module):
    """nn.Module whose named_parameters() follow `segments` in order."""

    def __init__(self, segments=TOY_SEGMENTS, readout_name=TOY_READOUT, grad_seed=1234,
                 grad_scale=0.5, init=None, grad_table=None):
        super().__init__()
        self.readout_name = readout_name
        self._segments = list(segments)
        for name, shape in self._segments:
            mod = self
            parts = name.split(".")
            for part in parts[:-1]:
                if not hasattr(mod, part):
                    mod.add_module(part, nn.Module())
                mod = getattr(mod, part)
            mod.register_parameter(parts[-1], nn.Parameter(torch.zeros(shape, dtype=torch.float32)))
        self.grad_seed = grad_seed
        self.grad_scale = grad_scale
        # optional precomputed grads_for_step vectors (index = step), e.g. on the device
        self.grad_table = grad_table
        self.step = 0
        if init is not None:
            self.load_flat(init)

    @property
    def n(self):
        return numel_of(self._segments)

    def load_flat(self, vec):
        vec = torch.tensor(np.asarray(vec, dtype=np.float32))  # copy: params become views of it
        with torch.no_grad():
            torch.nn.utils.vector_to_parameters(vec.to(next(self.parameters()).device),
                                                self.parameters())

    def forward(self, x):
        params = list(self.parameters())
        if torch.is_grad_enabled():
            if self.grad_table is not None:
                gt = self.grad_table[self.step].to(params[0].device)
            else:
                g = grads_for_step(self.grad_seed, self.step, self.n, self.grad_scale)
                gt = torch.from_numpy(g).to(params[0].device)
            self.step += 1
            grads, off = [], 0
            for p in params:
                k = p.numel()
                grads.append(gt[off:off + k].view_as(p))
                off += k
        else:
            grads = [torch.zeros_like(p) for p in params]
        return _PrescribedGrad.apply(x, grads, *params)


def fake_loader(batches: int, batch_size: int = 4, device="cpu"):
    """A list works as a loader: len() and iteration are all the Runners use."""
    x = torch.zeros(batch_size, 1, device=device)
    y = torch.zeros(batch_size, dtype=torch.long, device=device)
    return [(x, y) for _ in range(batches)]


class MLP(nn.Module):
    """mlp_mnist backbone with the reference's parameter names and shapes
    (networks/small_nets.py MLP(784, 10, width=1000, depth=3), readout
    'classifier'); written here so the GPU tests need no reference import."""

    def __init__(self, input_dim=784, output_dim=10, width=1000, depth=3):
        super().__init__()
        self.input_dim = input_dim
        layers, hin = [], input_dim
        for _ in range(depth):
            layers += [nn.Linear(hin, width), nn.ReLU()]
            hin = width
        self.layers = nn.Sequential(*layers)
        self.classifier = nn.Linear(width, output_dim)
        self.readout_name = "classifier"

    def forward(self, x):
        return self.classifier(self.layers(x.view(-1, self.input_dim)))


def det_normal(seed, k, numel):
    """Deterministic N(0,1) stream replacing torch.randn_like draw #k."""
    rng = np.random.default_rng([int(seed), 0xD4A7, int(k)])
    return rng.standard_normal(int(numel), dtype=np.float32)


def synthetic_mnist(seed, n, batch, device="cpu"):
    rng = np.random.default_rng([int(seed), 0xDA7A])
    x = torch.from_numpy(rng.standard_normal((n, 1, 28, 28), dtype=np.float32))
    y = torch.from_numpy(rng.integers(0, 10, size=n).astype(np.int64))
    return [(x[i:i + batch].to(device), y[i:i + batch].to(device)) for i in range(0, n, batch)]
