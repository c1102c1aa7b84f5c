"""Checksums of the deterministic test inputs (numpy streams) and of a CPU
MLP forward/backward, to compare machines."""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests")]
from fakenet import MLP, det_normal, init_vector, synthetic_mnist  # noqa: E402


def h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()[:12]


data = synthetic_mnist(1, 512, 128)
print("data", h(torch.cat([x for x, _ in data]).numpy()), h(torch.cat([y for _, y in data]).numpy()))
print("init", h(init_vector(2, 2797010, 0.03)))
print("noise", h(det_normal(3, 17, 784000)))
print("cos", repr(np.float64(0.02) * (1 + np.cos(0.375 * np.pi)) / 2))
net = MLP()
with torch.no_grad():
    torch.nn.utils.vector_to_parameters(torch.tensor(init_vector(2, 2797010, 0.03)), net.parameters())
for th in (1, 8):
    torch.set_num_threads(th)
    net.zero_grad()
    out = net(data[0][0])
    loss = torch.nn.CrossEntropyLoss()(out, data[0][1])
    loss.backward()
    g = torch.nn.utils.parameters_to_vector([p.grad for p in net.parameters()]).numpy()
    print("threads", th, "logits", h(out.detach().numpy()), "grad", h(g), "loss", repr(loss.item()))
print(torch.__config__.show().split("\n")[:12])
