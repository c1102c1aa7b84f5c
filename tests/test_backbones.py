"""The plain-torch backbones carry the reference's exact parameter tables."""
import pytest
import torch

from bayesdll_amd import shapes
from bayesdll_amd.backbones import backbone


@pytest.mark.parametrize("name,nc", [("mlp_mnist", None), ("resnet101", 1000), ("resnet101", 37),
                                     ("vit_l_32", 1000), ("vit_l_32", 37)])
def test_named_parameters_match_reference_table(name, nc):
    net = backbone(name, nc)
    segs, readout = shapes.segments(name, nc) if nc is not None else shapes.segments(name)
    got = [(n, tuple(p.shape)) for n, p in net.named_parameters()]
    assert got == [(n, tuple(s)) for n, s in segs]
    assert net.readout_name == readout
    assert sum(p.numel() for p in net.parameters()) == shapes.numel(segs)


def test_small_forward_shapes():
    net = backbone("mlp_mnist")
    assert net(torch.zeros(2, 1, 28, 28)).shape == (2, 10)
    vit = backbone("vit_l_32", 7)
    vit.encoder.layers = vit.encoder.layers[:1]  # one block is enough for a shape check
    assert vit(torch.zeros(1, 3, 224, 224)).shape == (1, 7)
