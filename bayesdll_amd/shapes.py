"""Parameter segment tables of the reference's backbones (shape/order contract).

networks/__init__.py:9-63 builds mlp_mnist (networks/small_nets.py), resnet101
and vit_l_32 (torchvision) and sets `readout_name`; the sampler only depends on
the resulting `named_parameters()` order, shapes, 'bias' names and readout —
which these tables reproduce without torchvision (not installed here):

    mlp_mnist          8 tensors   2,797,010 params   readout 'classifier'
    resnet101 (C=1000) 314 tensors 44,549,160 params  readout 'fc'
    vit_l_32  (C=1000) 296 tensors 306,535,400 params readout 'heads.head'
"""
from __future__ import annotations

import numpy as np


def mlp_mnist(num_classes=10, width=1000, depth=3, input_dim=784):
    segs, hin = [], input_dim
    for i in range(depth):
        segs += [(f"layers.{2 * i}.weight", (width, hin)), (f"layers.{2 * i}.bias", (width,))]
        hin = width
    segs += [("classifier.weight", (num_classes, width)), ("classifier.bias", (num_classes,))]
    return segs, "classifier"


def resnet101(num_classes=1000):
    segs = [("conv1.weight", (64, 3, 7, 7)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    inplanes = 64
    for li, (planes, blocks) in enumerate([(64, 3), (128, 4), (256, 23), (512, 3)], start=1):
        for b in range(blocks):
            pre = f"layer{li}.{b}."
            segs += [(pre + "conv1.weight", (planes, inplanes, 1, 1)),
                     (pre + "bn1.weight", (planes,)), (pre + "bn1.bias", (planes,)),
                     (pre + "conv2.weight", (planes, planes, 3, 3)),
                     (pre + "bn2.weight", (planes,)), (pre + "bn2.bias", (planes,)),
                     (pre + "conv3.weight", (planes * 4, planes, 1, 1)),
                     (pre + "bn3.weight", (planes * 4,)), (pre + "bn3.bias", (planes * 4,))]
            if b == 0:
                segs += [(pre + "downsample.0.weight", (planes * 4, inplanes, 1, 1)),
                         (pre + "downsample.1.weight", (planes * 4,)),
                         (pre + "downsample.1.bias", (planes * 4,))]
            inplanes = planes * 4
    segs += [("fc.weight", (num_classes, 2048)), ("fc.bias", (num_classes,))]
    return segs, "fc"


def vit_l_32(num_classes=1000, hidden=1024, mlp=4096, layers=24, patch=32, image=224):
    seq = (image // patch) ** 2 + 1
    segs = [("class_token", (1, 1, hidden)), ("conv_proj.weight", (hidden, 3, patch, patch)),
            ("conv_proj.bias", (hidden,)), ("encoder.pos_embedding", (1, seq, hidden))]
    for i in range(layers):
        pre = f"encoder.layers.encoder_layer_{i}."
        segs += [(pre + "ln_1.weight", (hidden,)), (pre + "ln_1.bias", (hidden,)),
                 (pre + "self_attention.in_proj_weight", (3 * hidden, hidden)),
                 (pre + "self_attention.in_proj_bias", (3 * hidden,)),
                 (pre + "self_attention.out_proj.weight", (hidden, hidden)),
                 (pre + "self_attention.out_proj.bias", (hidden,)),
                 (pre + "ln_2.weight", (hidden,)), (pre + "ln_2.bias", (hidden,)),
                 (pre + "mlp.0.weight", (mlp, hidden)), (pre + "mlp.0.bias", (mlp,)),
                 (pre + "mlp.3.weight", (hidden, mlp)), (pre + "mlp.3.bias", (hidden,))]
    segs += [("encoder.ln.weight", (hidden,)), ("encoder.ln.bias", (hidden,)),
             ("heads.head.weight", (num_classes, hidden)), ("heads.head.bias", (num_classes,))]
    return segs, "heads.head"


BACKBONES = {"mlp_mnist": mlp_mnist, "resnet101": resnet101, "vit_l_32": vit_l_32}


def segments(backbone, num_classes=None):
    fn = BACKBONES[backbone]
    return fn() if num_classes is None else fn(num_classes)


def numel(segs):
    return int(sum(int(np.prod(s)) for _, s in segs))
