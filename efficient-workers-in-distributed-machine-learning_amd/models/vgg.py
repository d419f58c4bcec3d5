"""CIFAR VGG family (VGG-11/13/16/19, with and without BatchNorm).

Parity: ``PyTorch-parameter-server/src/model_ops/vgg.py`` -- feature stacks of 3x3 convs from the
standard configurations A/B/D/E, a 512-512 classifier with dropout, conv weights initialised
N(0, sqrt(2/(k*k*C_out))) with zero bias (``vgg.py:31-36``).  ``vgg11_bn`` (the reference's
"VGG11", ``util.py:17-18``) has 9,756,426 parameters in 38 tensors.

Unlike the reference, every factory honours ``num_classes`` (the reference's vgg13_bn etc. ignore
it).
"""
import math

import torch
import torch.nn as nn

from . import fused
from .fused import FusedFeatures

_CFG = {
    "A": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "B": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "D": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "E": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
          512, 512, 512, 512, "M"],
}


def _features(cfg, batch_norm: bool, in_channels: int = 3) -> nn.Sequential:
    """The conv stack; a :class:`FusedFeatures` (runs conv-BN-ReLU-pool groups through the fused
    NHWC kernels on the GPU, plain ``nn.Sequential`` semantics otherwise)."""
    layers = []
    c = in_channels
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            continue
        layers.append(nn.Conv2d(c, v, kernel_size=3, padding=1))
        if batch_norm:
            layers.append(nn.BatchNorm2d(v))
        layers.append(nn.ReLU(inplace=True))
        c = v
    return FusedFeatures(*layers)


class VGG(nn.Module):
    def __init__(self, features: nn.Module, num_classes: int = 10):
        super().__init__()
        self.features = features
        self.classifier = nn.Sequential(
            nn.Dropout(),
            nn.Linear(512, 512),
            nn.ReLU(True),
            nn.Dropout(),
            nn.Linear(512, 512),
            nn.ReLU(True),
            nn.Linear(512, num_classes),
        )
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / fan))
                m.bias.data.zero_()

    def forward(self, x):
        feat = self.features(x)
        f = feat.flatten(1)
        if fused.active(f):  # hipBLASLt GEMMs + fused activation/dropout kernels (ops/head.py)
            from ..ops.head import vgg_head

            # the last BN layer's backward may ride in the first Linear's (ops/head.py)
            return vgg_head(self.classifier, f, getattr(feat, "_ew_bn_node", None))
        return self.classifier(f)

    def fused_loss(self, x, y):
        """(mean cross-entropy, logits) with the loss riding in the last Linear's forward launch
        (``ops/head.py`` ``vgg_head_loss``; opt-in ``EWDML_HEAD_TAIL=1``: the classifier tail and
        the loss in one launch each way, ``vgg_loss``), or None where neither applies (the caller
        then runs ``forward`` and its own loss)."""
        if not (x.is_cuda and x.dtype == torch.float32 and fused.active(x)):
            return None
        from ..ops import head as head_ops

        if not head_ops._TAIL:
            if not head_ops._HEAD_CE:
                return None
            # the loss riding in the last Linear's launch (ops/head.py vgg_head_loss)
            feat = self.features(x)
            f = feat.flatten(1)
            node = getattr(feat, "_ew_bn_node", None)
            if not head_ops.head_ce_supported(self.classifier, f, y):
                from ..ops.nn import cross_entropy

                out = head_ops.vgg_head(self.classifier, f, node) if fused.active(f) else \
                    self.classifier(f)
                return cross_entropy(out, y), out.detach()
            return head_ops.vgg_head_loss(self.classifier, f, y, node)

        probe = torch.empty((x.shape[0], self.classifier[1].in_features), dtype=x.dtype,
                            device=x.device)
        if not head_ops.tail_supported(self.classifier, probe, y):
            return None
        f = self.features(x).flatten(1)
        if not head_ops.tail_supported(self.classifier, f, y):  # not expected: same checks
            from ..ops.nn import cross_entropy

            out = head_ops.vgg_head(self.classifier, f) if fused.active(f) else self.classifier(f)
            return cross_entropy(out, y), out.detach()
        return head_ops.vgg_loss(self.classifier, f, y)


def _make(cfg_key, bn, num_classes=10):
    return VGG(_features(_CFG[cfg_key], bn), num_classes=num_classes)


def vgg11(num_classes=10):
    return _make("A", False, num_classes)


def vgg11_bn(num_classes=10):
    return _make("A", True, num_classes)


def vgg13(num_classes=10):
    return _make("B", False, num_classes)


def vgg13_bn(num_classes=10):
    return _make("B", True, num_classes)


def vgg16(num_classes=10):
    return _make("D", False, num_classes)


def vgg16_bn(num_classes=10):
    return _make("D", True, num_classes)


def vgg19(num_classes=10):
    return _make("E", False, num_classes)


def vgg19_bn(num_classes=10):
    return _make("E", True, num_classes)
