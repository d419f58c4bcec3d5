"""ResNets: the CIFAR variants of the reference plus an ImageNet-stem variant.

Parity: ``PyTorch-parameter-server/src/model_ops/resnet.py`` -- BasicBlock / Bottleneck with
projection shortcuts, 3x3 stride-1 stem, 4 stages (64/128/256/512 planes).  ResNet-18 has
11,173,962 parameters (62 tensors); ResNet-50 with 10 classes has 23,520,842 (161 tensors).

Fixed reference defects:
  * every factory takes ``num_classes`` (the reference's ResNet34/50 do not);
  * the CIFAR head uses adaptive average pooling, so it still equals ``avg_pool2d(4)`` on 32x32
    inputs but no longer crashes on other resolutions;
  * ``stem="imagenet"`` gives the standard 7x7/2 conv + 3x3/2 max-pool stem used for the
    224x224 ResNet-50 config (BASELINE.json config #5).

On the GPU (``models.fused`` enabled) every BN runs through the fused NHWC kernels
(``ewdml.ops.nn.bn_act``): conv-BN-ReLU, shortcut conv-BN, and the block output
``relu(bn3(conv3) + shortcut)`` as one BN+add+ReLU kernel set; the stride-1 3x3 and 1x1
convolutions run the MFMA implicit-GEMM kernels (``ewdml.ops.conv``); same modules and state_dict.
"""
import os

import torch.nn as nn
import torch.nn.functional as F

from . import fused


def _conv(m, x):
    """``m(x)``; stride-1 3x3 / 1x1 layers on channels_last bf16 run the MFMA implicit-GEMM
    kernels (``ewdml.ops.conv``), as does the 3-channel CIFAR stem; the others (strided, the
    ImageNet 7x7/2 stem) MIOpen."""
    from ..ops.conv import conv2d_module

    return conv2d_module(m, x)


# identity-residual gradients through a GradSink (False: autograd sums them; A/B and tests)
_RESIDUAL_SINK = True
# ... for projection shortcuts too (EWDML_PROJ_SINK=0: identity shortcuts only; A/B)
_PROJ_SINK = os.environ.get("EWDML_PROJ_SINK", "1") != "0"


def set_residual_sink(on: bool):
    global _RESIDUAL_SINK
    _RESIDUAL_SINK = bool(on)


def _residual_block(x, main, bn_last, sc):
    """``relu(bn_last(main(x, sink)) + shortcut(x))`` on the fused kernels.  With an MFMA first
    conv, the shortcut's gradient of the block input is not summed by autograd: the last BN's
    backward (identity shortcut) or the projection conv's backward (through ``sink_tap``)
    deposits it in a :class:`GradSink` and the first conv's backward-data epilogue adds it (one
    launch less per block, and the block input's gradient is that conv's output alone, so the
    previous block's BN can take its backward statistics from the same epilogue)."""
    from ..ops.conv import GradSink, epilogue_fusion_ok, sink_tap
    from ..ops.nn import bn_act, kernel_path

    sink = GradSink() if (_RESIDUAL_SINK and x.requires_grad and epilogue_fusion_ok(x)) else None
    h, first_mfma = main(x, sink)
    if sink is not None and first_mfma:
        if len(sc) and _PROJ_SINK:
            return bn_act(h, bn_last, "add_relu", res=_shortcut(sc, sink_tap(x, sink)))
        if not len(sc) and kernel_path(h, bn_last, x):
            return bn_act(h, bn_last, "add_relu", res=x.detach(), res_sink=sink)
    return bn_act(h, bn_last, "add_relu", res=_shortcut(sc, x))


def _lazy_into(conv, h) -> bool:
    """Whether BN-ReLU output (of input ``h``) may stay unwritten because ``conv`` -- its only
    consumer -- runs the fp32 Winograd path, whose input transform applies the BN layer on the
    fly (as models/fused.py does for VGG), or is a 1x1 conv whose GEMM forms it in its operand
    staging (forward and weight gradient; EWDML_LAZY_BN=0: always materialise)."""
    if not fused._LAZY:
        return False
    pad = 0 if tuple(conv.kernel_size) == (1, 1) else 1
    if not (conv.stride in (1, (1, 1)) and conv.padding in (pad, (pad, pad))
            and conv.dilation in (1, (1, 1)) and conv.groups == 1):
        return False
    from ..ops import conv as conv_hip

    # the conv must also take the MFMA path at all (channels_last weight, 16-B pointers, C % 64:
    # conv2d_module's own test, on h as the stand-in of the same-shaped BN output), else it would
    # fall back to a kernel that reads the never-written activation
    return (conv_hip.enabled() and conv_hip.module_supported(conv, h)
            and conv_hip.lazy_input_ok(tuple(h.shape), h.dtype, conv.weight))


def _shortcut(sc, x):
    """Identity or projection (1x1 conv + BN, through the fused BN kernel)."""
    if len(sc) == 0:
        return x
    from ..ops.nn import bn_act

    return bn_act(_conv(sc[0], x), sc[1], "none")


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != planes * self.expansion:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, planes * self.expansion, 1, stride, bias=False),
                nn.BatchNorm2d(planes * self.expansion),
            )

    def _main(self, x, sink):
        """conv2(relu(bn1(conv1(x)))) -> (h, whether conv1 took the sink)."""
        from ..ops.conv import conv2d_module, module_supported
        from ..ops.nn import bn_act

        first = sink is not None and module_supported(self.conv1, x)
        h = conv2d_module(self.conv1, x, sink if first else None)
        out = bn_act(h, self.bn1, "relu", lazy=_lazy_into(self.conv2, h))
        return _conv(self.conv2, out), first

    def forward(self, x):
        if fused.active(x):
            return _residual_block(x, self._main, self.bn2, self.shortcut)
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return F.relu(out + self.shortcut(x))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != planes * self.expansion:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, planes * self.expansion, 1, stride, bias=False),
                nn.BatchNorm2d(planes * self.expansion),
            )

    def _main(self, x, sink):
        """conv3(relu(bn2(conv2(relu(bn1(conv1(x))))))) -> (h, whether conv1 took the sink)."""
        from ..ops.conv import conv2d_module, module_supported
        from ..ops.nn import bn_act

        first = sink is not None and module_supported(self.conv1, x)
        h = conv2d_module(self.conv1, x, sink if first else None)
        out = bn_act(h, self.bn1, "relu", lazy=_lazy_into(self.conv2, h))
        h2 = _conv(self.conv2, out)
        out = bn_act(h2, self.bn2, "relu", lazy=_lazy_into(self.conv3, h2))
        return _conv(self.conv3, out), first

    def forward(self, x):
        if fused.active(x):
            return _residual_block(x, self._main, self.bn3, self.shortcut)
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return F.relu(out + self.shortcut(x))


class ResNet(nn.Module):
    def __init__(self, block, num_blocks, num_classes=10, stem="cifar", in_channels=3):
        super().__init__()
        self.in_planes = 64
        self.stem = stem
        if stem == "cifar":
            self.conv1 = nn.Conv2d(in_channels, 64, 3, 1, 1, bias=False)
        elif stem == "imagenet":
            self.conv1 = nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False)
        else:
            raise ValueError(f"unknown stem {stem!r}")
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], 1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], 2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], 2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], 2)
        self.linear = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, n, stride):
        layers = []
        for s in [stride] + [1] * (n - 1):
            layers.append(block(self.in_planes, planes, s))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*layers)

    def forward(self, x):
        if fused.active(x):
            from ..ops.nn import bn_act

            out = bn_act(_conv(self.conv1, x), self.bn1, "relu")  # CIFAR stem: MFMA stem kernels
        else:
            out = F.relu(self.bn1(self.conv1(x)))
        if self.stem == "imagenet":
            if fused.active(x):
                from ..ops.nn import maxpool3x3s2  # NHWC HIP kernels (gather backward)

                out = maxpool3x3s2(out)
            else:
                out = F.max_pool2d(out, 3, 2, 1)
        out = self.layer4(self.layer3(self.layer2(self.layer1(out))))
        if fused.active(out):
            # NHWC pool kernels + the MFMA head linear (ops/head.py): no torch reduce / copy /
            # hipBLASLt launches in the step
            from ..ops import head as head_ops
            from ..ops.nn import global_avg_pool

            out = global_avg_pool(out)
            if head_ops.linear_supported(self.linear, out):
                return head_ops.head_linear(out, self.linear)
            return self.linear(out)
        out = F.adaptive_avg_pool2d(out, 1).flatten(1)
        return self.linear(out)


def ResNet18(num_classes=10, stem="cifar"):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, stem)


def ResNet34(num_classes=10, stem="cifar"):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, stem)


def ResNet50(num_classes=10, stem="cifar"):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, stem)


def ResNet101(num_classes=10, stem="cifar"):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, stem)


def ResNet152(num_classes=10, stem="cifar"):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, stem)
