"""Execution of conv -> BatchNorm -> ReLU [-> MaxPool 2x2] stacks through the fused NHWC kernels.

:class:`FusedFeatures` is an ``nn.Sequential`` (same modules, parameters and ``state_dict`` keys as
the plain stack the reference builds in ``src/model_ops/vgg.py:39-52``) whose forward, on
channels_last device activations, runs each ``Conv2d, BatchNorm2d, ReLU[, MaxPool2d(2, 2)]`` group
as ``conv2d(x, w)`` (bias folded into the BN kernel) + :func:`ewdml.ops.nn.bn_relu`, and a lone
``MaxPool2d(2, 2)`` as :func:`ewdml.ops.nn.maxpool2x2`.  On the CPU, or for shapes the kernels do
not take, it is exactly ``nn.Sequential.forward``.

``set_enabled(False)`` (``--fused-nn off``) restores the module-by-module path everywhere.
"""
import os

import torch
import torch.nn as nn

_ENABLED = True
# BN layers feeding a Winograd conv leave their apply (forward and backward) to that conv's input
# transforms (EWDML_LAZY_BN=0: always materialise the activations)
_LAZY = os.environ.get("EWDML_LAZY_BN", "1") != "0"


def set_enabled(on: bool):
    global _ENABLED
    _ENABLED = bool(on)


def enabled() -> bool:
    return _ENABLED


def active(x) -> bool:
    """Run the fused kernels for this activation (device tensor, fused path enabled)."""
    return _ENABLED and x.is_cuda


def is_pool2(m) -> bool:
    def two(v):
        return v == 2 or v == (2, 2)

    return (isinstance(m, nn.MaxPool2d) and two(m.kernel_size)
            and two(m.stride if m.stride is not None else m.kernel_size)
            and m.padding in (0, (0, 0)) and m.dilation in (1, (1, 1)) and not m.ceil_mode
            and not m.return_indices)


def pool2(x):
    """``F.max_pool2d(x, 2, 2)``, through the HIP kernel on the GPU."""
    if _ENABLED and x.is_cuda:
        from ..ops.nn import maxpool2x2

        return maxpool2x2(x)
    return torch.nn.functional.max_pool2d(x, 2, 2)


class FusedFeatures(nn.Sequential):
    def _plan(self):
        plan = getattr(self, "_ew_plan", None)
        if plan is not None and plan[0] == len(self):
            return plan[1]
        mods = list(self)
        groups, i = [], 0
        while i < len(mods):
            m = mods[i]
            if (isinstance(m, nn.Conv2d) and i + 2 < len(mods)
                    and isinstance(mods[i + 1], nn.BatchNorm2d) and isinstance(mods[i + 2], nn.ReLU)
                    and m.padding_mode == "zeros"):
                pool = i + 3 < len(mods) and is_pool2(mods[i + 3])
                groups.append(("cbr", mods[i:i + (4 if pool else 3)], pool))
                i += 4 if pool else 3
            elif is_pool2(m):
                groups.append(("pool", [m], True))
                i += 1
            else:
                groups.append(("mod", [m], False))
                i += 1
        self._ew_plan = (len(self), groups)
        return groups

    @staticmethod
    def _lazy_into(plan, gi, h, pool) -> bool:
        """Whether group gi's BN-ReLU(-pool) output feeds only the next group's conv and that
        conv forms its input on the fly (Winograd input transform, 2x2-map GEMM operand load): then
        that conv applies the BN layer
        (ops/nn.py bn_relu(lazy=True)) and the activation is never written."""
        # pooled layers stay materialised: recomputing the 2x2 max for every patch element
        # (16 reads of h per element) costs more than the apply kernel it would save
        # (profiles/vgg11_bs128_fp32_current_graph.txt: conv3/5/7 input 20/17.5/16.7 us lazy
        # against 16.2/10.9/10.4 us apply + transform); their backward stays lazy
        if not _LAZY or pool or gi + 1 >= len(plan) or plan[gi + 1][0] != "cbr":
            return False
        from ..ops import conv as conv_hip

        nxt = plan[gi + 1][1][0]
        if not (nxt.stride in (1, (1, 1)) and nxt.padding in (1, (1, 1))
                and nxt.dilation in (1, (1, 1)) and nxt.groups == 1):
            return False
        N, C, H, W = h.shape
        shape = (N, C, H // 2, W // 2) if pool else (N, C, H, W)
        return conv_hip.enabled() and conv_hip.lazy_input_ok(shape, h.dtype, nxt.weight)

    def forward(self, x):
        if not (_ENABLED and x.is_cuda):
            return super().forward(x)
        from ..ops import conv as conv_hip
        from ..ops import nn as fnn

        plan = self._plan()
        for gi, (kind, mods, pool) in enumerate(plan):
            if kind == "cbr":
                conv, bn = mods[0], mods[1]
                if conv_hip.supported(x, conv.weight, conv.stride, conv.padding, conv.dilation,
                                      conv.groups):
                    h = conv_hip.conv3x3(x, conv.weight)  # MFMA implicit GEMM (ops/conv.py)
                else:  # a lazily produced input (BN apply left to a Winograd conv) is written first
                    h = conv._conv_forward(fnn.materialize(x), conv.weight, None)
                if fnn.nhwc_supported(h, pool):
                    x = fnn.bn_relu(h, conv.bias, bn, pool, lazy=self._lazy_into(plan, gi, h, pool))
                else:
                    if conv.bias is not None:
                        h = h + conv.bias.to(h.dtype).view(1, -1, 1, 1)
                    for m in mods[1:]:
                        h = m(h)
                    x = h
            elif kind == "pool":
                x = fnn.maxpool2x2(fnn.materialize(x))
            else:
                x = mods[0](fnn.materialize(x))
        return x
