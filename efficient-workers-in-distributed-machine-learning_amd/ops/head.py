"""VGG classifier head (``Dropout, Linear, ReLU, Dropout, Linear, ReLU, Linear``) on the GPU with
hand-written activation/dropout kernels (``ops/csrc/nn.hip``: ``k_act_dropout_fwd/bwd``).

Per step PyTorch runs the head as 9 forward and 13 backward kernels (dropout x2, ReLU clamps,
GEMMs, bias-gradient reductions, dropout / threshold backward) plus two per-replay RNG offset
fills under HIP graphs.  Here: the Linear GEMMs stay on hipBLASLt (``addmm`` with the bias in the
epilogue), each ``ReLU -> Dropout`` / ``ReLU`` / ``Dropout`` is one kernel per direction, and the
backward kernel also writes the preceding Linear's bias gradient -- 6 forward and 10 backward
kernels, same math as ``nn.Dropout`` / ``nn.ReLU`` / ``nn.Linear`` (masks from a counter-based
hash keyed per step by a device counter, so masks differ from PyTorch's generator; the keep
probability and 1/(1-p) scaling are the same).

Parity: the reference's classifier, ``src/model_ops/vgg.py:15-43``.
"""
import os

import torch
import torch.nn as nn

from . import _ptr, _stream, require

_SALT = 0x5EED
_ENABLED = os.environ.get("EWDML_HEAD", "fused") == "fused"  # EWDML_HEAD=torch: A/B


def set_seed(seed: int, rank: int = 0):
    """Dropout mask stream per (seed, rank) (called by the trainer)."""
    global _SALT
    _SALT = (int(seed) * 1000003 + int(rank) * 7919 + 0x5EED) & 0xFFFFFFFF


def _ctr(mod, device):
    """Per-layer device counter: [key step, arrival ticket of the backward's blocks]."""
    c = getattr(mod, "_ew_drop_ctr", None)
    if c is None or c.device != device:
        c = torch.zeros(2, dtype=torch.int32, device=device)
        mod._ew_drop_ctr = c
    return c



def _p(d):
    return float(d.p) if (d is not None and d.training) else 0.0


class _ActDropout(torch.autograd.Function):
    """z = act(y) * mask / (1 - p) (no Linear: the head's input dropout)."""

    @staticmethod
    def forward(ctx, y, p, relu, ctr):
        C_ = require()
        z = torch.empty_like(y)
        C_.act_dropout_fwd(_ptr(y), _ptr(z), y.numel(), p, int(relu), _ptr(ctr), _SALT, _stream())
        ctx.p, ctx.relu, ctx.salt = p, relu, _SALT
        ctx.save_for_backward(y, ctr)
        return z

    @staticmethod
    def backward(ctx, dz):
        C_ = require()
        y, ctr = ctx.saved_tensors
        dz = dz.contiguous()
        dy = torch.empty_like(y)
        rows, C = y.shape
        C_.act_dropout_bwd(_ptr(dz), _ptr(y), _ptr(dy), 0, 0, rows, C, ctx.p, int(ctx.relu),
                           _ptr(ctr), ctx.salt, _stream())
        return dy, None, None, None


class _LinearActDropout(torch.autograd.Function):
    """z = act(x W^T + b) * mask / (1 - p); backward fuses the bias gradient into the mask pass."""

    @staticmethod
    def forward(ctx, x, w, b, p, relu, ctr):
        C_ = require()
        y = torch.addmm(b, x, w.t())
        z = torch.empty_like(y)
        C_.act_dropout_fwd(_ptr(y), _ptr(z), y.numel(), p, int(relu), _ptr(ctr), _SALT, _stream())
        ctx.p, ctx.relu, ctx.salt = p, relu, _SALT
        ctx.save_for_backward(x, w, y, ctr)
        return z

    @staticmethod
    def backward(ctx, dz):
        C_ = require()
        x, w, y, ctr = ctx.saved_tensors
        dz = dz.contiguous()
        rows, C = y.shape
        dy = torch.empty_like(y)
        db = torch.empty(C, dtype=w.dtype, device=w.device)
        C_.act_dropout_bwd(_ptr(dz), _ptr(y), _ptr(dy), _ptr(db), int(db.dtype == torch.bfloat16),
                           rows, C, ctx.p, int(ctx.relu), _ptr(ctr), ctx.salt, _stream())
        need = ctx.needs_input_grad
        dx = dy @ w if need[0] else None
        dw = dy.t() @ x if need[1] else None
        return dx, dw, (db if need[2] else None), None, None, None


def _head_layout(cls):
    mods = list(cls)
    if len(mods) != 7:
        return None
    d0, l1, r1, d1, l2, r2, l3 = mods
    ok = (isinstance(d0, nn.Dropout) and isinstance(l1, nn.Linear) and isinstance(r1, nn.ReLU)
          and isinstance(d1, nn.Dropout) and isinstance(l2, nn.Linear)
          and isinstance(r2, nn.ReLU) and isinstance(l3, nn.Linear))
    return mods if ok else None


def supported(cls, x) -> bool:
    mods = _head_layout(cls)
    if not _ENABLED or mods is None or not (x.is_cuda and x.dim() == 2 and x.dtype == torch.bfloat16):
        return False
    l1, l2 = mods[1], mods[4]
    for lin in (l1, l2):
        if lin.bias is None or lin.weight.dtype != torch.bfloat16 or lin.bias.dtype != torch.bfloat16:
            return False
        if lin.out_features % 8:
            return False
    return x.is_contiguous() and x.numel() < 2 ** 31 and x.shape[1] % 8 == 0


def vgg_head(cls, x):
    """``cls(x)`` for VGG's classifier ``nn.Sequential`` through the fused kernels."""
    if not supported(cls, x):
        return cls(x)
    d0, l1, _, d1, l2, _, l3 = list(cls)
    h = _ActDropout.apply(x, _p(d0), False, _ctr(d0, x.device))
    h = _LinearActDropout.apply(h, l1.weight, l1.bias, _p(d1), True, _ctr(d1, x.device))
    h = _LinearActDropout.apply(h, l2.weight, l2.bias, 0.0, True, _ctr(l2, x.device))
    return torch.nn.functional.linear(h, l3.weight, l3.bias)
