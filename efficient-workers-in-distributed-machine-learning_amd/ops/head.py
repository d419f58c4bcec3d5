"""VGG classifier head (``Dropout, Linear, ReLU, Dropout, Linear, ReLU, Linear``) on the GPU:
one hand-written MFMA kernel per Linear and direction (``ops/csrc/head.hip``).

Per step PyTorch runs the head as 9 forward and 13 backward kernels (dropout x2, ReLU clamps,
hipBLASLt GEMMs, bias-gradient reductions, dropout / threshold backward) plus two per-replay RNG
offset fills under HIP graphs (~114 us of a ~1.05 ms VGG-11 step).  Here 3 forward and 3 backward
kernels: the input Dropout is applied to the first GEMM's operand on load, bias + ReLU + Dropout
run in the GEMM epilogue, and each backward launch recomputes its masks on load and computes the
weight, bias and input gradients together.  Same math as ``nn.Dropout`` / ``nn.ReLU`` /
``nn.Linear`` with bf16 or fp32 operands (``v_mfma_f32_16x16x32_bf16`` /
``v_mfma_f32_16x16x4_f32``) and fp32 accumulation; masks come from a counter-based hash keyed
per step by a per-layer device counter (so they differ from PyTorch's generator; the keep
probability and 1/(1-p) scaling are the same).  :class:`_ActDropout` (one act/dropout kernel per
direction, ``ops/csrc/nn.hip``) remains as a standalone op.

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


# counter words: [0] mask step, [1] act_dropout_bwd's ticket, [32, 32 + TICKET_INTS) the head
# backward's grid arrival ticket (ops/csrc/head.hip HD_TICKET)
_CTR_INTS = 32 + 9 * 32


def _ctr(mod, device):
    """Per-layer device dropout counter (zeros; see ``_CTR_INTS``)."""
    c = getattr(mod, "_ew_drop_ctr", None)
    if c is None or c.device != device:
        c = torch.zeros(_CTR_INTS, dtype=torch.int32, device=device)
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


def _drop_args(d):
    """(counter pointer, salt, p) of a dropout spec ``(ctr, salt, p)`` or None."""
    if d is None or d[2] <= 0.0:
        return 0, 0, 0.0
    return _ptr(d[0]), int(d[1]) & 0xFFFFFFFF, float(d[2])


class _HeadLinear(torch.autograd.Function):
    """z = drop_out(act(drop_in(x) W^T + b)); ``din`` / ``dout``: dropout specs (ctr, salt, p) or
    None.  The backward launch advances the counters of the masks it recomputed when
    ``advance``."""

    @staticmethod
    def forward(ctx, x, w, b, relu, din, dout, advance):
        C_ = require()
        B, K = x.shape
        N = w.shape[0]
        z = torch.empty((B, N), dtype=x.dtype, device=x.device)
        y = torch.empty((B, N), dtype=x.dtype, device=x.device) if relu else None
        C_.head_fwd(_ptr(x), _ptr(w), _ptr(b), _ptr(z), _ptr(y), B, N, K, int(relu),
                    *_drop_args(din), *_drop_args(dout), _stream(), int(x.dtype == torch.float32))
        ctx.relu, ctx.din, ctx.dout, ctx.advance = relu, din, dout, advance
        ctx.save_for_backward(x, w, y)
        return z

    @staticmethod
    def backward(ctx, dz):
        C_ = require()
        x, w, y = ctx.saved_tensors
        dz = dz.contiguous()
        if dz.data_ptr() % 16:
            dz = dz.clone()
        B, K = x.shape
        N = w.shape[0]
        need = ctx.needs_input_grad
        dx = torch.empty_like(x) if need[0] else None
        dw = torch.empty_like(w)
        db = torch.empty(N, dtype=w.dtype, device=w.device)
        C_.head_bwd(_ptr(dz), _ptr(y), _ptr(x), _ptr(w), _ptr(dx), _ptr(dw), _ptr(db),
                    int(db.dtype == torch.bfloat16), B, N, K, int(ctx.relu),
                    *_drop_args(ctx.dout), *_drop_args(ctx.din), int(ctx.advance), _stream(),
                    int(x.dtype == torch.float32))
        return dx, (dw if need[1] else None), (db if need[2] else None), None, None, None, None


def head_linear(x, lin, relu=False, din=None, dout=None, advance=True):
    """``drop_out(act(lin(drop_in(x))))`` through the head kernels; ``din`` / ``dout``: dropout
    specs ``(counter, salt, p)`` (see :func:`_ctr`) or None."""
    return _HeadLinear.apply(x, lin.weight, lin.bias, bool(relu), din, dout, bool(advance))


def _head_layout(cls):
    mods = list(cls)
    if len(mods) != 7:
        return None
    d0, l1, r1, d1, l2, r2, l3 = mods
    ok = (isinstance(d0, nn.Dropout) and isinstance(l1, nn.Linear) and isinstance(r1, nn.ReLU)
          and isinstance(d1, nn.Dropout) and isinstance(l2, nn.Linear)
          and isinstance(r2, nn.ReLU) and isinstance(l3, nn.Linear))
    return mods if ok else None


def _lin_ok(lin, x_width, dtype):
    w, b = lin.weight, lin.bias
    return (b is not None and w.dtype == dtype and b.dtype == dtype
            and w.is_contiguous() and b.is_contiguous() and w.shape[1] == x_width
            and x_width % 32 == 0 and w.data_ptr() % 16 == 0)


def linear_supported(lin, x) -> bool:
    """Whether ``lin(x)`` (one ``nn.Linear`` on a device [B, K] activation) runs the head kernels."""
    return (_ENABLED and isinstance(lin, nn.Linear) and x.is_cuda and x.dim() == 2
            and x.dtype in (torch.bfloat16, torch.float32) and _lin_ok(lin, x.shape[1], x.dtype)
            and x.is_contiguous() and x.data_ptr() % 16 == 0 and 0 < x.shape[0]
            and x.shape[0] * max(x.shape[1], lin.out_features) < 2 ** 31)


def supported(cls, x) -> bool:
    mods = _head_layout(cls)
    if not _ENABLED or mods is None or not (x.is_cuda and x.dim() == 2
                                            and x.dtype in (torch.bfloat16, torch.float32)):
        return False
    l1, l2, l3 = mods[1], mods[4], mods[6]
    dt = x.dtype
    if not (_lin_ok(l1, x.shape[1], dt) and _lin_ok(l2, l1.out_features, dt)
            and _lin_ok(l3, l2.out_features, dt)):
        return False
    return (x.is_contiguous() and x.data_ptr() % 16 == 0 and 0 < x.shape[0]
            and x.shape[0] * max(x.shape[1], l1.out_features, l2.out_features) < 2 ** 31)


def _spec(d, device, layer):
    """Dropout spec of module ``d`` (None when inactive): its counter, a per-layer salt."""
    p = _p(d)
    if p <= 0.0:
        return None
    return (_ctr(d, device), (_SALT ^ (0x9E3779B9 * (layer + 1))) & 0xFFFFFFFF, p)


def vgg_head(cls, x):
    """``cls(x)`` for VGG's classifier ``nn.Sequential`` through the fused kernels."""
    if not supported(cls, x):
        return cls(x)
    d0, l1, _, d1, l2, _, l3 = list(cls)
    dev = x.device
    h = head_linear(x, l1, relu=True, din=_spec(d0, dev, 0), dout=_spec(d1, dev, 1))
    h = head_linear(h, l2, relu=True)
    return head_linear(h, l3)
