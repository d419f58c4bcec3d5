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
    def forward(ctx, x, w, b, relu, din, dout, advance, bn_node=None):
        C_ = require()
        B, K = x.shape
        N = w.shape[0]
        z = torch.empty((B, N), dtype=x.dtype, device=x.device)
        y = torch.empty((B, N), dtype=x.dtype, device=x.device) if relu else None
        C_.head_fwd(_ptr(x), _ptr(w), _ptr(b), _ptr(z), _ptr(y), B, N, K, int(relu),
                    *_drop_args(din), *_drop_args(dout), _stream(), int(x.dtype == torch.float32))
        ctx.relu, ctx.din, ctx.dout, ctx.advance = relu, din, dout, advance
        ctx.bn_node = bn_node
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
        node, ctx.bn_node = ctx.bn_node, None
        link = _head_bn_link(node, x) if (dx is not None and db.dtype == torch.float32) else None
        if link is None:
            C_.head_bwd(_ptr(dz), _ptr(y), _ptr(x), _ptr(w), _ptr(dx), _ptr(dw), _ptr(db),
                        int(db.dtype == torch.bfloat16), B, N, K, int(ctx.relu),
                        *_drop_args(ctx.dout), *_drop_args(ctx.din), int(ctx.advance), _stream(),
                        int(x.dtype == torch.float32))
        else:
            # the backward statistics + finalisation of the BN layer x comes from ride in the
            # input-gradient blocks; its backward then only applies (ops/nn.py _BNAct)
            from .nn import bn_fin_outputs

            h, code, stats = link
            fin = bn_fin_outputs(node, K, x.device)
            coef, dgm, dbt, dcb = fin
            cb_dtype = getattr(node, "cb_dtype", None)
            C_.head_bwd_bn(_ptr(dz), _ptr(y), _ptr(x), _ptr(w), _ptr(dx), _ptr(dw), _ptr(db), B, N,
                           K, int(ctx.relu), *_drop_args(ctx.dout), *_drop_args(ctx.din),
                           int(ctx.advance), _ptr(h), _ptr(code), _ptr(stats), _ptr(coef),
                           _ptr(dgm), _ptr(dbt), _ptr(dcb), int(cb_dtype == torch.bfloat16),
                           _ptr(_bn_ticks(x.device, K)), _stream())
            node._ew_pre_bwd = (None, 0, dx, dx._version, fin)
            global BN_RIDES
            BN_RIDES += 1
        return (dx, (dw if need[1] else None), (db if need[2] else None), None, None, None, None,
                None)


class _HeadLinearCE(torch.autograd.Function):
    """(mean cross-entropy, logits) of ``x W^T + b`` against ``y``: the cross-entropy rides in the
    Linear's forward launch (ops/csrc/head.hip HdCe, <= 16 classes), d(loss)/d(logits) for the
    trainer's unit seed written there too (as ``ops.nn.cross_entropy``), so the backward is the
    Linear's one launch."""

    @staticmethod
    def forward(ctx, x, w, b, y):
        from .nn import _unit_seed

        C_ = require()
        B, K = x.shape
        N = w.shape[0]
        dev = x.device
        z = torch.empty((B, N), dtype=x.dtype, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        loss = torch.empty((), **f32)
        lse = torch.empty(B, **f32)
        lossrow = torch.empty(B, **f32)
        want = torch.is_grad_enabled() and _unit_seed() is not None
        dlog = torch.empty_like(z) if want else None
        tick = _ctr(_HeadLinearCE, dev)[2:3]  # word 2: free in the counter layout (_CTR_INTS)
        C_.head_fwd_ce(_ptr(x), _ptr(w), _ptr(b), _ptr(z), B, N, K, _ptr(y), _ptr(lossrow),
                       _ptr(loss), _ptr(lse), _ptr(dlog), _ptr(tick), _stream(),
                       int(x.dtype == torch.float32))
        ctx.save_for_backward(x, w, z, y, lse)
        ctx.dlog = dlog
        ctx.mark_non_differentiable(z)
        ctx.set_materialize_grads(False)
        return loss, z

    @staticmethod
    def backward(ctx, gloss, _gz):
        from .nn import _unit_seed

        C_ = require()
        x, w, z, y, lse = ctx.saved_tensors
        dlog, ctx.dlog = ctx.dlog, None
        B, K = x.shape
        N = w.shape[0]
        need = ctx.needs_input_grad
        if gloss is None:
            return None, None, None, None
        seed = _unit_seed()
        if not (dlog is not None and seed is not None and gloss.numel() == 1
                and gloss.dtype == torch.float32 and gloss.data_ptr() == seed.data_ptr()):
            dlog = torch.empty_like(z)
            g = gloss.detach().float().contiguous()
            C_.cross_entropy_bwd(_ptr(z), _ptr(y), _ptr(lse), _ptr(g), B, N,
                                 int(z.dtype == torch.bfloat16), _ptr(dlog), _stream())
        dx = torch.empty_like(x) if need[0] else None
        dw = torch.empty_like(w)
        db = torch.empty(N, dtype=w.dtype, device=w.device)
        C_.head_bwd(_ptr(dlog), 0, _ptr(x), _ptr(w), _ptr(dx), _ptr(dw), _ptr(db),
                    int(db.dtype == torch.bfloat16), B, N, K, 0, 0, 0, 0.0, 0, 0, 0.0, 1,
                    _stream(), int(x.dtype == torch.float32))
        return dx, (dw if need[1] else None), (db if need[2] else None), None


# the backward of the BN + ReLU + 2x2-pool layer feeding the head (VGG's last conv block) riding in
# the first Linear's input-gradient launch (ops/csrc/head.hip HdBnB); EWDML_HEAD_BN=0: its own
# statistics + finalize launches
_HEAD_BN = os.environ.get("EWDML_HEAD_BN", "1") != "0"
BN_RIDES = 0  # head backward launches that formed the BN layer's finalisation (tests)
_BN_TICKS = {}


def _bn_ticks(device, K):
    t = _BN_TICKS.get((device.index, K))
    if t is None:
        t = _BN_TICKS[(device.index, K)] = torch.zeros(max(1, K // 16), dtype=torch.int32,
                                                       device=device)
    return t


def _head_bn_link(node, x):
    """(h, code, stats) of the fused BN layer ``node`` (``ops.nn.bn_act`` ctx) whose pooled 1x1
    output, flattened, is ``x`` -- a BN + ReLU + 2x2 max pool over 2x2 maps, fp32 -- or None."""
    if node is None or not _HEAD_BN or x.dtype != torch.float32:
        return None
    try:
        h, res, code, stats = node.saved_tensors
    except RuntimeError:  # already freed
        return None
    B, K = x.shape
    if not (node.pool and node.mode == "relu" and res is None and code is not None
            and h.dtype == torch.float32 and tuple(h.shape) == (B, K, 2, 2)
            and h.is_contiguous(memory_format=torch.channels_last) and K % 16 == 0):
        return None
    return h, code, stats


def head_linear(x, lin, relu=False, din=None, dout=None, advance=True, bn_node=None):
    """``drop_out(act(lin(drop_in(x))))`` through the head kernels; ``din`` / ``dout``: dropout
    specs ``(counter, salt, p)`` (see :func:`_ctr`) or None; ``bn_node``: the ``_BNAct`` node of
    the BN layer ``x`` is the flattened output of (its backward may ride in this one's)."""
    return _HeadLinear.apply(x, lin.weight, lin.bias, bool(relu), din, dout, bool(advance),
                             bn_node)


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


# VGG classifier tail (fc2 + fc3 + cross-entropy, one launch each way) instead of head.hip's
# per-Linear kernels + the cross-entropy kernel: opt-in (EWDML_HEAD_TAIL=1).  Three launches fewer,
# but its forward's chain (tile GEMM, ticket, logit shares, loss, dh2, ticket) took 23.7 us
# against 17.7 for the three launches it replaces: 1.200 vs 1.193 ms per VGG-11 step
# (profiles/ab/README.md)
_TAIL = os.environ.get("EWDML_HEAD_TAIL", "0") == "1"
_TAIL_WS = {}  # (device index, B, N2) -> (workspace, tickets): zeroed once, kept zero


class _HeadTail(torch.autograd.Function):
    """(mean cross-entropy, logits) of ``relu(h1 W2^T + b2) W3^T + b3`` against ``y`` -- VGG's
    classifier after its first Linear -- in one launch each way (ops/csrc/head_tail.hip)."""

    @staticmethod
    def forward(ctx, h1, y, w2, b2, w3, b3):
        C_ = require()
        B, K1 = h1.shape
        N2, K = w2.shape[0], w3.shape[0]
        dev = h1.device
        f32 = dict(dtype=torch.float32, device=dev)
        h2 = torch.empty(B, N2, **f32)
        dh2 = torch.empty(B, N2, **f32)
        logits = torch.empty(B, K, **f32)
        dlogits = torch.empty(B, K, **f32)
        lossrow = torch.empty(B, **f32)
        loss = torch.empty((), **f32)
        key = (dev.index, B, N2)
        ws = _TAIL_WS.get(key)
        if ws is None:
            ws = _TAIL_WS[key] = (torch.zeros(C_.tail_ws_floats(B, N2), **f32),
                                  torch.zeros(C_.tail_counters(B), dtype=torch.int32, device=dev))
        C_.tail_fwd(_ptr(h1), _ptr(w2), _ptr(b2), _ptr(w3), _ptr(b3), _ptr(y), B, K1, N2, K,
                    _ptr(h2), _ptr(logits), _ptr(dlogits), _ptr(dh2), _ptr(lossrow), _ptr(loss),
                    _ptr(ws[0]), ws[0].numel(), _ptr(ws[1]), ws[1].numel(), _stream())
        ctx.save_for_backward(h1, h2, dh2, dlogits, w2)
        ctx.shapes = (w3.shape, b2.shape, b3.shape)
        ctx.mark_non_differentiable(logits)
        ctx.set_materialize_grads(False)
        return loss, logits

    @staticmethod
    def backward(ctx, gloss, _glogits):
        C_ = require()
        h1, h2, dh2, dlogits, w2 = ctx.saved_tensors
        B, K1 = h1.shape
        N2, K = w2.shape[0], dlogits.shape[1]
        g = gloss.detach().to(torch.float32).contiguous()
        dh1 = torch.empty_like(h1)
        dw2, db2 = torch.empty_like(w2), torch.empty(N2, dtype=torch.float32, device=h1.device)
        dw3 = torch.empty(K, N2, dtype=torch.float32, device=h1.device)
        db3 = torch.empty(K, dtype=torch.float32, device=h1.device)
        C_.tail_bwd(_ptr(h1), _ptr(h2), _ptr(dh2), _ptr(dlogits), _ptr(w2), _ptr(g), B, K1, N2, K,
                    _ptr(dh1), _ptr(dw2), _ptr(db2), _ptr(dw3), _ptr(db3), _stream())
        return dh1, None, dw2, db2, dw3, db3


def tail_supported(cls, x, y) -> bool:
    """The fused classifier tail applies: fp32 VGG head layout, <= 16 classes, widths % 16, int64
    labels, no autocast."""
    if not (_TAIL and supported(cls, x) and x.dtype == torch.float32 and y is not None
            and y.dtype == torch.int64 and y.dim() == 1 and y.shape[0] == x.shape[0]
            and y.is_contiguous() and not torch.is_autocast_enabled("cuda")):
        return False
    l2, l3 = cls[4], cls[6]
    return (0 < l3.out_features <= 16 and l2.in_features % 16 == 0 and l2.out_features % 16 == 0
            and l3.weight.is_contiguous() and l3.bias.is_contiguous()
            and l2.weight.data_ptr() % 16 == 0)


def vgg_loss(cls, x, y):
    """(mean cross-entropy, logits) of VGG's classifier on ``x`` against ``y``: the first Linear
    (with both dropouts) on head.hip's kernels, the rest on the fused tail."""
    d0, l1, _, d1, l2, _, l3 = list(cls)
    dev = x.device
    h1 = head_linear(x, l1, relu=True, din=_spec(d0, dev, 0), dout=_spec(d1, dev, 1))
    return _HeadTail.apply(h1, y, l2.weight, l2.bias, l3.weight, l3.bias)


# the cross-entropy riding in the last Linear's forward launch (_HeadLinearCE), opt-in
# (EWDML_HEAD_CE=1): one launch fewer, but the step is unchanged (VGG-11 1.1691 / 1.1714 vs
# 1.1684 / 1.1667 ms, profiles/ab/README.md): the row losses' ticket chain takes about what the
# separate cross-entropy launch took
_HEAD_CE = os.environ.get("EWDML_HEAD_CE", "0") == "1"


def head_ce_supported(cls, x, y) -> bool:
    """VGG's classifier with the loss riding in its last Linear applies: head layout, <= 16
    classes, int64 labels, no autocast."""
    return (_HEAD_CE and supported(cls, x) and y is not None and y.dtype == torch.int64
            and y.dim() == 1 and y.shape[0] == x.shape[0] and y.is_contiguous()
            and 0 < cls[6].out_features <= 16 and not torch.is_autocast_enabled("cuda"))


def vgg_head_loss(cls, x, y, bn_node=None):
    """(mean cross-entropy, logits) of VGG's classifier on ``x``: head.hip's kernels, the loss in
    the last Linear's launch."""
    d0, l1, _, d1, l2, _, l3 = list(cls)
    dev = x.device
    h = head_linear(x, l1, relu=True, din=_spec(d0, dev, 0), dout=_spec(d1, dev, 1),
                    bn_node=bn_node)
    h = head_linear(h, l2, relu=True)
    return _HeadLinearCE.apply(h, l3.weight, l3.bias, y)


def vgg_head(cls, x, bn_node=None):
    """``cls(x)`` for VGG's classifier ``nn.Sequential`` through the fused kernels; ``bn_node``:
    see :func:`head_linear`."""
    if not supported(cls, x):
        return cls(x)
    d0, l1, _, d1, l2, _, l3 = list(cls)
    dev = x.device
    h = head_linear(x, l1, relu=True, din=_spec(d0, dev, 0), dout=_spec(d1, dev, 1),
                    bn_node=bn_node)
    h = head_linear(h, l2, relu=True)
    return head_linear(h, l3)
