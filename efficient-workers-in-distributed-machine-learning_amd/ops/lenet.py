"""LeNet's fp32 training step as four HIP launches (``ops/csrc/lenet_f32.hip``).

``lenet_loss(model, x, y)`` returns ``(loss, logits)`` -- the mean cross-entropy of
``models.LeNet`` on ``(x, y)`` with autograd wired to the fused backward -- or None when the fast
path does not apply (CPU, bf16 autocast, ``fc_relu``, other shapes); the trainer then runs the
module composition.  Forward: conv1+pool+relu+conv2+pool+relu per image quarter, fc1 tiles whose
last arrivals form fc2, the cross-entropy, d(logits) and d(fc1 out).  Backward: fc gradients and
d(a2) in one launch, the conv gradients in one more.  Parity: the module path of
``models/lenet.py`` (``PyTorch-parameter-server/src/model_ops/lenet.py:15-36``) with the
reference's ``nn.CrossEntropyLoss`` (``src/distributed_worker.py:249-251``).
"""
import os

import torch

from . import _ptr, _stream, available, require

# EWDML_LENET_FUSED=0: the module composition (A/B, tests)
_ON = os.environ.get("EWDML_LENET_FUSED", "1") != "0"
_WS = {}  # (device index, B) -> (workspace floats, ticket ints): zeroed once, kept zero


def _ws(device, B):
    key = (device.index, B)
    ws = _WS.get(key)
    if ws is None:
        C_ = require()
        ws = (torch.zeros(C_.lenet_ws_floats(B), dtype=torch.float32, device=device),
              torch.zeros(C_.lenet_counters(B), dtype=torch.int32, device=device))
        _WS[key] = ws
    return ws


def _params(model):
    return (model.conv1.weight, model.conv1.bias, model.conv2.weight, model.conv2.bias,
            model.fc1.weight, model.fc1.bias, model.fc2.weight, model.fc2.bias)


def supported(model, x, y) -> bool:
    """The fused step applies: device fp32 LeNet (no fc ReLU), 1x28x28 inputs, int64 labels,
    <= 16 classes, dense 16-byte-aligned tensors, no autocast."""
    if not (_ON and x.is_cuda and available() and torch.is_grad_enabled()):
        return False
    if getattr(model, "fc_relu", False) or torch.is_autocast_enabled("cuda"):
        return False
    if x.dtype != torch.float32 or tuple(x.shape[1:]) != (1, 28, 28) or not x.is_contiguous():
        return False
    if y.dtype != torch.int64 or y.dim() != 1 or y.shape[0] != x.shape[0] or not y.is_contiguous():
        return False
    ps = _params(model)
    shapes = ((20, 1, 5, 5), (20,), (50, 20, 5, 5), (50,), (500, 800), (500,), None, None)
    for p, s in zip(ps, shapes):
        if p is None or p.dtype != torch.float32 or not p.is_contiguous() or p.device != x.device:
            return False
        if s is not None and tuple(p.shape) != s:
            return False
    K = ps[6].shape[0]
    if not (0 < K <= 16 and tuple(ps[6].shape) == (K, 500) and tuple(ps[7].shape) == (K,)):
        return False
    return all(t.data_ptr() % 16 == 0 for t in (x, ps[0], ps[2], ps[4]))


class _LeNetStep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, w1, b1, w2, b2, wf1, bf1, wf2, bf2, batch=None):
        C_ = require()
        B, K = x.shape[0], wf2.shape[0]
        dev = x.device
        f32 = dict(dtype=torch.float32, device=dev)
        a1 = torch.empty(B, 2880, **f32)
        code1 = torch.empty(B, 2880, dtype=torch.uint8, device=dev)
        a2 = torch.empty(B, 800, **f32)
        code2 = torch.empty(B, 800, dtype=torch.uint8, device=dev)
        h1 = torch.empty(B, 500, **f32)
        logits = torch.empty(B, K, **f32)
        dlogits = torch.empty(B, K, **f32)
        dh1 = torch.empty(B, 500, **f32)
        lossrow = torch.empty(B, **f32)
        loss = torch.empty((), **f32)
        ws, cnt = _ws(dev, B)
        C_.lenet_fwd(_ptr(x), _ptr(w1), _ptr(b1), _ptr(w2), _ptr(b2), _ptr(wf1), _ptr(bf1),
                     _ptr(wf2), _ptr(bf2), _ptr(y), B, K, _ptr(a1), _ptr(code1), _ptr(a2),
                     _ptr(code2), _ptr(h1), _ptr(logits), _ptr(dlogits), _ptr(dh1),
                     _ptr(lossrow), _ptr(loss), _ptr(ws), ws.numel(), _ptr(cnt), cnt.numel(),
                     _stream(), *_batch_ptrs(batch))
        ctx.save_for_backward(x, w2, wf1, a1, code1, a2, code2, h1, dlogits, dh1)
        ctx.params = (w1, b1, w2, b2, wf1, bf1, wf2, bf2)
        ctx.mark_non_differentiable(logits)
        ctx.set_materialize_grads(False)  # no zero-filled d(logits) launch
        return loss, logits

    @staticmethod
    def backward(ctx, gloss, _glogits):
        C_ = require()
        x, w2, wf1, a1, code1, a2, code2, h1, dlogits, dh1 = ctx.saved_tensors
        params, ctx.params = ctx.params, None
        B, K = x.shape[0], dlogits.shape[1]
        g = gloss.detach().to(torch.float32).contiguous()
        grads = [torch.empty_like(p) for p in params]
        dp2 = torch.empty(B, 800, dtype=torch.float32, device=x.device)
        ws, cnt = _ws(x.device, B)
        C_.lenet_bwd(_ptr(x), _ptr(w2), _ptr(wf1), _ptr(a1), _ptr(code1), _ptr(a2), _ptr(code2),
                     _ptr(h1), _ptr(dlogits), _ptr(dh1), _ptr(g), B, K, _ptr(dp2),
                     *[_ptr(t) for t in grads], _ptr(ws), ws.numel(), _ptr(cnt), cnt.numel(),
                     _stream())
        return (None, None, *grads, None)


def _batch_ptrs(batch):
    """lenet_fwd's batch-source arguments (data/loader.py take_deferred), zeros for none."""
    if batch is None:
        return (0, 0, 0, 0, 0, 0, 0.0, 1.0)
    src, labels, perm, state, done, mean, inv_std = batch
    return (_ptr(src), _ptr(labels), _ptr(perm), perm.numel(), _ptr(state), _ptr(done),
            float(mean), float(inv_std))


def lenet_loss(model, x, y):
    """(mean cross-entropy, logits) of ``model`` (a ``models.LeNet``) through the fused kernels,
    or None where they do not apply.  ``x`` may be a fused loader's deferred batch buffer
    (``_ew_batch``): the conv launch then forms the batch (and its labels in ``y``) itself."""
    if not supported(model, x, y):
        return None
    ldr = getattr(x, "_ew_batch", None)
    batch = None
    if ldr is not None and ldr.bx is x and ldr.by is y:
        batch = ldr.take_deferred()
    return _LeNetStep.apply(x, y, *_params(model), batch)
