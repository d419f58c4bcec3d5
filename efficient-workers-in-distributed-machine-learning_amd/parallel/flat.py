"""Flat, bucketed parameter and gradient storage.

All trainable parameters become views of ONE contiguous fp32 buffer and their ``.grad`` views of a
second one, laid out in *reverse* registration order (the order backward produces gradients) with
every tensor 64-element (256 B) aligned.  Consequences:

* autograd accumulates straight into the flat gradient buffer (``AccumulateGrad`` adds in place
  into an existing ``.grad``), so a bucket is a contiguous range ready for a collective with no
  copy -- what Horovod's fusion buffer (``--fusion-threshold-mb 32``, ``Horovod all reduce.ipynb``)
  emulates by copying;
* the optimizer is one multi-tensor kernel over the buffer instead of the reference's per-tensor
  loop (``optim/sgd.py:75``);
* a checkpoint/broadcast of the model is one tensor.

Parity: the per-layer gather buffers of ``sync_replicas_master_nn.py:49-86`` (GradientAccumulator)
and ``distributed_worker.py:41-59`` (ModelBuffer) are replaced by these views.
"""
from dataclasses import dataclass
from typing import List

import torch

from ..compress.plan import BucketPlan

ALIGN = 64


def _align(n, a=ALIGN):
    return (n + a - 1) // a * a


def _same_layout(g, p):
    """Same memory order (strides of non-singleton dims equal)."""
    return all(a == b for a, b, n in zip(g.stride(), p.stride(), p.shape) if n > 1)


@dataclass
class Bucket:
    index: int
    start: int  # element offset in the flat buffer
    length: int
    params: List[torch.nn.Parameter]
    plan: BucketPlan


MAX_TENSORS_PER_BUCKET = 128  # kernel pointer-table capacity (ops.MAX_TENSORS_PER_BUCKET)


class FlatModel:
    def __init__(self, model, bucket_bytes: int = 8 << 20, reverse: bool = True,
                 attach_grads: bool = True, bf16_params: bool = False):
        """``model``: an ``nn.Module`` or an iterable of parameters.

        ``attach_grads=True``: every ``p.grad`` is a view of ``self.grad`` and autograd accumulates
        into it.  ``False``: ``p.grad`` is left to autograd (``zero_grad`` sets it to None, so the
        incoming gradient is stolen, not added) and the exchange reads each tensor in place
        through a pointer table -- no per-parameter accumulate kernels, no buffer fill.

        ``bf16_params=True`` (needs ``attach_grads=False``): the weights and biases of conv and
        linear layers become bf16 views of ``self.shadow``, a bf16 copy of the fp32 master
        ``self.data`` that the optimizer kernels rewrite (round-to-nearest-even) after every
        update.  Under bf16 autocast this computes exactly what autocast computes (it would cast
        the same fp32 master to the same bf16 values every forward), without the per-step weight
        casts and without casting the bf16 weight gradients back to fp32."""
        seen = set()
        params = []
        plist = model.parameters() if isinstance(model, torch.nn.Module) else model
        if not isinstance(model, torch.nn.Module):
            model = None
        for p in plist:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append(p)
        if reverse:
            params = params[::-1]
        self.model = model
        self.params = params
        dev = params[0].device
        offs = []
        total = 0
        for p in params:
            offs.append(total)
            total += _align(p.numel())
        self.offsets = offs
        self.numel = total
        self.param_numel = sum(p.numel() for p in params)
        self.attach_grads = attach_grads
        if bf16_params and attach_grads:
            raise ValueError("bf16 compute parameters need attach_grads=False")
        lowp = set()
        if bf16_params and model is not None:
            for m in model.modules():
                if isinstance(m, (torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.Conv3d,
                                  torch.nn.Linear)):
                    lowp.update(id(q) for q in m.parameters(recurse=False))
        self.bf16_ids = lowp
        self.data = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.shadow = torch.zeros(total, dtype=torch.bfloat16, device=dev) if lowp else None
        for p, o in zip(params, offs):
            if p.dtype != torch.float32:
                raise TypeError("flat buffers hold fp32 master weights; keep params fp32 "
                                "(compute in bf16 via autocast)")
            n = p.numel()
            dv = self.data[o:o + n].as_strided(p.shape, p.stride())
            dv.copy_(p.data)
            if id(p) in lowp:
                sv = self.shadow[o:o + n].as_strided(p.shape, p.stride())
                sv.copy_(dv)
                dv = sv
            p.data = dv
            p.grad = self.grad[o:o + n].as_strided(p.shape, p.stride()) if attach_grads else None
        self.buckets = self._make_buckets(bucket_bytes)

    def _make_buckets(self, bucket_bytes):
        cap = max(1, bucket_bytes // 4)
        groups, cur = [], []
        for i, p in enumerate(self.params):
            cur.append(i)
            end = self.offsets[i] + _align(p.numel())
            if end - self.offsets[cur[0]] >= cap or len(cur) >= MAX_TENSORS_PER_BUCKET:
                groups.append(cur)
                cur = []
        if cur:
            groups.append(cur)
        buckets = []
        for bi, g in enumerate(groups):
            start = self.offsets[g[0]]
            end = self.offsets[g[-1]] + _align(self.params[g[-1]].numel())
            plan = BucketPlan(numels=[self.params[i].numel() for i in g],
                              offsets=[self.offsets[i] - start for i in g],
                              ratio=1.0, bucket_offset=start, length=end - start)
            buckets.append(Bucket(bi, start, end - start, [self.params[i] for i in g], plan))
        return buckets

    def bucket_of(self):
        """param id -> bucket index."""
        return {id(p): b.index for b in self.buckets for p in b.params}

    def grad_view(self, b: Bucket) -> torch.Tensor:
        return self.grad[b.start:b.start + b.length]

    def data_view(self, b: Bucket) -> torch.Tensor:
        return self.data[b.start:b.start + b.length]

    def sync_shadow(self):
        """Refresh the bf16 compute copy from the fp32 master (after a non-kernel update)."""
        if self.shadow is not None:
            self.shadow.copy_(self.data)

    def shadow_view(self, b: "Bucket" = None):
        if self.shadow is None:
            return None
        return self.shadow if b is None else self.shadow[b.start:b.start + b.length]

    def master_view(self, p):
        i = next(k for k, q in enumerate(self.params) if q is p)
        o = self.offsets[i]
        return self.data[o:o + p.numel()].as_strided(p.shape, p.stride())

    def master_state_dict(self, model):
        """``model.state_dict()`` with every parameter taken from the fp32 master."""
        sd = model.state_dict()
        if self.shadow is None:
            return sd
        for name, p in model.named_parameters():
            if id(p) in self.bf16_ids:
                sd[name] = self.master_view(p)
        return sd

    def load_state_dict(self, model, sd):
        """Load parameters into the fp32 master (and refresh the bf16 copy) plus buffers."""
        model.load_state_dict(sd)
        if self.shadow is not None:
            for name, p in model.named_parameters():
                if id(p) in self.bf16_ids:
                    self.master_view(p).copy_(sd[name])
            self.sync_shadow()

    def zero_grad(self):
        if self.attach_grads:
            self.grad.zero_()
        else:
            for p in self.params:
                p.grad = None

    def bucket_grads(self, b: Bucket):
        """The bucket's gradients: the flat view, or (pointer mode) autograd's tensors in plan
        order (unused parameters contribute zeros)."""
        if self.attach_grads:
            return self.grad_view(b)
        out = []
        for p in b.params:
            g = p.grad
            if g is None:
                g = torch.zeros_like(p)  # p's strides (its flat memory order)
                p.grad = g
            elif not _same_layout(g, p):
                # the kernels read each gradient densely in the memory order of its slot in the
                # flat buffer, i.e. with the parameter's strides (channels_last conv weights
                # included); autograd normally already produces that layout
                h = torch.empty_like(p, dtype=g.dtype)
                h.copy_(g)
                g = h
                p.grad = g
            out.append(g)
        return out

    def reattach_grads(self):
        """Restore the ``.grad`` views (e.g. after user code set them to None)."""
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + 1].data_ptr():
                p.grad = self.grad[o:o + p.numel()].as_strided(p.shape, p.stride())
