"""Gradient codecs: one object per exchange, bound to the bucket plans of a model.

``kind``:
  * ``none``  -- dense fp32 all-reduce (reference Method 3, push+pull of raw gradients)
  * ``fp16`` / ``bf16`` -- dense half-precision all-reduce (Horovod ``Compression.fp16``,
    ``horvod_pytorch.py:191-192``)
  * ``qsgd``  -- dense stochastic quantisation to int8/int4 (Method 4)
  * ``topk``  -- top-k sparsification, fp32 values (``TopKCompressor``)
  * ``topk_qsgd`` -- top-k then QSGD (Method 5); the flagship codec

Device tensors go through the HIP kernels (``ops``); CPU tensors through the torch oracle.  On a
GPU box a missing extension raises instead of silently falling back.
"""
import os

import torch

from .. import ops

# EWDML_ORACLE=1: run the torch oracle on device tensors too (eager experiments with codec
# variants before they have kernels; needs flat gradient views, EWDML_GRAD_VIEWS=1)
_FORCE_ORACLE = os.environ.get("EWDML_ORACLE") == "1"
from . import oracle
from .plan import BucketPlan, Layout
from .rng import stream_key

KINDS = ("none", "fp16", "bf16", "qsgd", "topk", "topk_qsgd")


class Codec:
    def __init__(self, kind: str = "topk_qsgd", ratio: float = 0.01, levels: int = 127,
                 bits: int = 8, norm: str = "max", seed: int = 0, dense_below: int = 0):
        if kind not in KINDS:
            raise ValueError(f"unknown codec {kind!r}; choose from {KINDS}")
        if bits not in (4, 8):
            raise ValueError("bits must be 8 or 4")
        if kind in ("qsgd", "topk_qsgd"):
            lim = 127 if bits == 8 else 7
            if not 1 <= levels <= lim:
                raise ValueError(f"QSGD levels must be in [1, {lim}] for {bits}-bit codes")
        if not 0.0 < ratio <= 1.0:
            raise ValueError("top-k ratio must be in (0, 1]")
        self.kind, self.ratio, self.levels, self.bits, self.norm = kind, ratio, levels, bits, norm
        self.seed = seed
        self.dense_below = int(dense_below)
        self.plans = []
        self.layouts = []
        self.dplans = []
        self.device = None

    # -- properties -------------------------------------------------------------------------
    @property
    def allreduce(self) -> bool:
        """Dense codecs are summed by the collective itself (all-reduce)."""
        return self.kind in ("none", "fp16", "bf16")

    @property
    def wire_dtype(self):
        return {"none": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}.get(self.kind)

    def describe(self) -> str:
        if self.kind == "topk_qsgd":
            return f"topk{self.ratio:g}+qsgd{self.bits}b(s={self.levels},{self.norm})"
        if self.kind == "qsgd":
            return f"qsgd{self.bits}b(s={self.levels},{self.norm})"
        if self.kind == "topk":
            return f"topk{self.ratio:g}"
        return self.kind

    # -- binding ----------------------------------------------------------------------------
    def bind(self, plans, device):
        self.device = torch.device(device)
        self.plans = list(plans)
        self._bound = {}  # ratio -> (plans, layouts, device plans): see set_ratio
        if self.allreduce:
            self.layouts = [None] * len(self.plans)
            return self
        lk = "qsgd" if self.kind == "qsgd" else self.kind
        if self.kind in ("topk", "topk_qsgd"):
            # the plans carry k; rebuild with this codec's ratio if needed
            self.plans = [p if (p.ratio == self.ratio and p.dense_below == self.dense_below)
                          else BucketPlan(p.numels, p.offsets, self.ratio, p.bucket_offset,
                                          p.length, self.dense_below) for p in self.plans]
        self.layouts = [Layout.build(lk, p, self.bits) for p in self.plans]
        if self.device.type == "cuda":
            if ops.hip_required():
                ops.require()
            self.dplans = [ops.DevicePlan(p, self.device) for p in self.plans]
        self._bound[self.ratio] = (self.plans, self.layouts, self.dplans)
        return self

    def set_ratio(self, ratio: float):
        """Switch a bound top-k codec to another density (top-k warm-up): the per-tensor k, the
        payload layouts and the device tables change; bindings are cached per ratio."""
        if self.kind not in ("topk", "topk_qsgd"):
            raise ValueError("only top-k codecs have a density")
        if not 0.0 < ratio <= 1.0:
            raise ValueError("top-k ratio must be in (0, 1]")
        if ratio == self.ratio:
            return self
        hit = self._bound.get(ratio)
        if hit is None:
            plans = [BucketPlan(p.numels, p.offsets, ratio, p.bucket_offset, p.length,
                                self.dense_below) for p in self.plans]
            layouts = [Layout.build(self.kind, p, self.bits) for p in plans]
            dplans = ([ops.DevicePlan(p, self.device) for p in plans]
                      if self.device.type == "cuda" else [])
            hit = self._bound[ratio] = (plans, layouts, dplans)
        self.ratio = ratio
        self.plans, self.layouts, self.dplans = hit
        return self

    def payload_bytes(self, b: int) -> int:
        if self.allreduce:
            p = self.plans[b]
            return p.length * self.wire_dtype.itemsize
        return self.layouts[b].nbytes

    def dense_bytes(self, b: int) -> int:
        return self.plans[b].numel * 4

    def key(self, step: int, rank: int) -> int:
        return stream_key(self.seed, step, rank)

    # -- encode / decode ----------------------------------------------------------------------
    def encode(self, b: int, grad: torch.Tensor, payload: torch.Tensor, step: int, rank: int,
               resid: torch.Tensor = None, key_tensor: torch.Tensor = None, dgc: dict = None,
               ef21: bool = False, apply: dict = None):
        """Compress bucket ``b`` of the flat gradient (``grad`` = that bucket's view).  ``dgc``:
        error feedback with momentum correction (top-k codecs; ``oracle.dgc_accumulate``).
        ``apply`` (GPU top-k, a world of one): the encode also applies the decoded update
        (``ops.topk_encode``), so no decode launch follows."""
        if dgc is not None and (resid is None or self.kind not in ("topk", "topk_qsgd")):
            raise ValueError("momentum correction needs a top-k codec and a residual")
        plan, lay = self.plans[b], self.layouts[b]
        key = self.key(step, rank)
        on_dev = (grad[0] if isinstance(grad, (list, tuple)) else grad).is_cuda
        if ef21 and (resid is None or self.kind not in ("topk", "topk_qsgd")):
            raise ValueError("EF21 needs a top-k codec and the gradient estimate")
        if on_dev and not _FORCE_ORACLE:
            if ef21:
                raise NotImplementedError("EF21 encode on the GPU: run with EWDML_ORACLE=1")
            if self.kind == "qsgd":
                ops.qsgd_encode(self.dplans[b], grad, payload, lay, self.levels, self.norm, key,
                                resid, key_tensor)
            else:
                ops.topk_encode(self.dplans[b], grad, payload, lay, self.levels, self.norm, key,
                                resid, key_tensor, dgc=dgc, apply=apply)
            return
        if apply is not None:
            raise ValueError("the encode-side apply runs on the GPU codec only")
        if isinstance(grad, (list, tuple)):
            raise TypeError("CPU encode takes the bucket's flat gradient view")
        if self.kind == "qsgd":
            out = oracle.encode_qsgd(grad, plan, lay, self.levels, self.norm, key, resid)
        else:
            out = oracle.encode_topk(grad, plan, lay, self.levels, self.norm, key, resid, dgc,
                                     ef21)
        payload[:lay.nbytes].copy_(out)

    def decode(self, b: int, recv: torch.Tensor, out: torch.Tensor, scale: float):
        """``out`` (bucket view) = scale * sum over ranks of the decoded payloads in ``recv``."""
        plan, lay = self.plans[b], self.layouts[b]
        if recv.is_cuda and not _FORCE_ORACLE:
            fn = ops.qsgd_decode_apply if self.kind == "qsgd" else ops.topk_decode_apply
            fn(self.dplans[b], recv, lay, self.levels, grad_out=out, grad_scale=scale)
            return
        out[:plan.length].copy_(oracle.decode_sum(recv, plan, lay, self.levels, scale))

    def decode_apply_sgd(self, b: int, recv: torch.Tensor, scale: float, param: torch.Tensor,
                         mom: torch.Tensor, hp: dict, first: bool, grad_out=None, shadow=None,
                         key_state=None, rank: int = 0):
        """Fused decode -> average -> SGD step of bucket ``b`` (one kernel on the GPU).
        ``key_state`` (device int32 {step, key}): also advance the RNG key to the next step.
        ``mom`` may be None with ``hp["momentum"] == 0`` (momentum-corrected error feedback: the
        momentum ran on the sender, the update is p -= lr * mean)."""
        if mom is None and hp["momentum"] != 0:
            raise ValueError("a momentum step needs the momentum buffer")
        plan, lay = self.plans[b], self.layouts[b]
        if recv.is_cuda and not _FORCE_ORACLE:
            fn = ops.qsgd_decode_apply if self.kind == "qsgd" else ops.topk_decode_apply
            fn(self.dplans[b], recv, lay, self.levels, param=param, mom=mom, grad_out=grad_out,
               lr=hp["lr"], momentum=hp["momentum"], dampening=hp["dampening"],
               weight_decay=hp["weight_decay"], grad_scale=scale, nesterov=hp["nesterov"],
               first=first, shadow=shadow, key_state=key_state, key_seed=self.seed,
               key_rank=rank, lr_tensor=hp.get("lr_t"))
            return
        g = oracle.decode_sum(recv, plan, lay, self.levels, scale)
        if grad_out is not None:
            grad_out[:plan.length].copy_(g)
        for off, n in zip(plan.offsets, plan.numels):
            oracle.sgd_apply(param[off:off + n], None if mom is None else mom[off:off + n],
                             g[off:off + n], hp["lr"],
                             hp["momentum"], hp["dampening"], hp["weight_decay"],
                             hp["nesterov"], first)


def make_codec(kind: str = "topk_qsgd", **kw) -> Codec:
    return Codec(kind, **kw)
