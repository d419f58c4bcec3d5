"""Optimizers over the flat parameter buffer with *explicit* gradients.

Parity: ``optim/sgd.py:11-91`` (SGD whose ``step(grads=...)`` takes the averaged gradient received
from the server; momentum buffer initialised to the first gradient, dampening, Nesterov, weight
decay) and ``optim/adam.py:12-94`` (Adam/AMSGrad with explicit gradients).  The reference loops
over parameter tensors; these run one HIP kernel over a flat range (``ops.sgd_flat`` /
``ops.adam_flat``), and the top-k / QSGD exchanges fuse the SGD update into their decode kernel
(``Codec.decode_apply_sgd``) so the averaged gradient never round-trips through HBM.
"""
import math

import torch

from .. import ops
from ..compress import oracle


class DeviceScalar:
    """An fp32 scalar in device memory that the kernels read at run time (a captured HIP graph
    keeps its kernels' arguments frozen, so a learning-rate schedule is fed through this), updated
    by stream-ordered copies from a ring of pinned host slots (no host synchronisation)."""

    def __init__(self, value: float, device):
        self.t = torch.full((1,), float(value), dtype=torch.float32, device=device)
        self._ring = [(torch.zeros(1, dtype=torch.float32).pin_memory(), None) for _ in range(8)]
        self._slot = 0

    def set(self, value: float):
        host, ev = self._ring[self._slot]
        if ev is not None:
            ev.synchronize()  # the slot's previous copy has been consumed
        host[0] = float(value)
        self.t.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ring[self._slot] = (host, ev)
        self._slot = (self._slot + 1) % len(self._ring)


class _LrMixin:
    """``lr`` as a host value mirrored into ``lr_t`` (device) on the GPU."""

    @property
    def lr(self) -> float:
        return self._lr

    @lr.setter
    def lr(self, value: float):
        self._lr = float(value)
        dev = getattr(self, "_lr_dev", None)
        if dev is not None:
            dev.set(self._lr)

    @property
    def lr_t(self):
        dev = getattr(self, "_lr_dev", None)
        return None if dev is None else dev.t

    def _init_lr(self, lr, device):
        self._lr_dev = DeviceScalar(lr, device) if device.type == "cuda" else None
        self._lr = float(lr)


class FlatSGD(_LrMixin):
    fusable = True

    def __init__(self, flat, lr=0.01, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        self.flat = flat
        self._init_lr(lr, flat.data.device)
        self.momentum, self.dampening = momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        self.mom = torch.zeros_like(flat.data)
        self.steps = 0

    @property
    def first(self) -> bool:
        return self.steps == 0

    def hparams(self) -> dict:
        return dict(lr=self.lr, momentum=self.momentum, dampening=self.dampening,
                    weight_decay=self.weight_decay, nesterov=self.nesterov, lr_t=self.lr_t)

    def step_range(self, start: int, length: int, grad: torch.Tensor, grad_scale: float = 1.0):
        """Apply SGD to ``flat.data[start:start+length]`` with ``grad`` (same length) * scale."""
        p = self.flat.data[start:start + length]
        m = self.mom[start:start + length]
        if p.is_cuda:
            sh = self.flat.shadow[start:start + length] if self.flat.shadow is not None else None
            ops.sgd_flat(p, m, grad, self.lr, self.momentum, self.dampening, self.weight_decay,
                         grad_scale, self.nesterov, self.first, shadow=sh, lr_tensor=self.lr_t)
            return
        g = grad.to(torch.float32)
        if grad_scale != 1.0:
            g = g * grad_scale
        oracle.sgd_apply(p, m, g, self.lr, self.momentum, self.dampening, self.weight_decay,
                         self.nesterov, self.first)

    def step(self, grad: torch.Tensor = None, grad_scale: float = 1.0):
        """Whole-model step (``grad`` defaults to the flat gradient buffer)."""
        self.step_range(0, self.flat.numel, self.flat.grad if grad is None else grad, grad_scale)
        self.end_step()

    def step_bucket_ptrs(self, b, dp, grads, grad_scale: float = 1.0):
        """SGD of bucket ``b`` from its per-tensor gradients ``grads`` (pointer mode), one
        launch; no :meth:`end_step`."""
        p = self.flat.data_view(b)
        m = self.mom[b.start:b.start + b.length]
        ops.sgd_ptrs(dp, grads, p, m, self.lr, self.momentum, self.dampening, self.weight_decay,
                     grad_scale, self.nesterov, self.first, shadow=self.flat.shadow_view(b),
                     lr_tensor=self.lr_t)

    def end_step(self):
        self.steps += 1

    def state_dict(self):
        hp = {k: v for k, v in self.hparams().items() if k != "lr_t"}
        return {"kind": "sgd", "mom": self.mom, "steps": self.steps, **hp}

    def load_state_dict(self, sd):
        self.mom.copy_(sd["mom"])
        self.steps = int(sd["steps"])
        for k in ("lr", "momentum", "dampening", "weight_decay", "nesterov"):
            if k in sd:
                setattr(self, k, sd[k])


class FlatAdam(_LrMixin):
    fusable = False

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False):
        self.flat = flat
        self._init_lr(lr, flat.data.device)
        self.betas, self.eps = betas, eps
        self.weight_decay, self.amsgrad = weight_decay, amsgrad
        self.exp_avg = torch.zeros_like(flat.data)
        self.exp_avg_sq = torch.zeros_like(flat.data)
        self.max_exp_avg_sq = torch.zeros_like(flat.data) if amsgrad else None
        self.steps = 0
        # device copy of the step count: the kernel derives the bias correction from it, so a
        # captured HIP graph replays the current step's correction (not the capture step's)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=flat.data.device) \
            if flat.data.is_cuda else None

    def step_range(self, start, length, grad, grad_scale=1.0):
        t = self.steps + 1
        b1, b2 = self.betas
        sl = slice(start, start + length)
        p = self.flat.data[sl]
        vmax = self.max_exp_avg_sq[sl] if self.amsgrad else None
        if p.is_cuda:
            lr_step = self.lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
            sh = self.flat.shadow[sl] if self.flat.shadow is not None else None
            ops.adam_flat(p, self.exp_avg[sl], self.exp_avg_sq[sl], vmax, grad, lr_step, b1, b2,
                          self.eps, self.weight_decay, grad_scale, self.amsgrad, shadow=sh,
                          step=self.step_t, lr=self.lr, lr_tensor=self.lr_t)
            return
        g = grad.to(torch.float32) * grad_scale
        oracle.adam_apply(p, self.exp_avg[sl], self.exp_avg_sq[sl],
                          vmax if vmax is not None else torch.empty(0), g, self.lr, b1, b2,
                          self.eps, self.weight_decay, t, self.amsgrad)

    def step(self, grad=None, grad_scale=1.0):
        self.step_range(0, self.flat.numel, self.flat.grad if grad is None else grad, grad_scale)
        self.end_step()

    def end_step(self):
        self.steps += 1
        if self.step_t is not None:
            self.step_t.add_(1)  # on the stream: captured into the step graph

    def state_dict(self):
        return {"kind": "adam", "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "max_exp_avg_sq": self.max_exp_avg_sq, "steps": self.steps, "lr": self.lr}

    def load_state_dict(self, sd):
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        if self.amsgrad and sd.get("max_exp_avg_sq") is not None:
            self.max_exp_avg_sq.copy_(sd["max_exp_avg_sq"])
        self.steps = int(sd["steps"])
        if self.step_t is not None:
            self.step_t.fill_(self.steps)
        self.lr = sd.get("lr", self.lr)


def make_optimizer(name, flat, **kw):
    name = name.lower()
    if name == "sgd":
        return FlatSGD(flat, **{k: v for k, v in kw.items()
                                if k in ("lr", "momentum", "dampening", "weight_decay",
                                         "nesterov")})
    if name in ("adam", "amsgrad"):
        return FlatAdam(flat, lr=kw.get("lr", 1e-3), weight_decay=kw.get("weight_decay", 0.0),
                        amsgrad=(name == "amsgrad") or kw.get("amsgrad", False))
    raise ValueError(f"unknown optimizer {name!r}")
