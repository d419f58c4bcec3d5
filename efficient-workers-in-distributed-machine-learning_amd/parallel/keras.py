"""Keras-style ``fit`` loop and the Horovod Keras callbacks, on the ewdml Horovod API.

The reference's TF/Keras example (``tensorflow_mnist.py:5-79``) trains through
``horovod.tensorflow.keras``: ``hvd.DistributedOptimizer(opt, backward_passes_per_step=1,
average_aggregated_gradients=True)`` (``:42-43``), the callbacks
``BroadcastGlobalVariablesCallback(0)`` (``:56``), ``MetricAverageCallback()`` (``:62``),
``LearningRateWarmupCallback(initial_lr=scaled_lr, warmup_epochs=3, verbose=1)`` (``:67``), a
rank-0-only ``ModelCheckpoint('./checkpoint-{epoch}.h5')`` (``:71-72``) and
``model.fit(dataset, steps_per_epoch=500 // hvd.size(), callbacks=..., epochs=24, verbose=...)``
(``:79``).  TensorFlow is not part of this stack (PyTorch-ROCm on MI355X), so this module gives the
same training contract to PyTorch modules: :func:`fit` runs the epochs/steps loop and calls the
callbacks at the Keras hook points; the callbacks do what Horovod's do, through
:mod:`ewdml.parallel.horovod` (RCCL on GPU, Gloo on CPU).

Semantics kept from Horovod's Keras callbacks:

* ``BroadcastGlobalVariablesCallback(root)``: parameters, buffers and optimizer state from
  ``root`` before the first batch (Horovod TF2 does it after the first batch only because Keras
  creates variables lazily; PyTorch modules exist up front).
* ``MetricAverageCallback()``: every metric in the epoch logs is averaged over ranks at epoch end,
  before the callbacks after it read them.
* ``LearningRateWarmupCallback(initial_lr, warmup_epochs, momentum_correction, steps_per_epoch)``:
  per batch during warm-up, ``lr = initial_lr / size * (e * (size - 1) / warmup_epochs + 1)`` with
  ``e = epoch + (batch + 1) / steps_per_epoch`` (Goyal et al., 2017: from ``initial_lr / size`` to
  ``initial_lr`` over the warm-up), momentum scaled by ``new_lr / old_lr`` for the batch in which
  the lr changes (momentum correction), ``initial_lr`` from the end of warm-up on.
* ``ModelCheckpoint(filepath)``: ``filepath.format(epoch=epoch + 1, **logs)`` on rank 0 only.
"""
from typing import Callable, Dict, Iterable, List, Optional

import torch

from . import horovod as hvd


class Callback:
    """Keras hook points.  ``self.model`` / ``self.optimizer`` / ``self.params`` are set by
    :func:`fit` before ``on_train_begin``."""

    model = None
    optimizer = None
    params: Dict = {}

    def on_train_begin(self, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass

    def on_batch_begin(self, batch, logs=None):
        pass

    def on_batch_end(self, batch, logs=None):
        pass


def _inner(opt):
    return getattr(opt, "optimizer", opt)  # the DistributedOptimizer's wrapped optimizer


class BroadcastGlobalVariablesCallback(Callback):
    def __init__(self, root_rank: int = 0):
        self.root_rank = root_rank

    def on_train_begin(self, logs=None):
        hvd.broadcast_parameters(self.model.state_dict(), root_rank=self.root_rank)
        hvd.broadcast_optimizer_state(_inner(self.optimizer), root_rank=self.root_rank)


class MetricAverageCallback(Callback):
    def on_epoch_end(self, epoch, logs=None):
        if not logs:
            return
        keys = sorted(k for k, v in logs.items() if isinstance(v, (int, float)))
        vals = hvd._comm().all_reduce_scalars([float(logs[k]) for k in keys], op="sum")
        for k, v in zip(keys, vals):
            logs[k] = v / hvd.size()


class LearningRateWarmupCallback(Callback):
    """Horovod's linear LR warm-up (``tensorflow_mnist.py:65-66``).  Horovod's momentum
    correction (momentum *= new_lr / old_lr while the lr changes) exists because Keras SGD keeps
    the lr inside its velocity (v = m v - lr g).  torch.optim.SGD applies the lr outside the
    buffer (p -= lr * buf), so an lr change already rescales the whole history: there the
    correction would double-scale momentum, and it is applied only to optimizers that declare
    ``lr_in_velocity = True``."""

    def __init__(self, initial_lr: float, warmup_epochs: int = 5, momentum_correction: bool = True,
                 steps_per_epoch: Optional[int] = None, verbose: int = 0):
        self.initial_lr = float(initial_lr)
        self.warmup_epochs = warmup_epochs
        self.momentum_correction = momentum_correction
        self.steps_per_epoch = steps_per_epoch
        self.verbose = verbose
        self.epoch = 0
        self._restore = None

    def multiplier(self, epoch: float) -> float:
        size = hvd.size()
        return 1.0 / size * (epoch * (size - 1) / self.warmup_epochs + 1)

    def on_train_begin(self, logs=None):
        if self.steps_per_epoch is None:
            self.steps_per_epoch = self.params.get("steps")

    def on_epoch_begin(self, epoch, logs=None):
        self.epoch = epoch

    def on_batch_begin(self, batch, logs=None):
        if self.epoch >= self.warmup_epochs:
            return
        e = self.epoch + (batch + 1) / float(self.steps_per_epoch)
        new_lr = self.initial_lr * self.multiplier(e)
        opt = _inner(self.optimizer)
        self._restore = []
        for g in opt.param_groups:
            old = g["lr"]
            g["lr"] = new_lr
            if (self.momentum_correction and getattr(opt, "lr_in_velocity", False)
                    and g.get("momentum") and old > 0 and old != new_lr):
                self._restore.append((g, g["momentum"]))
                g["momentum"] = g["momentum"] * new_lr / old

    def on_batch_end(self, batch, logs=None):
        for g, m in self._restore or ():
            g["momentum"] = m
        self._restore = None

    def on_epoch_end(self, epoch, logs=None):
        if epoch == self.warmup_epochs - 1:
            for g in _inner(self.optimizer).param_groups:
                g["lr"] = self.initial_lr
            if self.verbose and hvd.rank() == 0:
                print(f"Epoch {epoch + 1}: finished gradual learning rate warmup to "
                      f"{self.initial_lr:g}.")
        if logs is not None:
            logs["lr"] = _inner(self.optimizer).param_groups[0]["lr"]


class ModelCheckpoint(Callback):
    """Saves ``model.state_dict()`` (safetensors-free torch.save of tensors only, loadable with
    ``weights_only=True``) at every epoch end; put it in the list on rank 0 only, as the
    reference does (``tensorflow_mnist.py:71-72``)."""

    def __init__(self, filepath: str):
        self.filepath = filepath
        self.saved: List[str] = []

    def on_epoch_end(self, epoch, logs=None):
        path = self.filepath.format(epoch=epoch + 1, **(logs or {}))
        torch.save({k: v.detach().cpu() for k, v in self.model.state_dict().items()}, path)
        self.saved.append(path)


class History(Callback):
    def __init__(self):
        self.history: Dict[str, List[float]] = {}

    def on_epoch_end(self, epoch, logs=None):
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


def fit(model: torch.nn.Module, data: Iterable, optimizer, loss_fn: Callable, epochs: int = 1,
        steps_per_epoch: Optional[int] = None, callbacks: Optional[List[Callback]] = None,
        verbose: int = 1, device=None) -> History:
    """Keras ``Model.fit`` for a PyTorch module: ``data`` yields ``(x, y)`` batches (an endless
    iterator with ``steps_per_epoch``, or an iterable re-entered each epoch), ``optimizer`` is
    typically :func:`ewdml.parallel.horovod.DistributedOptimizer`.  Logs per epoch: mean loss and
    accuracy over the epoch's batches (this rank's; :class:`MetricAverageCallback` averages them
    over ranks)."""
    hist = History()
    cbs = list(callbacks or []) + [hist]
    params = {"epochs": epochs, "steps": steps_per_epoch, "verbose": verbose}
    for cb in cbs:
        cb.model, cb.optimizer, cb.params = model, optimizer, params
    it = iter(data) if steps_per_epoch is not None else None
    model.train()
    for cb in cbs:
        cb.on_train_begin({})
    for epoch in range(epochs):
        for cb in cbs:
            cb.on_epoch_begin(epoch, {})
        src = it if it is not None else iter(data)
        tot = torch.zeros(3, dtype=torch.float64, device=device)  # loss sum, correct, samples
        step = 0
        while steps_per_epoch is None or step < steps_per_epoch:
            try:
                x, y = next(src)
            except StopIteration:
                break
            for cb in cbs:
                cb.on_batch_begin(step, {})
            optimizer.zero_grad()
            out = model(x)
            loss = loss_fn(out, y)
            loss.backward()
            optimizer.step()
            with torch.no_grad():
                tot[0] += loss.detach().double() * y.shape[0]
                tot[1] += (out.argmax(1) == y).sum().double()
                tot[2] += y.shape[0]
            for cb in cbs:
                cb.on_batch_end(step, {})
            step += 1
        n = max(float(tot[2]), 1.0)
        logs = {"loss": float(tot[0]) / n, "accuracy": float(tot[1]) / n}
        for cb in cbs:
            cb.on_epoch_end(epoch, logs)
        if verbose and hvd.rank() == 0:
            print(f"Epoch {epoch + 1}/{epochs} - " +
                  " - ".join(f"{k}: {v:.4f}" for k, v in logs.items()), flush=True)
    for cb in cbs:
        cb.on_train_end({})
    return hist


class callbacks:  # noqa: N801 - the ``hvd.callbacks.X`` spelling of the reference
    BroadcastGlobalVariablesCallback = BroadcastGlobalVariablesCallback
    MetricAverageCallback = MetricAverageCallback
    LearningRateWarmupCallback = LearningRateWarmupCallback
