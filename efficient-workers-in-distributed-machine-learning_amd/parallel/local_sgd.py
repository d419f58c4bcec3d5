"""Periodic synchronisation (local SGD) -- reference Method 6.

The report's Method 6 (``Report.zip:main.tex:119,156``; commented code in
``distributed_worker.py:197-209``, ``sync_replicas_master_nn.py:166-171``, ``capture_grad``
``:306-314``) lets every worker apply its own gradient and communicates only every 20 iterations,
after which all workers adopt the weights of the worker with the best test accuracy.  The reference
has no code for the best-worker selection; it is implemented here.

Modes:
  * ``model`` (Method 6's default) -- local steps everywhere; on sync steps each rank compresses
    its *model delta* since the last sync with the wrapped exchange's codec and all-gathers it;
    the deltas are averaged and added to the common anchor (compressed model averaging).  With
    ``select_best`` every rank instead applies the *best rank's* compressed delta, which the
    all-gather already delivered: adopting the winner costs no extra weight traffic, only its BN
    statistics (counted).
  * ``grad`` -- on sync steps the step's gradient goes through the wrapped exchange (compressed,
    averaged, applied); other steps apply the local gradient.  The replicas have drifted apart
    over the local steps and the same averaged gradient does not bring them back, so the weights
    of rank 0 (or of the best rank with ``select_best``) are broadcast densely at every sync
    point (counted; the reference's commented code never re-synchronised).
The best rank is measured on a fixed held-out batch (``score_fn``).
"""
import torch

from .engine import StepStats, sync_buffers


class LocalSGDExchange:
    def __init__(self, inner, every: int, mode: str = "grad", select_best: bool = False,
                 score_fn=None):
        if every < 1:
            raise ValueError("sync_every must be >= 1")
        self.inner, self.every, self.mode = inner, every, mode
        self.select_best, self.score_fn = select_best, score_fn
        self.flat, self.comm, self.opt = inner.flat, inner.comm, inner.opt
        self.step_idx = 0
        self.anchor = self.flat.data.clone() if mode == "model" else None
        self.last = StepStats()
        self.best_rank_history = []

    @property
    def is_sync(self) -> bool:
        return (self.step_idx + 1) % self.every == 0

    def begin(self):
        if self.is_sync and self.mode == "grad":
            self.inner.begin()

    def finish(self):
        sync = self.is_sync
        stats = StepStats()
        if sync and self.mode == "grad":
            self.inner.finish()
            stats = self.inner.bytes_per_step()
            if self.comm.world > 1:
                # re-converge the drifted replicas on the best (or rank 0's) dense weights
                src = self._best() if self.select_best else 0
                self._adopt(src)
                n = self.flat.numel * 4
                stats.wire_bytes_sent += n if self.comm.rank == src else 0
                stats.wire_bytes_recv += 0 if self.comm.rank == src else n
        else:
            self.opt.step(grad=self.flat.grad)  # local step with the rank's own gradient
            if sync:  # model mode
                delta = self.flat.grad
                torch.sub(self.flat.data, self.anchor, out=delta)
                self.inner.begin()
                self.inner.finish(apply=False)
                stats = self.inner.bytes_per_step()
                if self.select_best and self.comm.world > 1:
                    # every rank holds every rank's compressed delta: apply the winner's
                    src = self._best()
                    self.inner.decode_rank(src)
                    buf = self._sync_bn(src)
                    stats.wire_bytes_sent += buf if self.comm.rank == src else 0
                    stats.wire_bytes_recv += 0 if self.comm.rank == src else buf
                else:
                    self.inner.decode_average()
                torch.add(self.anchor, self.flat.grad, out=self.flat.data)
                self.anchor.copy_(self.flat.data)
                self.flat.sync_shadow()
        self.last = stats
        self.step_idx += 1

    def _best(self) -> int:
        score = float(self.score_fn()) if self.score_fn is not None else 0.0
        scores = self.comm.all_gather_object(score)
        best = max(range(len(scores)), key=lambda r: (scores[r], -r))
        self.best_rank_history.append(best)
        return best

    def _sync_bn(self, src: int) -> int:
        """Broadcast the model's buffers (BN running statistics) from ``src``; returns bytes."""
        if self.flat.model is None:
            return 0
        sync_buffers(self.flat.model, self.comm, src=src)
        return sum(b.numel() * b.element_size() for b in self.flat.model.buffers()
                   if b.dtype.is_floating_point or b.dtype in (torch.int64, torch.int32))

    def _adopt(self, src: int):
        self.comm.broadcast(self.flat.data, src=src)
        self.flat.sync_shadow()
        if self.flat.model is not None:
            sync_buffers(self.flat.model, self.comm, src=src)
        if self.anchor is not None:
            self.anchor.copy_(self.flat.data)

    def bytes_per_step(self):
        return self.inner.bytes_per_step()

    def close(self):
        self.inner.close()
