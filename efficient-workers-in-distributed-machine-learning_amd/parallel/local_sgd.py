"""Periodic synchronisation (local SGD) -- reference Method 6.

The report's Method 6 (``Report.zip:main.tex:119,156``; commented code in
``distributed_worker.py:197-209``, ``sync_replicas_master_nn.py:166-171``, ``capture_grad``
``:306-314``) lets every worker apply its own gradient and communicates only every 20 iterations,
after which all workers adopt the weights of the worker with the best test accuracy.  The reference
has no code for the best-worker selection; it is implemented here.

Modes:
  * ``grad``  -- on sync steps the step's gradient goes through the wrapped exchange (compressed,
    averaged, applied); other steps apply the local gradient.
  * ``model`` -- local steps everywhere; on sync steps each rank compresses its *model delta*
    since the last sync with the wrapped exchange's codec, the deltas are averaged and added to the
    common anchor (compressed model averaging).
``select_best`` then broadcasts the weights (and BN statistics) of the best rank, measured on a
fixed held-out batch.  Those bytes are counted (the report's 1.48 MB figure omits them).  In
``grad`` mode without ``select_best`` the replicas have drifted apart over the local steps and the
same averaged gradient does not bring them back, so rank 0's weights are broadcast at every sync
point (counted the same way; the reference's commented code never re-synchronised).
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
        if sync and self.mode == "grad":
            self.inner.finish()
        else:
            self.opt.step(grad=self.flat.grad)  # local step with the rank's own gradient
            if sync:  # model mode
                delta = self.flat.grad
                torch.sub(self.flat.data, self.anchor, out=delta)
                self.inner.begin()
                self.inner.finish(apply=False)
                self.inner.decode_average()
                torch.add(self.anchor, self.flat.grad, out=self.flat.data)
                self.anchor.copy_(self.flat.data)
        stats = StepStats()
        if sync:
            stats = self.inner.bytes_per_step()
            src = None
            if self.select_best and self.comm.world > 1:
                self._adopt_best()
                src = self.best_rank_history[-1]
            elif self.mode == "grad" and self.comm.world > 1:
                self._adopt(0)  # re-converge the drifted replicas on rank 0's weights
                src = 0
            if src is not None:
                n = self.flat.numel * 4
                stats.wire_bytes_sent += n if self.comm.rank == src else 0
                stats.wire_bytes_recv += 0 if self.comm.rank == src else n
        self.last = stats
        self.step_idx += 1

    def _adopt_best(self):
        score = float(self.score_fn()) if self.score_fn is not None else 0.0
        scores = self.comm.all_gather_object(score)
        best = max(range(len(scores)), key=lambda r: (scores[r], -r))
        self.best_rank_history.append(best)
        self._adopt(best)

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
