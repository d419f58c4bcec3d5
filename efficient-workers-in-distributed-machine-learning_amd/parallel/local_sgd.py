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
    ``select_best`` every rank -- the winner included -- sets its weights to
    ``anchor + decode(payload of the best rank)``, which the all-gather already delivered:
    adopting the winner costs no extra weight traffic, only its BN statistics (counted), and the
    replicas stay bitwise identical.  The adoption is lossy by the codec's error: the part of the
    winner's delta that top-k dropped is not applied at this sync.  With error feedback (the
    default for top-k codecs) it is not lost either: the winner keeps it in its residual and
    sends it with its next delta, while the other ranks zero their residuals (their own unsent
    drift belongs to a trajectory that was abandoned).
  * ``grad`` -- on sync steps the step's gradient goes through the wrapped exchange (compressed,
    averaged, applied); other steps apply the local gradient.  The replicas have drifted apart
    over the local steps and the same averaged gradient does not bring them back, so the weights
    of rank 0 (or of the best rank with ``select_best``) are broadcast densely at every sync
    point (counted; the reference's commented code never re-synchronised).
The best rank is measured on a fixed held-out batch (``score_fn``).

With pointer-mode gradients (``FlatModel(attach_grads=False)``, the GPU default) a local step
reads autograd's gradient tensors in place: one fused SGD launch per bucket (``ops.sgd_ptrs``), or
a gather into ``flat.grad`` per bucket for other optimizers -- never the per-parameter
accumulate-adds of attached ``.grad`` views.  The model delta of a sync step is staged in
``flat.grad`` and the wrapped exchange encodes from there (``src_flat``).
"""
import torch

from .. import ops
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
        self.best_t = None  # device index of the last sync's winner (model mode)
        self._plans = None  # pointer mode: per-bucket device plans of the local step
        self.clock = None  # Stopwatch of --phase-timing (the trainer sets it here and on inner)

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
            if self.clock is not None:
                self.clock.mark("backward")
            self.local_step()  # with the rank's own gradient
            if self.clock is not None:
                self.clock.mark("decode_update")
            if sync:  # model mode
                delta = self.flat.grad
                torch.sub(self.flat.data, self.anchor, out=delta)
                self.inner.src_flat = True
                try:
                    self.inner.begin()
                    self.inner.finish(apply=False)
                finally:
                    self.inner.src_flat = False
                stats = self.inner.bytes_per_step()
                if self.select_best and (self.comm.world > 1 or self.comm.kind != "local"):
                    # every rank holds every rank's compressed delta: apply the winner's.  The
                    # choice stays on the device (scores all-gathered, argmax, the winner's
                    # payload row and BN buffers selected by index), so this step has no host
                    # round trip and is captured as a HIP graph like the local steps
                    best = self._best_dev()
                    self.inner.decode_rank(best)
                    resid = self.inner.resid
                    if resid is not None:  # only the winner's unsent delta carries over
                        won = (best == self.comm.rank).to(resid.dtype)
                        resid.mul_(won)
                    buf = self._sync_bn_dev(best)
                    stats.wire_bytes_sent += (self.comm.world - 1) * buf
                    stats.wire_bytes_recv += (self.comm.world - 1) * buf
                else:
                    self.inner.decode_average()
                torch.add(self.anchor, self.flat.grad, out=self.flat.data)
                self.anchor.copy_(self.flat.data)
                self.flat.sync_shadow()
                if self.clock is not None:
                    self.clock.mark("decode_update")
        self.last = stats
        self.step_idx += 1

    def local_step(self):
        """Optimizer step with this rank's own gradient."""
        flat = self.flat
        if flat.attach_grads:
            self.opt.step(grad=flat.grad)
            return
        if self._plans is None:
            self._plans = [ops.DevicePlan(b.plan, flat.data.device) for b in flat.buckets]
        if getattr(self.opt, "fusable", False):
            for b, dp in zip(flat.buckets, self._plans):
                self.opt.step_bucket_ptrs(b, dp, flat.bucket_grads(b))
            self.opt.end_step()
            return
        for b, dp in zip(flat.buckets, self._plans):  # other optimizers: gather, then step
            ops.pack_grads(dp, flat.bucket_grads(b), flat.grad_view(b))
        self.opt.step(grad=flat.grad)

    def _best(self) -> int:
        score = float(self.score_fn()) if self.score_fn is not None else 0.0
        scores = self.comm.all_gather_object(score)
        best = max(range(len(scores)), key=lambda r: (scores[r], -r))
        self.best_rank_history.append(best)
        return best

    def _best_dev(self) -> torch.Tensor:
        """Index (int64 [1], on the device) of the rank with the highest held-out score, lowest
        rank on ties -- the same choice as :meth:`_best` without leaving the device."""
        dev = self.flat.data.device
        s = self.score_fn() if self.score_fn is not None else 0.0
        s = torch.as_tensor(s, dtype=torch.float32, device=dev).reshape(1)
        scores = torch.empty(self.comm.world, dtype=torch.float32, device=dev)
        self.comm.all_gather(scores, s)
        best = torch.argmax(scores).reshape(1)  # first maximum: lowest rank on ties
        if not (dev.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            self.best_rank_history.append(int(best))
        self.best_t = best
        return best

    def _sync_bn_dev(self, best: torch.Tensor) -> int:
        """Every rank takes rank ``best``'s buffers (BN running statistics): one all-gather per
        buffer dtype and an index select on the device.  Returns the bytes per rank."""
        model = self.flat.model
        if model is None:
            return 0
        groups = {}
        for b in model.buffers():
            if b.dtype.is_floating_point or b.dtype in (torch.int64, torch.int32):
                groups.setdefault(b.dtype, []).append(b)
        nbytes = 0
        for dt, bufs in groups.items():
            mine = torch.cat([b.detach().reshape(-1) for b in bufs])
            allb = torch.empty(self.comm.world * mine.numel(), dtype=dt, device=mine.device)
            self.comm.all_gather(allb, mine)
            win = allb.view(self.comm.world, -1).index_select(0, best)[0]
            o = 0
            for b in bufs:
                b.data.copy_(win[o:o + b.numel()].view_as(b))
                o += b.numel()
            nbytes += mine.numel() * mine.element_size()
        return nbytes

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
