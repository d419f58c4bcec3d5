"""Gradient exchange engine: buckets, comm/backward overlap, fused apply.

Per step (``begin`` -> ``loss.backward()`` -> ``finish``):

1. As autograd finishes accumulating the last gradient of a bucket, a post-accumulate hook
   records an event on the compute stream and, on a side HIP stream that waits on it, runs the
   codec's encode kernels and issues the bucket's collective (RCCL all-gather of the packed
   payloads, or all-reduce for dense codecs).  Backward of the earlier layers keeps running on the
   compute stream meanwhile -- the overlap that the reference only prototyped with per-layer MPI
   ``Isend`` in ``LeNetSplit.backward_normal`` (``model_ops/lenet.py:111-186``).  Captured steps
   (``side_stream=False``) issue the same work at the same point on the compute stream: a fork
   would turn the step graph into a DAG, which ROCm replays node by node from the host.
2. ``finish`` makes the compute stream wait for every collective, then per bucket runs ONE fused
   kernel: decode all N payloads in rank order -> scale 1/N -> SGD update of that bucket's
   parameters (``Codec.decode_apply_sgd``).  Dense codecs get one flat SGD kernel.

Every rank decodes the same bytes in the same order, so replicas stay bitwise identical without
re-broadcasting weights.  That is the all-to-all counterpart of the reference's star
(``sync_replicas_master_nn.py:158-232``: gather -> sum -> /(N-1) -> broadcast) with no idle server.
"""
import contextlib
import time

import torch

from .. import ops


class StepStats:
    __slots__ = ("payload_bytes", "wire_bytes_sent", "wire_bytes_recv", "dense_bytes",
                 "collectives")

    def __init__(self):
        self.payload_bytes = 0
        self.wire_bytes_sent = 0
        self.wire_bytes_recv = 0
        self.dense_bytes = 0
        self.collectives = 0


class GradientExchange:
    """All-to-all exchange: all-reduce for dense codecs, all-gather of payloads otherwise."""

    def __init__(self, flat, comm, codec, optimizer, overlap: bool = True,
                 error_feedback: bool = False, predivide: float = 1.0, seed_offset: int = 0,
                 side_stream: bool = True, ef_mode: str = "dgc"):
        self.flat, self.comm, self.codec, self.opt = flat, comm, codec, optimizer
        self.device = flat.data.device
        self.cuda = self.device.type == "cuda"
        self.codec.bind([b.plan for b in flat.buckets], self.device)
        self.nb = len(flat.buckets)
        self.N = comm.world
        self.predivide = predivide
        self.seed_offset = seed_offset
        self.payload, self.recv, self.send = [], [], []
        for b in flat.buckets:
            if codec.allreduce:
                self.payload.append(None)
                self.recv.append(None)
                self.send.append(None if codec.wire_dtype == torch.float32 else torch.zeros(
                    b.length, dtype=codec.wire_dtype, device=self.device))
            else:
                self.payload.append(None)
                self.recv.append(None)
                self.send.append(None)
        if not codec.allreduce:
            self._alloc_payloads()
        self.resid = torch.zeros_like(flat.grad) if (error_feedback and not codec.allreduce) else None
        # error feedback with momentum correction (DGC, oracle.dgc_accumulate): the sender runs the
        # momentum before top-k and keeps a per-rank velocity; the decode then steps without one.
        # Only for top-k codecs under momentum SGD (dense QSGD's residual holds just the rounding
        # error, and Adam has no velocity to correct): plain error feedback otherwise.
        # local: the same sender-side momentum without masking and with the lr inside the
        # residual (error feedback on the update).  ef21: EF21 -- every rank keeps a running
        # estimate h of its gradient and sends top-k(g - h); all ranks add the average to a
        # global estimate G and take an ordinary momentum step on G every step (no bursts).
        if ef_mode not in ("dgc", "plain", "local", "ef21"):
            raise ValueError("ef_mode must be 'dgc', 'plain', 'local' or 'ef21'")
        topk = codec.kind in ("topk", "topk_qsgd")
        sgd_m = (getattr(optimizer, "fusable", False)
                 and getattr(optimizer, "momentum", 0.0) != 0.0)
        self.dgc = self.resid is not None and ef_mode in ("dgc", "local") and topk and sgd_m
        self.dgc_mask = ef_mode == "dgc"
        self.ef21 = self.resid is not None and ef_mode == "ef21" and topk
        self.ef_mode = None if self.resid is None else (
            ef_mode if (self.dgc or self.ef21) else "plain")
        self.vel = torch.zeros_like(flat.grad) if self.dgc else None
        self.gest = torch.zeros_like(flat.grad) if self.ef21 else None  # EF21's global G
        if not flat.attach_grads and not self.cuda:
            raise ValueError("pointer-mode gradients need the HIP kernels (device tensors)")
        self._pack_plans = [ops.DevicePlan(b.plan, self.device) for b in flat.buckets] \
            if (codec.allreduce and not flat.attach_grads) else None
        self.overlap = overlap
        # overlap without side_stream: each bucket is still encoded and exchanged as soon as its
        # gradients exist (interleaved with the rest of backward), in the compute stream's order
        self.side = torch.cuda.Stream(device=self.device) \
            if (self.cuda and overlap and side_stream) else None
        self._bucket_of = flat.bucket_of()
        self._sizes = [len(b.params) for b in flat.buckets]
        self._count = [0] * self.nb
        self._launched = [False] * self.nb
        self._works = [None] * self.nb
        self._next = 0
        self._active = False
        self.step_idx = 0
        self.defer_comm = False
        # encode from flat.grad instead of autograd's tensors (local SGD's model deltas live
        # there even when the step's gradients are read through pointer tables)
        self.src_flat = False
        self.use_dev_key = False
        # device RNG state {step, key} read by the captured encode kernels; the step's last decode
        # kernel advances it in place (dev_key_advance), so graph replays need no host upload
        self.key_state = torch.zeros(2, dtype=torch.int32, device=self.device)
        self.key_dev = self.key_state[1:2]
        self.dev_key_advance = False
        self._key_ring, self._key_slot = None, 0
        self._hooks = []
        self.seg = None  # SegmentedCapture while a segmented step capture is recording
        self._final = False
        if overlap:
            for p in flat.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
                # ours flush deferred weight-gradient transforms before reading (ops/conv.py)
                p._ew_engine_hooks = getattr(p, "_ew_engine_hooks", 0) + 1
        self.last = StepStats()

    def _alloc_payloads(self):
        for b in self.flat.buckets:
            P = self.codec.payload_bytes(b.index)
            recv = torch.zeros(self.N * P, dtype=torch.uint8, device=self.device)
            # encode straight into this rank's slot of the gather buffer: an in-place
            # all-gather (RCCL: sendbuff == recvbuff + rank * count), no local copy
            r = self.comm.rank
            self.payload[b.index] = recv[r * P:(r + 1) * P]
            self.recv[b.index] = recv

    def set_ratio(self, ratio: float):
        """Top-k density warm-up: re-plan the codec and the payload buffers for ``ratio``
        (every rank switches at the same step, so the fixed-size all-gathers still match; a
        captured step graph must be re-captured)."""
        if self.codec.allreduce or ratio == self.codec.ratio:
            return False
        self.codec.set_ratio(ratio)
        self._alloc_payloads()
        return True

    # -- accounting ---------------------------------------------------------------------------
    def bytes_per_step(self) -> StepStats:
        """Algorithmic bytes of one exchange (what RCCL moves per rank, ring/direct algorithms)."""
        s = StepStats()
        N = self.N
        for b in self.flat.buckets:
            P = self.codec.payload_bytes(b.index)
            s.payload_bytes += P
            s.dense_bytes += self.codec.dense_bytes(b.index)
            if N > 1:
                if self.codec.allreduce:
                    s.wire_bytes_sent += 2 * (N - 1) * P // N
                    s.wire_bytes_recv += 2 * (N - 1) * P // N
                else:
                    s.wire_bytes_sent += (N - 1) * P
                    s.wire_bytes_recv += (N - 1) * P
                s.collectives += 1
        return s

    # -- step protocol ------------------------------------------------------------------------
    def begin(self):
        """Call before ``loss.backward()``; gradients must be zero (``flat.zero_grad()``)."""
        if self.cuda:
            from ..ops.conv import new_pass

            new_pass()  # tied-weight detection of the deferred weight-gradient transforms
        self._count = [0] * self.nb
        self._launched = [False] * self.nb
        self._works = [None] * self.nb
        self._next = 0
        self._active = True

    def _on_grad(self, p):
        if not self._active:
            return
        b = self._bucket_of[id(p)]
        self._count[b] += 1
        # Launch strictly in bucket order so every rank issues its collectives in the same
        # sequence, whatever order autograd finishes the buckets in (a mismatch would deadlock).
        ready = []
        while self._next < self.nb and self._count[self._next] >= self._sizes[self._next]:
            if not self._launched[self._next]:
                ready.append(self._next)
            self._next += 1
        if ready:
            self._launch_group(ready)

    def _stream_ctx(self):
        if self.side is None:
            return contextlib.nullcontext()
        ev = torch.cuda.Event()
        ev.record()
        self.side.wait_event(ev)
        return torch.cuda.stream(self.side)

    def _launch_group(self, bis):
        """Encode buckets ``bis`` (ready together) and (unless deferred) issue their collectives:
        on the side stream (eager overlap), in-stream (one captured graph), or -- while a
        segmented capture is recording -- as a graph of their own on the comm stream, between
        two compute segments (:class:`SegmentedCapture`)."""
        for bi in bis:
            self._launched[bi] = True
        if self.cuda:  # a deferred Winograd weight-gradient output transform completes dw first
            from ..ops.conv import flush_pending, pending

            flush_pending()
            assert not pending(), "deferred weight-gradient transform still pending at encode"
        if self.seg is not None:
            # segmented capture: buckets wait for the next split point (a byte threshold of the
            # step's gradient); their encode + collective then become one comm-stream graph
            # that overlaps the rest of backward.  Past the last split (and at the end of the
            # backward pass) they are issued in-stream, into the current compute segment.
            seg = self.seg
            seg.pending += list(bis)
            seg.ready_bytes += sum(4 * self.flat.buckets[bi].length for bi in bis)
            if seg.want_split(self._final):
                group = seg.pending
                seg.pending = []

                def issue():
                    for bi in group:
                        self._encode(bi)
                        self._works[bi] = self._collective(bi)
                seg.split(issue)
            elif self._final or seg.splits_left == 0:
                group, seg.pending = seg.pending, []
                for bi in group:
                    self._encode(bi)
                    self._works[bi] = self._collective(bi)
            return
        for bi in bis:
            with self._stream_ctx():
                self._encode(bi)
                if not self.defer_comm:
                    self._works[bi] = self._collective(bi)

    def _encode(self, bi: int):
        b = self.flat.buckets[bi]
        g = self.flat.grad_view(b) if self.src_flat else self.flat.bucket_grads(b)
        if self.codec.allreduce:
            dst = self.flat.grad_view(b) if self.send[bi] is None else self.send[bi]
            if not (self.flat.attach_grads or self.src_flat):  # one gather(+cast) kernel
                ops.pack_grads(self._pack_plans[bi], g, dst, 1.0 / self.predivide)
            elif self.send[bi] is None:
                if self.predivide != 1.0:
                    g.mul_(1.0 / self.predivide)
            elif self.cuda:
                ops.cast_scale(g, self.send[bi], 1.0 / self.predivide)
            else:
                self.send[bi].copy_(g * (1.0 / self.predivide))
            return
        resid = None if self.resid is None else self.resid[b.start:b.start + b.length]
        dgc = None
        if self.dgc:
            o = self.opt
            dgc = dict(velocity=self.vel[b.start:b.start + b.length], momentum=o.momentum,
                       dampening=o.dampening, nesterov=o.nesterov, weight_decay=o.weight_decay,
                       param=self.flat.data_view(b), mask=self.dgc_mask,
                       lr=None if self.dgc_mask else o.lr,
                       lr_t=None if self.dgc_mask else getattr(o, "lr_t", None))
        self.codec.encode(bi, g, self.payload[bi], self.step_idx + self.seed_offset,
                          self.comm.rank, resid,
                          key_tensor=self.key_dev if self.use_dev_key else None, dgc=dgc,
                          ef21=self.ef21)

    def _collective(self, bi: int):
        if self.codec.allreduce:
            t = self.flat.grad_view(self.flat.buckets[bi]) if self.send[bi] is None \
                else self.send[bi]
            return self.comm.all_reduce(t, async_op=True)
        return self.comm.all_gather(self.recv[bi], self.payload[bi], async_op=True)

    def launch_pending(self):
        rest = [bi for bi in range(self.nb) if not self._launched[bi]]
        self._final = True  # backward is over: nothing left to overlap with
        try:
            if rest or (self.seg is not None and self.seg.pending):
                self._launch_group(rest)
        finally:
            self._final = False

    def join_side(self):
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)

    def communicate(self):
        """Issue the deferred collectives (split-graph mode: outside any captured graph)."""
        for bi in range(self.nb):
            self._works[bi] = self._collective(bi)

    def wait(self):
        for w in self._works:
            if w is not None:
                w.wait()
        self._works = [None] * self.nb

    def set_device_key(self, step: int = None):
        """Upload this step's RNG state {step, key} (graph replay reads the key from device
        memory; with ``dev_key_advance`` the decode kernel moves it on to the next step)."""
        s = (self.step_idx if step is None else step) + self.seed_offset
        key = self.codec.key(s, self.comm.rank)
        vals = [((v + (1 << 31)) % (1 << 32)) - (1 << 31) for v in (s & 0xFFFFFFFF, key)]
        if self.key_state.device.type != "cuda":
            self.key_state.copy_(torch.tensor(vals, dtype=torch.int32))
            return
        # asynchronous upload from a ring of pinned slots: a pageable host->device copy would
        # block the host until the previous graph replay drained, leaving the GPU idle while the
        # next replay is launched.  A slot is reused only after its previous copy completed.
        if self._key_ring is None:
            self._key_ring = [(torch.zeros(2, dtype=torch.int32).pin_memory(), None)
                              for _ in range(8)]
        host, ev = self._key_ring[self._key_slot]
        if ev is not None:
            ev.synchronize()
        host[0], host[1] = vals[0], vals[1]
        self.key_state.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._key_ring[self._key_slot] = (host, ev)
        self._key_slot = (self._key_slot + 1) % len(self._key_ring)

    def finish(self, apply: bool = True):
        """Complete every bucket's exchange and (by default) apply the optimizer step."""
        self.launch_pending()
        if self.defer_comm:
            self.join_side()
            self.communicate()
        self.wait()
        self.join_side()
        self._active = False
        if apply:
            self.apply()
        self.last = self.bytes_per_step()
        self.step_idx += 1

    def apply(self):
        scale = self.predivide / self.N
        opt = self.opt
        if self.codec.allreduce:
            if self.codec.wire_dtype == torch.float32:
                opt.step_range(0, self.flat.numel, self.flat.grad, scale)
            else:
                for b in self.flat.buckets:
                    opt.step_range(b.start, b.length, self.send[b.index], scale)
        else:
            for b in self.flat.buckets:
                recv = self.recv[b.index].view(self.N, -1)
                if self.ef21:  # G += mean of the sent differences; momentum step on G
                    gv = self.flat.grad_view(b)
                    self.codec.decode(b.index, recv, gv, scale)
                    G = self.gest[b.start:b.start + b.length]
                    G.add_(gv)
                    opt.step_range(b.start, b.length, G, 1.0)
                elif getattr(opt, "fusable", False):
                    adv = self.dev_key_advance and self.use_dev_key and b.index == self.nb - 1
                    hp, mom = opt.hparams(), opt.mom[b.start:b.start + b.length]
                    if self.dgc:  # momentum and weight decay already ran on the sender
                        hp = dict(hp, momentum=0.0, dampening=0.0, weight_decay=0.0,
                                  nesterov=False)
                        if not self.dgc_mask:  # ... and the lr: p -= mean(sent)
                            hp.update(lr=1.0, lr_t=None)
                        mom = None
                    self.codec.decode_apply_sgd(b.index, recv, scale, self.flat.data_view(b),
                                                mom, hp, opt.first,
                                                shadow=self.flat.shadow_view(b),
                                                key_state=self.key_state if adv else None,
                                                rank=self.comm.rank)
                else:
                    gv = self.flat.grad_view(b)
                    self.codec.decode(b.index, recv, gv, scale)
                    opt.step_range(b.start, b.length, gv, 1.0)
        opt.end_step()

    def decode_average(self):
        """Write the averaged exchanged gradient into ``flat.grad`` (no optimizer step)."""
        scale = self.predivide / self.N
        if self.codec.allreduce:
            if self.codec.wire_dtype == torch.float32:
                self.flat.grad.mul_(scale)
            else:
                for b in self.flat.buckets:
                    self.flat.grad_view(b).copy_(self.send[b.index].float() * scale)
            return
        for b in self.flat.buckets:
            self.codec.decode(b.index, self.recv[b.index].view(self.N, -1),
                              self.flat.grad_view(b), scale)

    def decode_rank(self, src):
        """Write rank ``src``'s decoded payload (unscaled) into ``flat.grad``: local SGD's
        best-worker adoption reads the winner's compressed delta out of the all-gather.  ``src``
        may be a device index tensor (the row is then selected on the device)."""
        if self.codec.allreduce:
            raise ValueError("decode_rank needs a compressing (all-gather) codec")
        for b in self.flat.buckets:
            rows = self.recv[b.index].view(self.N, -1)
            row = rows.index_select(0, src.reshape(1)) if torch.is_tensor(src) \
                else rows[src:src + 1]
            self.codec.decode(b.index, row, self.flat.grad_view(b), 1.0)

    def close(self):
        if self._hooks:
            for p in self.flat.params:
                p._ew_engine_hooks = max(0, getattr(p, "_ew_engine_hooks", 1) - 1)
        for h in self._hooks:
            h.remove()
        self._hooks = []


class SegmentedCapture:
    """A training step captured as HIP graphs that let the collectives overlap backward.

    One forked graph (compute stream -> comm stream -> join) replays node by node from the host
    on ROCm 7.2 (7.9 ms of host time per ResNet-50 step against 0.16 ms for a linear graph:
    profiles/ab/bucket_overlap.txt), so the step is cut into *linear* graphs instead:

    * compute segments on the step stream, split where a gradient bucket becomes complete
      (the exchange hook calls :meth:`split` from inside backward);
    * per split, one graph on the comm stream with that bucket's encode kernels and its RCCL
      collective;
    * the apply graph (fused decode + SGD) after the last segment.

    :meth:`replay` launches segment i, records an event, makes the comm stream wait for it and
    launches comm graph i there, then launches segment i+1 -- so bucket i's encode and all-gather
    run while the GPU is still in the backward of the earlier layers, the overlap the reference
    prototyped with per-layer ``Isend`` in ``LeNetSplit.backward_normal``
    (``src/model_ops/lenet.py:111-186``) and Horovod performs in its background thread
    (``horvod_pytorch.py:197-201``).  Captures use the relaxed mode: a split may end a capture
    begun on another thread (autograd's device thread runs the hooks)."""

    def __init__(self, gstream, cstream, mode: str = "relaxed", total_bytes: int = 0,
                 splits: int = 1):
        self.gs, self.cs, self.mode = gstream, cstream, mode
        # split points: the first time the ready gradient bytes reach k / (splits + 1) of the
        # step's total; each split costs a graph boundary and a stream hop, so a few large
        # comm graphs beat one per bucket
        self.thresholds = [total_bytes * k / (splits + 1) for k in range(1, splits + 1)]
        self.pending, self.ready_bytes = [], 0
        self.pool = torch.cuda.graph_pool_handle()
        self.cpool = torch.cuda.graph_pool_handle()  # comm graphs run beside the segments
        self.segments, self.comms, self.apply = [], [], None
        self.cur = None
        self._evs = []
        self._done = torch.cuda.Event()

    @property
    def splits_left(self) -> int:
        return len(self.thresholds) - len(self.comms)

    def want_split(self, final: bool) -> bool:
        """Split now?  Not at the end of backward (nothing left to overlap)."""
        if final or not self.pending or self.splits_left <= 0:
            return False
        return self.ready_bytes >= self.thresholds[len(self.comms)]

    def begin(self):
        self.cur = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.gs):
            self.cur.capture_begin(pool=self.pool, capture_error_mode=self.mode)

    def split(self, issue):
        with torch.cuda.stream(self.gs):
            self.cur.capture_end()
        self.segments.append(self.cur)
        self.cur = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.cs):
            g.capture_begin(pool=self.cpool, capture_error_mode=self.mode)
            try:
                issue()
            finally:
                g.capture_end()
        self.comms.append(g)
        self._evs.append(torch.cuda.Event())
        self.begin()

    def end(self):
        with torch.cuda.stream(self.gs):
            self.cur.capture_end()
        self.segments.append(self.cur)
        self.cur = None

    def abort(self):
        """End a capture left open by a failure (the stream must not stay capturing)."""
        if self.cur is not None:
            try:
                with torch.cuda.stream(self.gs):
                    self.cur.capture_end()
            except Exception:  # noqa: BLE001 - the original failure is what gets reported
                pass
            self.cur = None

    @property
    def launches(self) -> int:
        return len(self.segments) + len(self.comms) + (self.apply is not None)

    def replay(self):
        cur = torch.cuda.current_stream()
        for i, seg in enumerate(self.segments):
            seg.replay()
            if i < len(self.comms):
                ev = self._evs[i]
                ev.record(cur)
                self.cs.wait_event(ev)
                with torch.cuda.stream(self.cs):
                    self.comms[i].replay()
        if self.comms:
            self._done.record(self.cs)
            cur.wait_event(self._done)
        if self.apply is not None:
            self.apply.replay()


def sync_params(flat, comm, src: int = 0):
    """Broadcast the flat parameters from ``src`` (fixes the reference's independent random init,
    SURVEY Appendix B #1; Horovod's ``broadcast_parameters``, ``horvod_pytorch.py:187``)."""
    comm.broadcast(flat.data, src=src)
    flat.sync_shadow()


def sync_buffers(model, comm, src: int = 0, only_to: int = None):
    """Broadcast the model's buffers (BN running statistics, counters) from ``src``.  With
    ``only_to``, only that rank (and ``src``) keeps the values: the others receive into scratch
    copies, so their own statistics are untouched."""
    for buf in model.buffers():
        if buf.dtype.is_floating_point or buf.dtype in (torch.int64, torch.int32):
            keep = only_to is None or comm.rank in (src, only_to)
            t = buf.data if keep else buf.data.clone()
            comm.broadcast(t, src=src)


class Stopwatch:
    """HIP-event (GPU) or wall-clock (CPU) phase timer."""

    def __init__(self, cuda: bool):
        self.cuda = cuda
        self.marks = []

    def mark(self, name: str):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append((name, e))
        else:
            self.marks.append((name, time.perf_counter()))

    def phases(self):
        """{phase: ms} between consecutive marks (synchronises on GPU)."""
        out = {}
        if len(self.marks) < 2:
            return out
        if self.cuda:
            self.marks[-1][1].synchronize()
        for (n0, a), (n1, b) in zip(self.marks, self.marks[1:]):
            out[n1] = a.elapsed_time(b) if self.cuda else (b - a) * 1e3
        return out

    def reset(self):
        self.marks = []
