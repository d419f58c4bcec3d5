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
import math
import os
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
        self.local_apply = False  # enable_local_apply
        self.local_apply_dense = False
        # producer staging (ops/csrc/dgc_stage.h): the kernel forming a weight gradient (the
        # small-map backward) runs this exchange's momentum-corrected error-feedback staging
        # itself -- velocity and e written, the gradient never stored -- and sets the tensor's
        # stamp word, so the encode's first pass reads e alone for it.  Every parameter is armed
        # with its slots (ops/conv.py _stage_args decides per launch whether it may apply)
        self.stamps = None
        if self.dgc and self.cuda and not flat.attach_grads:
            self.stamps = [torch.zeros(len(b.params), dtype=torch.int32, device=self.device)
                           for b in flat.buckets]
            o = optimizer
            vp, rp, pp = self.vel.data_ptr(), self.resid.data_ptr(), flat.data.data_ptr()
            lrt = getattr(o, "lr_t", None)
            lrp = lrt.data_ptr() if (not self.dgc_mask and lrt is not None) else 0
            for b, st in zip(flat.buckets, self.stamps):
                for ti, (p, off) in enumerate(zip(b.params, b.plan.offsets)):
                    base = 4 * (b.start + off)
                    p._ew_dgc_stage = (vp + base, rp + base, pp + base, float(o.momentum),
                                       float(1.0 - o.dampening), float(o.weight_decay),
                                       int(bool(o.nesterov)), lrp, st.data_ptr() + 4 * ti)
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
        self.clock = None  # Stopwatch of --phase-timing (marks on the step's stream)
        if overlap:
            for p in flat.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
                # ours flush deferred weight-gradient transforms before reading (ops/conv.py)
                p._ew_engine_hooks = getattr(p, "_ew_engine_hooks", 0) + 1
        self.last = StepStats()

    def enable_local_apply(self) -> bool:
        """A world of one: the all-gather of one payload is that payload, so the top-k encode's
        write pass applies the decoded update itself (``ops.topk_encode(apply=...)``, bitwise the
        decode's) and :meth:`apply` launches no decode.  Only where the decode is the sparse one
        (momentum-corrected error feedback under momentum SGD: no receiver momentum) and the step
        always applies (the trainer's all-to-all step; not ``finish(apply=False)`` callers).
        The caller guarantees that the encode runs after backward produced every gradient (one
        bucket, no segmented step): the apply moves parameters.  Returns whether it is on."""
        codec = self.codec
        ok = bool(self.cuda and self.N == 1 and self.nb == 1 and not self.ef21
                  and not codec.allreduce and codec.kind in ("topk", "topk_qsgd")
                  and getattr(codec, "norm", "max") == "max"
                  and getattr(self.opt, "fusable", False) and ops._TOPK_PREDICT
                  and not self.src_flat)
        # momentum-corrected EF: the sparse step at the sent coordinates; otherwise (no EF or
        # plain EF: the momentum runs on the receiver) the dense step over the whole bucket,
        # which the one-launch encode (k_pk_one) runs chunk by chunk after its write
        self.local_apply_dense = ok and not self.dgc
        if self.local_apply_dense:
            ok = all(ops.topk_one_launch(dp) for dp in codec.dplans)
        self.local_apply = ok
        return self.local_apply

    def _apply_hp(self, bi: int) -> dict:
        """The sparse decode's SGD arguments of bucket ``bi`` (momentum-corrected EF: momentum and
        weight decay ran on the sender; without masking the lr is inside the residual)."""
        o = self.opt
        hp = dict(o.hparams(), momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False)
        if not self.dgc_mask:
            hp.update(lr=1.0, lr_t=None)
        return hp

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
        clk = self.clock if self.side is None else None  # marks partition ONE stream
        for bi in bis:
            with self._stream_ctx():
                if clk is not None:
                    clk.mark("backward")  # the compute since the previous mark
                self._encode(bi)
                if clk is not None:
                    clk.mark("encode")
                if not self.defer_comm:
                    self._works[bi] = self._collective(bi)
                    if clk is not None:
                        clk.mark("collective")

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
                       lr_t=None if self.dgc_mask else getattr(o, "lr_t", None),
                       stamps=self.stamps[bi] if self.stamps is not None else None)
        apply = None
        if self.local_apply:  # world of one: the write pass applies the update (no decode)
            adv = self.dev_key_advance and self.use_dev_key and bi == self.nb - 1
            o = self.opt
            hp = o.hparams() if self.local_apply_dense else self._apply_hp(bi)
            apply = dict(param=self.flat.data_view(b), shadow=self.flat.shadow_view(b),
                         lr=hp["lr"], lr_tensor=hp.get("lr_t"),
                         grad_scale=self.predivide / self.N,
                         key_state=self.key_state if adv else None, key_seed=self.codec.seed,
                         key_rank=self.comm.rank)
            if self.local_apply_dense:  # the receiver's momentum SGD over every element
                apply.update(mom=o.mom[b.start:b.start + b.length], momentum=hp["momentum"],
                             dampening=hp["dampening"], weight_decay=hp["weight_decay"],
                             nesterov=hp["nesterov"], first=o.first)
        self.codec.encode(bi, g, self.payload[bi], self.step_idx + self.seed_offset,
                          self.comm.rank, resid,
                          key_tensor=self.key_dev if self.use_dev_key else None, dgc=dgc,
                          ef21=self.ef21, apply=apply)

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
        if self.clock is not None:
            self.clock.mark("collective")  # waiting for the issued collectives
        self._active = False
        if apply:
            self.apply()
            if self.clock is not None:
                self.clock.mark("decode_update")
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
                elif self.local_apply:
                    continue  # applied by the encode's write pass (enable_local_apply)
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

    def codec_health(self) -> dict:
        """Counters of this exchange's HIP top-k encodes (synchronises): the predictive encode's
        fast / full tensor-encodes, and look-back failures -- a write block that gave up waiting
        on its predecessor (bounded spin) wrote its entries at wrong offsets, so every rank would
        decode a corrupted gradient: that raises here instead of training on silently."""
        codec = self.codec
        if not self.cuda or codec.kind not in ("topk", "topk_qsgd") or codec.allreduce:
            return {}
        tot = {"lookback_errors": 0, "fast": 0, "full": 0}
        misses = []  # per bucket: its tensors' full-path counts
        seen = set()
        for _, _, dplans in getattr(codec, "_bound", {}).values():
            for dp in dplans:
                if id(dp) in seen:
                    continue
                seen.add(id(dp))
                st = ops.topk_stats(dp)
                misses.append(st.pop("full_by_tensor", []))
                for k, v in st.items():
                    tot[k] += v
        if tot["lookback_errors"]:
            raise RuntimeError(f"top-k encode: {tot['lookback_errors']} write block(s) gave up on "
                               "the decoupled look-back; the payload offsets are corrupt")
        return {"topk_encode_fast": tot["fast"], "topk_encode_full": tot["full"],
                "topk_encode_full_by_tensor": misses}

    def close(self):
        if self.stamps is not None:
            for p in self.flat.params:
                if hasattr(p, "_ew_dgc_stage"):
                    del p._ew_dgc_stage
            self.stamps = None
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
                 splits: int = 1, device_handoff: bool = False):
        self.gs, self.cs, self.mode = gstream, cstream, mode
        # device hand-offs (ops/csrc/stream_flag.hip): each compute segment ends with a signal
        # kernel, each comm graph starts with a wait kernel on it and ends with a signal, and the
        # apply is captured into the last segment behind a wait on the comm graphs -- no event
        # record / stream wait between the replays (a cross-queue event hop measured ~20 us of
        # GPU time each) and one graph fewer per step.  Off: events and an apply graph (needed
        # by --phase-timing's per-phase marks).
        self.device = bool(device_handoff)
        # int32 counter lines (128 B each): 0 error count, 1 comm-graphs-done, 2 its wait's seen
        # count, then per split a (fork signal, fork seen) pair
        self.flags = torch.zeros(32 * (3 + 2 * max(1, splits)), dtype=torch.int32,
                                 device=torch.cuda.current_device()) if self.device else None
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

    def _end_segment(self):
        """End the current compute segment's capture; an empty one (a split right at the end of
        backward, nothing captured since) is kept as ``None`` and never replayed."""
        import warnings

        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            with torch.cuda.stream(self.gs):
                self.cur.capture_end()
        empty = False
        for w in caught:
            if "Graph is empty" in str(w.message):
                empty = True
            else:  # anything else is re-issued
                warnings.warn_explicit(w.message, w.category, w.filename, w.lineno)
        self.segments.append(None if empty else self.cur)
        self.cur = None

    def split(self, issue):
        i = len(self.comms)
        if self.device:  # the segment's last kernel: its gradients are complete
            with torch.cuda.stream(self.gs):
                ops.flag_signal(self.flags, 3 + 2 * i)
        self._end_segment()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.cs):
            g.capture_begin(pool=self.cpool, capture_error_mode=self.mode)
            try:
                if self.device:
                    ops.flag_wait(self.flags, 3 + 2 * i, 4 + 2 * i, 1, 0)
                issue()
                if self.device:
                    ops.flag_signal(self.flags, 1)
            finally:
                g.capture_end()
        self.comms.append(g)
        self._evs.append(torch.cuda.Event())
        self.begin()

    def join_comms(self):
        """Device hand-offs: the current (last) segment waits for every comm graph before the
        apply captured after this call."""
        if self.device and self.comms:
            with torch.cuda.stream(self.gs):
                ops.flag_wait(self.flags, 1, 2, len(self.comms), 0)

    def handoff_errors(self) -> int:
        """Wait kernels that gave up on their poll bound (synchronises; 0 when healthy)."""
        return int(self.flags[0].item()) if self.device else 0

    def end(self):
        self._end_segment()

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
        return (sum(s is not None for s in self.segments) + len(self.comms)
                + (self.apply is not None))

    def replay(self, clock=None):
        """Replay the step.  ``clock`` (--phase-timing): compute segments are booked as
        ``compute``, the compute stream's wait for the comm graphs as ``comm_wait`` (the exposed
        part of the collectives), the apply as ``decode_update``, and each comm graph's own span
        on the comm stream as the overlapped side interval ``comm_graph``."""
        cur = torch.cuda.current_stream()
        if self.device:  # the kernels hand off on the device: launch back to back
            for i, seg in enumerate(self.segments):
                if seg is not None:
                    seg.replay()
                if i < len(self.comms):
                    with torch.cuda.stream(self.cs):
                        self.comms[i].replay()
            if clock is not None:
                clock.mark("compute")
            return
        for i, seg in enumerate(self.segments):
            if seg is not None:
                seg.replay()
            if clock is not None:
                clock.mark("compute")
            if i < len(self.comms):
                ev = self._evs[i]
                ev.record(cur)
                self.cs.wait_event(ev)
                with torch.cuda.stream(self.cs):
                    t0 = clock.event(self.cs) if clock is not None else None
                    self.comms[i].replay()
                    if clock is not None:
                        clock.side("comm_graph", t0, clock.event(self.cs))
        if self.comms:
            self._done.record(self.cs)
            cur.wait_event(self._done)
            if clock is not None:
                clock.mark("comm_wait")
        if self.apply is not None:
            self.apply.replay()
            if clock is not None:
                clock.mark("decode_update")


# --hip-graph auto: a dense collective at least this large per rank per step (algorithmic wire
# bytes) is worth overlapping with backward at N > 1
OVERLAP_MIN_WIRE_BYTES = int(float(os.environ.get("EWDML_OVERLAP_MIN_MB", "4")) * (1 << 20))
# one comm graph per this many payload bytes (each split costs a graph boundary, ~0.1 ms at N=1)
OVERLAP_BYTES_PER_SPLIT = 32 << 20
OVERLAP_MAX_SPLITS = 3


def plan_graph_mode(world: int, comm_kind: str, codec_kind: str, grad_numel: int,
                    bits: int = 8, overlap: bool = True, bucket_bytes: int = 16 << 20,
                    model: str = None, topk_ratio: float = 0.01, dtype: str = "fp32") -> dict:
    """``--hip-graph auto`` for the all-to-all exchange (``GradientExchange``).

    * N = 1, or collectives on the process group (not capturable), or ``--no-overlap``: the
      one-graph step (``full``; the trainer demotes it to ``split`` for process-group
      collectives).  At N = 1 there is nothing to hide: the segmented step only adds graph
      boundaries (+11 % on dense VGG-11, profiles/ab/segmented_overlap.txt).
    * A configuration with a measured N = 1 profile (``parallel/step_model.py``): the mode the
      step model predicts faster at this N -- ``full`` (backward, then the collective) or
      ``segmented`` (per-bucket collectives on their own stream beside the rest of backward, as
      Horovod's background all-reduce does, ``horvod_pytorch.py:197-201``, and the reference's
      ``LeNetSplit`` prototyped, ``src/model_ops/lenet.py:111-186``).  The prediction of both is
      returned (``predicted_ms``) so a scaling run can be checked against it.
    * Otherwise the codec-kind rule: ``full`` for top-k payloads (a few hundred KiB per rank;
      their encode, which a segmented step runs on the comm stream, slows the concurrent backward
      GEMMs by more than it hides: +20 % at N = 1), ``segmented`` for dense collectives whose
      per-rank wire bytes reach ``OVERLAP_MIN_WIRE_BYTES``.
    * Segmented steps get one split per 32 MiB of payload (at most 3) and buckets small enough
      that every split point has buckets on both sides.

    Returns ``{"mode", "splits", "bucket_bytes", "wire_bytes", "reason"}`` (+ ``predicted_ms``)."""
    from .step_model import overlap_splits, predict, profile_for

    per_elem = {"none": 4.0, "fp16": 2.0, "bf16": 2.0, "qsgd": bits / 8.0}.get(codec_kind)
    payload = grad_numel * (per_elem or 0.0)
    # top-k payload per rank (estimate): k entries of one code byte (4-bit: half) + a 2-byte index
    pb = payload if per_elem is not None else grad_numel * topk_ratio * (2.0 + max(bits, 4) / 8.0)
    if codec_kind in ("none", "fp16", "bf16"):
        wire = 2.0 * (world - 1) / max(world, 1) * payload  # ring all-reduce
    else:
        wire = (world - 1) * pb  # all-gather
    out = {"mode": "full", "splits": 1, "bucket_bytes": int(bucket_bytes), "wire_bytes": int(wire)}
    splits = overlap_splits(payload, OVERLAP_MAX_SPLITS, OVERLAP_BYTES_PER_SPLIT)
    prof = profile_for(model, codec_kind, dtype)
    pred = None
    if prof is not None:
        # the all-reduce moves the wire dtype's bytes (fp16 / bf16 codecs: 2 per element)
        pred = predict(prof, world, codec_kind, pb, payload if per_elem is not None and
                       codec_kind in ("none", "fp16", "bf16") else 4.0 * grad_numel, splits)
        out["predicted_ms"] = pred
    if world <= 1:
        return dict(out, reason="one rank: nothing to overlap")
    if comm_kind != "rccl-stream":
        return dict(out, reason="process-group collectives are not captured")
    if not overlap:
        return dict(out, reason="--no-overlap")
    want = (4 * grad_numel) // (2 * (splits + 1))
    seg = {"mode": "segmented", "splits": splits,
           "bucket_bytes": int(min(bucket_bytes, max(1 << 20, want)))}
    if pred is not None:
        if pred["segmented"] < pred["full"]:
            return dict(out, **seg, reason="step model: overlap hides more than it costs")
        return dict(out, reason="step model: the one-graph step is faster")
    if per_elem is None:
        return dict(out, reason="top-k payloads are small; the encode would slow backward")
    if wire < OVERLAP_MIN_WIRE_BYTES:
        return dict(out, reason="collective below the overlap threshold")
    return dict(out, **seg, reason="dense collective overlapped with backward")


def replica_fingerprint(t: torch.Tensor) -> dict:
    """Order-sensitive fingerprint of a replica's flat fp32 parameters: the fp64 sum, an fp64
    position-weighted sum, and the XOR fold of the raw 32-bit words (bit-exact)."""
    x = t.detach().reshape(-1)
    if x.dtype != torch.float32:
        x = x.float()
    w = (torch.arange(x.numel(), device=x.device, dtype=torch.int64) % 65521 + 1).double()
    bits = x.contiguous().view(torch.int32)
    while bits.numel() > 1:
        if bits.numel() % 2:
            bits = torch.cat([bits, bits.new_zeros(1)])
        bits = torch.bitwise_xor(bits[0::2], bits[1::2])
    return {"sum": float(x.double().sum()), "wsum": float((x.double() * w).sum()),
            "xor": int(bits.item()) & 0xFFFFFFFF if bits.numel() else 0}


def check_replicas(comm, t: torch.Tensor) -> dict:
    """Collective: every rank's fingerprint of ``t``; ``identical`` when all are bitwise equal
    (synchronous data parallelism keeps every replica identical -- the property the reference's
    broadcast of the averaged gradient is meant to give, ``sync_replicas_master_nn.py:193-212``)."""
    fp = replica_fingerprint(t)
    allfp = comm.all_gather_object(fp)
    key = [(repr(f["sum"]), repr(f["wsum"]), f["xor"]) for f in allfp]  # NaN-safe comparison
    return {"identical": all(k == key[0] for k in key), "fingerprints": allfp}


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
    """Phase clock: HIP events on the step's stream (GPU) or wall clock (CPU).

    ``mark(name)`` closes the interval since the previous mark and books it under ``name``, so
    the marks of one step partition its timeline: the phases sum to the step time exactly
    (``--phase-timing``; the reference's per-worker ``time_send`` / ``time_recieve`` /
    computation split, ``src/distributed_worker.py:130-155, 214-231``).  Repeated names
    accumulate (e.g. one ``encode`` + ``collective`` pair per bucket).  ``side(name, a, b)`` books
    an interval of another stream (a collective overlapped with backward) that is not part of
    the partition.  Marks are skipped while a HIP graph is being captured."""

    COMM_PHASES = ("collective", "comm_wait")  # exposed communication (the rest is compute)

    def __init__(self, cuda: bool):
        self.cuda = cuda
        self.marks = []
        self.sides = []

    def _capturing(self) -> bool:
        return self.cuda and torch.cuda.is_current_stream_capturing()

    def mark(self, name: str):
        if self._capturing():
            return
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append((name, e))
        else:
            self.marks.append((name, time.perf_counter()))

    def event(self, stream=None):
        """A timing event recorded on ``stream`` (GPU), or the wall clock (CPU)."""
        if not self.cuda:
            return time.perf_counter()
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def side(self, name: str, start, end):
        self.sides.append((name, start, end))

    def _ms(self, a, b) -> float:
        return a.elapsed_time(b) if self.cuda else (b - a) * 1e3

    def phases(self) -> dict:
        """{phase: ms} summed over the step's intervals (synchronises on the GPU); ``side:*``
        entries are the overlapped intervals of other streams."""
        out = {}
        if self.cuda and (self.marks or self.sides):
            torch.cuda.synchronize()
        for (_, a), (n1, b) in zip(self.marks, self.marks[1:]):
            out[n1] = out.get(n1, 0.0) + self._ms(a, b)
        for n, a, b in self.sides:
            key = "side:" + n
            out[key] = out.get(key, 0.0) + self._ms(a, b)
        return out

    def total(self) -> float:
        """The step time: first to last mark."""
        if len(self.marks) < 2:
            return 0.0
        if self.cuda:
            self.marks[-1][1].synchronize()
        return self._ms(self.marks[0][1], self.marks[-1][1])

    @classmethod
    def split(cls, phases: dict) -> tuple:
        """(communication ms, computation ms) of a phase dict: the reference report's
        "Communication and Computation Time" split (exposed communication only; overlapped
        collectives are compute-stream time)."""
        comm = sum(v for k, v in phases.items() if k in cls.COMM_PHASES)
        comp = sum(v for k, v in phases.items() if not k.startswith("side:")
                   and k not in cls.COMM_PHASES)
        return comm, comp

    def reset(self):
        self.marks = []
        self.sides = []
