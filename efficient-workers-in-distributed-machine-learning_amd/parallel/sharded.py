"""Sharded parameter server: every rank owns 1/N of each bucket (``--topology sharded``).

SURVEY section 7.3 item 4(b).  The all-gather exchange (``engine.py``) makes every rank receive
N-1 peer payloads, so the pull traffic grows with N; the reference's star (``ps.py``,
``sync_replicas_master_nn.py:187-232``) bounds it by re-compressing the average on one server,
which then carries N-1 pushes alone.  Sharding the server role spreads that load:

1. each bucket is cut into N contiguous shards at 8192-element chunk boundaries; a shard's
   tensor segments form its own ``BucketPlan`` (top-k is taken per segment: k = max(1,
   int(n_seg * ratio)), the reference's ``TopK.py:7`` rule applied to the segment);
2. push: every rank encodes each shard of its gradient and one ``all_to_all`` hands shard r's
   payloads to rank r (fixed-size rows: every payload of a bucket is padded to its largest shard);
3. the owner decodes its N payloads, averages them (x 1/N) and re-encodes the averaged shard
   (the server's pull compression, ``sync_replicas_master_nn.py:193-212``);
4. pull: one ``all_gather`` of the owners' re-encoded shards; every rank decodes all N shards and
   applies the same optimizer step, so the replicas stay identical.

Per rank and step that is ~2 payloads on the wire in each direction whatever N is, against N-1
received payloads for the all-gather exchange, at the cost of a second quantisation (as in the
reference's PS) and two collectives per bucket.  Codecs run through the HIP kernels on the GPU
and through the torch oracle on the CPU (``compress/codecs.py``).
"""
import torch

from ..compress import CHUNK, BucketPlan, make_codec
from .engine import StepStats


def shard_plans(plan: BucketPlan, n: int, bucket_offset: int):
    """Cut a bucket plan into ``n`` contiguous, chunk-aligned shards.

    Returns ``[(start, length, BucketPlan | None)]`` per shard (element offsets relative to the
    bucket start); a shard holding no tensor elements (tiny bucket, many ranks) has plan None.
    """
    L = plan.length
    nch = (L + CHUNK - 1) // CHUNK
    cuts = [min(L, ((r * nch) // n) * CHUNK) for r in range(n)] + [L]
    out = []
    for r in range(n):
        s0, s1 = cuts[r], cuts[r + 1]
        numels, offsets = [], []
        for off, num in zip(plan.offsets, plan.numels):
            a, b = max(off, s0), min(off + num, s1)
            if a < b:
                numels.append(b - a)
                offsets.append(a - s0)
        sp = BucketPlan(numels, offsets, plan.ratio, bucket_offset + s0, s1 - s0) \
            if numels else None
        out.append((s0, s1 - s0, sp))
    return out


class ShardedPSExchange:
    """All ranks are workers and each owns one shard of every bucket (see module docstring)."""

    def __init__(self, flat, comm, kind: str, optimizer, **codec_kw):
        if kind in ("none", "fp16", "bf16"):
            raise ValueError("--topology sharded needs a compressing codec (topk, topk_qsgd, qsgd); "
                             "dense codecs use the all-reduce exchange")
        self.flat, self.comm, self.opt = flat, comm, optimizer
        self.device = flat.data.device
        self.N, self.rank = comm.world, comm.rank
        self.nb = len(flat.buckets)
        self.step_idx = 0
        self.shards = []  # per bucket: [(start, length, plan index or -1)]
        plans = []
        for b in flat.buckets:
            row = []
            for s0, ln, sp in shard_plans(b.plan, self.N, b.start):
                row.append((s0, ln, len(plans) if sp is not None else -1))
                if sp is not None:
                    plans.append(sp)
            self.shards.append(row)
        self.codec = make_codec(kind, **codec_kw).bind(plans, self.device)
        self.P = []  # per bucket: row size (bytes) = the largest shard payload
        self.send, self.recv, self.own, self.gathered = [], [], [], []
        for bi in range(self.nb):
            P = max([self.codec.payload_bytes(j) for _, _, j in self.shards[bi] if j >= 0] or [1])
            self.P.append(P)
            z = dict(dtype=torch.uint8, device=self.device)
            self.send.append(torch.zeros((self.N, P), **z))
            self.recv.append(torch.zeros((self.N, P), **z))
            self.gathered.append(torch.zeros(self.N * P, **z))
            self.own.append(self.gathered[bi][self.rank * P:(self.rank + 1) * P])
        self.avg = torch.zeros_like(flat.grad)
        self.last = StepStats()

        # split-graph protocol (runtime/trainer.py, as the parameter server's): graph A =
        # forward, backward and the push encodes (RNG key of step_idx from key_state), then the
        # eager collectives with the owners' average / re-encode between them, then graph B =
        # decode of every shard + optimizer step
        self.use_dev_key = self.dev_key_advance = self.defer_comm = self._active = False
        self.key_state = torch.zeros(2, dtype=torch.int32, device=self.device)
        self.key_dev = self.key_state[1:2]
        self.side = None
        self._encoded = False
        self.clock = None  # Stopwatch of --phase-timing

    def _mark(self, name):
        if self.clock is not None:
            self.clock.mark(name)

    def begin(self):
        self._encoded = False

    def set_device_key(self, step: int = None):
        """Upload the push encodes' key of ``step`` (default: the current step) for graph A."""
        from .ps import PSExchange

        PSExchange.set_device_key(self, step)

    @property
    def push(self):  # the push codec (PSExchange.set_device_key reads it)
        return self.codec

    def launch_pending(self):
        """Phase 1: encode every shard of every bucket of this rank's gradient."""
        if self._encoded:
            return
        self._mark("backward")
        kt = self.key_dev if self.use_dev_key else None
        for b in self.flat.buckets:
            g = self.flat.grad_view(b)
            for r, (s0, ln, j) in enumerate(self.shards[b.index]):
                if j >= 0:
                    Pj = self.codec.payload_bytes(j)
                    self.codec.encode(j, g[s0:s0 + ln], self.send[b.index][r, :Pj],
                                      self.step_idx, self.rank, key_tensor=kt)
        self._encoded = True
        self._mark("encode")

    def join_side(self):
        pass

    def wait(self):
        pass

    def communicate(self):
        """Phase 2: all-to-all of the shard payloads; each owner averages its N pushes and
        re-encodes the average; all-gather of the owners' payloads."""
        N, me = self.N, self.rank
        for b in self.flat.buckets:
            bi = b.index
            av = self.avg[b.start:b.start + b.length]
            self.comm.all_to_all(self.recv[bi], self.send[bi])
            self._mark("collective")
            s0, ln, j = self.shards[bi][me]
            if j >= 0:  # owner: average the N pushes of its shard, re-encode the average
                Pj = self.codec.payload_bytes(j)
                self.codec.decode(j, self.recv[bi][:, :Pj].contiguous(), av[s0:s0 + ln], 1.0 / N)
                self.codec.encode(j, av[s0:s0 + ln], self.own[bi][:Pj], self.step_idx, N + me)
            self._mark("aggregate")
            self.comm.all_gather(self.gathered[bi], self.own[bi])
            self._mark("collective")

    def apply(self):
        """Phase 3: decode every owner's averaged shard and take the optimizer step."""
        N = self.N
        for b in self.flat.buckets:
            bi, P = b.index, self.P[b.index]
            av = self.avg[b.start:b.start + b.length]
            rows = self.gathered[bi].view(N, P)
            for r, (s0, ln, j) in enumerate(self.shards[bi]):
                if j >= 0:
                    Pj = self.codec.payload_bytes(j)
                    self.codec.decode(j, rows[r:r + 1, :Pj].contiguous(), av[s0:s0 + ln], 1.0)
                else:
                    av[s0:s0 + ln].zero_()
        self.opt.step(grad=self.avg)

    def finish(self):
        self.launch_pending()
        self.communicate()
        self.apply()
        self._mark("decode_update")
        self._encoded = False
        self.last = self.bytes_per_step()
        self.step_idx += 1

    def bytes_per_step(self):
        s = StepStats()
        for b in self.flat.buckets:
            P = self.P[b.index]
            s.payload_bytes += sum(self.codec.payload_bytes(j)
                                   for _, _, j in self.shards[b.index] if j >= 0)
            s.dense_bytes += b.plan.numel * 4
            s.wire_bytes_sent += 2 * (self.N - 1) * P  # all-to-all rows + ring all-gather
            s.wire_bytes_recv += 2 * (self.N - 1) * P
            s.collectives += 2
        return s

    def close(self):
        pass
