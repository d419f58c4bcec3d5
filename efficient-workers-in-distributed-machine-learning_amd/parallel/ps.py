"""Parameter-server topology: rank 0 is the server, ranks 1..N-1 are workers.

Reproduces the reference's star (``sync_replicas_master_nn.py`` + ``distributed_worker.py``) for
every method, with the codecs applied for real:

* push: each worker encodes its gradient (push codec) and ``gather``s it to rank 0
  (``distributed_worker.py:317-351`` / ``sync_replicas_master_nn.py:218-232``);
* the server decodes the N-1 worker payloads (its own slot is a dummy, as in the reference's
  ``aggregate_gradient`` summing ``gradient[1:]``, ``:215-216``) and averages them (``:187-190``);
* pull ``grad`` (Methods 3-5): the server encodes the *averaged* gradient with the pull codec and
  broadcasts it (``:193-212``); every process decodes it and applies the same SGD step, so the
  server's replica tracks the workers' (the server's replica is what gets checkpointed);
* pull ``weights`` (Methods 1-2): the server steps its optimizer with the averaged gradient and
  broadcasts the flat weights (the reference's intended ``_bcast_weight``, which at HEAD
  broadcasts the wrong buffer -- SURVEY Appendix B #14).

Collectives are per bucket: one gather + one broadcast per bucket instead of 2 x #tensors
blocking Gloo round trips per step.  The server runs no forward/backward.

A step is three phases -- :meth:`launch_pending` (workers encode their push payloads),
:meth:`communicate` (gather, server decode / average / re-encode, broadcast) and :meth:`apply`
(workers decode the pull and step) -- so a worker's step can run as HIP graph A (forward,
backward, push encode) -> eager collectives -> graph B (pull decode + update), the trainer's
``split`` graph mode; the push codec then reads its RNG key from device memory.

k-of-n aggregation (``--mode kill --num-aggregate k``, the reference's declared-but-unused
straggler flags, ``distributed_nn.py:50-59``): the pushes become point-to-point sends, the server
averages the first ``k`` worker gradients to ARRIVE (arrival order of the first bucket; the same
workers for every bucket of the step) and drains the late ones without using them, so the step
protocol stays in lockstep; a worker still missing ``--kill-threshold`` seconds after the k-th
arrival aborts the job.  Which workers count is timing-dependent by design;
``self.last_aggregated`` records them.
"""
import datetime
import time

import torch

from .engine import StepStats


class PSExchange:
    server_rank = 0

    def __init__(self, flat, comm, push_codec, pull_codec, optimizer, pull: str = "grad",
                 aggregate: int = None, kill_threshold: float = None):
        if comm.world < 2:
            raise ValueError("the ps topology needs at least 2 processes (1 server + workers)")
        self.flat, self.comm, self.opt, self.pull = flat, comm, optimizer, pull
        self.device = flat.data.device
        self.push = push_codec.bind([b.plan for b in flat.buckets], self.device)
        self.pullc = pull_codec.bind([b.plan for b in flat.buckets], self.device)
        self.N = comm.world
        self.is_server = comm.rank == self.server_rank
        self.nb = len(flat.buckets)
        self.step_idx = 0
        self.payload, self.gathered, self.pull_buf = [], [], []
        for b in flat.buckets:
            P = self._nbytes(self.push, b)
            self.payload.append(torch.zeros(P, dtype=torch.uint8, device=self.device))
            self.gathered.append(torch.zeros((self.N, P), dtype=torch.uint8, device=self.device)
                                 if self.is_server else None)
            Q = self._nbytes(self.pullc, b)
            self.pull_buf.append(torch.zeros((1, Q), dtype=torch.uint8, device=self.device))
        self.avg = torch.zeros_like(flat.grad)
        self.last = StepStats()
        W = self.N - 1
        self.k = W if aggregate is None else max(1, min(int(aggregate), W))
        self.kill_threshold = kill_threshold
        self.last_aggregated = list(range(1, self.N))
        # split-graph protocol (runtime/trainer.py): the push encode in graph A reads the key of
        # step_idx from key_state (set_device_key), everything else is stream-ordered
        self.use_dev_key = self.dev_key_advance = self.defer_comm = self._active = False
        self.key_state = torch.zeros(2, dtype=torch.int32, device=self.device)
        self.key_dev = self.key_state[1:2]
        self.side = None
        self._encoded = False
        self.clock = None  # Stopwatch of --phase-timing

    @staticmethod
    def _nbytes(codec, b):
        if codec.allreduce:  # dense payload = raw gradient bytes in the codec's wire dtype
            return b.length * codec.wire_dtype.itemsize
        return codec.payload_bytes(b.index)

    # dense codecs ship the gradient bytes themselves
    def _encode(self, codec, bi, src, out, rank, key_tensor=None):
        if codec.allreduce:
            out.view(codec.wire_dtype).copy_(src.to(codec.wire_dtype))
        else:
            codec.encode(bi, src, out, self.step_idx, rank, key_tensor=key_tensor)

    def set_device_key(self, step: int = None):
        """Upload the push codec's key of ``step`` (default: the current step) for graph A."""
        s = self.step_idx if step is None else step
        key = self.push.key(s, self.comm.rank) if not self.push.allreduce else 0
        vals = [((v + (1 << 31)) % (1 << 32)) - (1 << 31) for v in (s & 0xFFFFFFFF, key)]
        if self.key_state.device.type != "cuda":
            self.key_state.copy_(torch.tensor(vals, dtype=torch.int32))
            return
        # stream-ordered upload from a ring of pinned slots (no host synchronisation)
        if getattr(self, "_ring", None) is None:
            self._ring = [(torch.zeros(2, dtype=torch.int32).pin_memory(), None) for _ in range(8)]
            self._slot = 0
        host, ev = self._ring[self._slot]
        if ev is not None:
            ev.synchronize()
        host[0], host[1] = vals[0], vals[1]
        self.key_state.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ring[self._slot] = (host, ev)
        self._slot = (self._slot + 1) % len(self._ring)

    def _decode(self, codec, bi, recv, out, scale):
        if codec.allreduce:
            n = recv.shape[0]
            vals = recv.view(codec.wire_dtype).view(n, -1).to(torch.float32)
            out.copy_(vals.sum(0) * scale)
        else:
            codec.decode(bi, recv, out, scale)

    def begin(self):
        self._encoded = False

    def _push_k_of_n(self, bi):
        """Point-to-point push; the server returns the worker ranks whose payload to use."""
        if not self.is_server:
            self.comm.isend(self.payload[bi], self.server_rank, tag=bi).wait()
            return None
        order = []
        # once k pushes have arrived the late ones get --kill-threshold seconds, then the step
        # (and the job) is aborted: the threshold bounds only this per-step push; setup /
        # checkpoint / eval collectives keep the process group's --comm-timeout
        thr = self.kill_threshold

        def stalled(ranks):
            return RuntimeError(f"--mode kill: worker(s) {sorted(ranks)} did not push bucket {bi} "
                                f"within {thr:g} s of the first {self.k}")

        if self.comm.backend == "gloo":
            # receive-from-any-source gives the arrival order of the first k (Gloo's irecv never
            # reports completion before wait()); the rest are waited for with the deadline
            tmp = self.payload[bi]  # the server's own payload buffer is otherwise unused
            for _ in range(self.k):
                src = self.comm.recv_any(tmp, tag=bi)
                self.gathered[bi][src].copy_(tmp)
                order.append(src)
            deadline = time.monotonic() + thr if thr else None
            rest = [r for r in range(1, self.N) if r not in order]
            works = {r: self.comm.irecv(self.gathered[bi][r], r, tag=bi) for r in rest}
            for r in rest:
                try:
                    if deadline is None:
                        works[r].wait()
                    else:
                        left = max(deadline - time.monotonic(), 1e-3)
                        works[r].wait(timeout=datetime.timedelta(seconds=left))
                except RuntimeError as e:
                    raise stalled([q for q in rest if q not in order]) from e
                order.append(r)
        else:  # RCCL: one receive per worker, arrival order by polling completion
            works = {r: self.comm.irecv(self.gathered[bi][r], r, tag=bi)
                     for r in range(1, self.N)}
            t_quorum = None
            while works:
                done = [r for r, w in sorted(works.items()) if w.is_completed()]
                for r in done:
                    order.append(r)
                    works.pop(r).wait()
                if t_quorum is None and len(order) >= self.k:
                    t_quorum = time.monotonic()
                if works and t_quorum is not None and thr and time.monotonic() - t_quorum > thr:
                    raise stalled(works)
                if not done:
                    time.sleep(0)
        if bi == 0:  # the step's workers are chosen on the first bucket
            self.last_aggregated = sorted(order[:self.k])
        return self.last_aggregated

    def launch_pending(self):
        """Phase 1 (workers): encode every bucket's push payload."""
        if self._encoded or self.is_server:
            return
        rank = self.comm.rank
        kt = self.key_dev if self.use_dev_key else None
        if self.clock is not None:
            self.clock.mark("backward")
        for b in self.flat.buckets:
            self._encode(self.push, b.index, self.flat.grad_view(b), self.payload[b.index], rank,
                         kt)
        self._encoded = True
        if self.clock is not None:
            self.clock.mark("encode")

    def join_side(self):
        pass

    def wait(self):
        pass

    def communicate(self):
        """Phase 2: gather the pushes, the server averages (and re-encodes the pull), broadcast."""
        W = self.N - 1
        rank = self.comm.rank
        clk = self.clock

        def mark(name):
            if clk is not None:
                clk.mark(name)

        for b in self.flat.buckets:
            bi = b.index
            av = self.avg[b.start:b.start + b.length]
            if self.k < W:
                use = self._push_k_of_n(bi)
                mark("collective")  # push (send / gather): the reference's time_send
                if self.is_server:
                    rows = torch.tensor(use, device=self.device)
                    self._decode(self.push, bi, self.gathered[bi].index_select(0, rows), av,
                                 1.0 / len(use))
            else:
                self.comm.gather(self.payload[bi], self.gathered[bi], dst=self.server_rank)
                mark("collective")
                if self.is_server:
                    self._decode(self.push, bi, self.gathered[bi][1:], av, 1.0 / W)
            if self.pull == "grad":
                if self.is_server:
                    self._encode(self.pullc, bi, av, self.pull_buf[bi][0], rank)
                    mark("aggregate")  # the server's decode / average / re-encode
                self.comm.broadcast(self.pull_buf[bi], src=self.server_rank)
                mark("collective")  # pull (broadcast): the reference's time_recieve
        if self.pull != "grad":
            if self.is_server:
                self.opt.step(grad=self.avg)
                mark("aggregate")
            self.comm.broadcast(self.flat.data, src=self.server_rank)
            mark("collective")

    def apply(self):
        """Phase 3: decode the pulled average and step (weights pull: already applied)."""
        if self.pull == "grad":
            for b in self.flat.buckets:
                bi = b.index
                self._decode(self.pullc, bi, self.pull_buf[bi],
                             self.avg[b.start:b.start + b.length], 1.0)
            self.opt.step(grad=self.avg)
        elif not self.is_server:
            self.opt.end_step()

    def finish(self):
        self.launch_pending()
        self.communicate()
        self.apply()
        if self.clock is not None:
            self.clock.mark("decode_update")
        self._encoded = False
        self.last = self.bytes_per_step()
        self.step_idx += 1

    def bytes_per_step(self):
        s = StepStats()
        for b in self.flat.buckets:
            push = self._nbytes(self.push, b)
            pull = self.flat.numel * 4 // self.nb if self.pull == "weights" else \
                self._nbytes(self.pullc, b)
            if self.pull == "weights":
                pull = b.length * 4
            s.payload_bytes += push
            s.dense_bytes += b.plan.numel * 4
            if self.is_server:
                s.wire_bytes_recv += push * (self.N - 1)
                s.wire_bytes_sent += pull * (self.N - 1)
            else:
                s.wire_bytes_sent += push
                s.wire_bytes_recv += pull
            s.collectives += 2
        return s

    def pull_bytes(self):
        return sum(b.length * 4 if self.pull == "weights" else self._nbytes(self.pullc, b)
                   for b in self.flat.buckets)

    def close(self):
        pass
