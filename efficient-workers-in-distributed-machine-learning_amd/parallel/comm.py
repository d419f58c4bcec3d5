"""Thin communicator over ``torch.distributed``.

On the GPU the process group is ``nccl``, which on ROCm *is* RCCL.  The data-plane collectives of
the training step (all-gather of packed payloads, all-reduce of dense buckets, broadcast,
all-to-all) go through a communicator of our own (``ops/csrc/rccl_comm.hip``): RCCL over xGMI,
enqueued on the caller's current HIP stream, so a captured step stays one linear graph (no fork into
the process group's private stream, no watchdog polling during capture).  ``EWDML_COMM=pg`` keeps
them on the process group instead (A/B; also the fallback if the communicator cannot be created).
Control-plane calls (barrier, scalar/object collectives, the parameter server's point-to-point
messages) stay on the process group.  On the CPU it is ``gloo`` (tests, ``BASELINE.json`` config
#1).  A world of one process needs no process group at all: collectives degenerate to local
copies.

Parity: replaces the reference's per-layer ``dist.gather`` / ``dist.broadcast`` call sites
(``distributed_worker.py:256,278,350``, ``sync_replicas_master_nn.py:212,223``) and Horovod's
``hvd.allreduce`` / ``broadcast_parameters`` (``horvod_pytorch.py:84-87,187-188``).
"""
import datetime
import os

import torch
import torch.distributed as dist


def init_distributed(backend: str = None, timeout_s: float = None, device=None) -> "Comm":
    """env:// rendezvous (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT as set by torchrun)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    force = os.environ.get("EWDML_FORCE_PG") == "1"  # real process group even for one rank
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if timeout_s:
            kw["timeout"] = datetime.timedelta(seconds=float(timeout_s))
        if backend == "nccl" and device is not None:
            kw["device_id"] = torch.device(device)
        dist.init_process_group(backend=backend, **kw)
    return Comm()


class Comm:
    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank, self.world, self.backend = 0, 1, "local"
        self._gloo_ag = self.backend == "gloo"
        # EWDML_FORCE_PG=1: issue real collectives even in a world of one (exercises RCCL and
        # graph capture of collectives on a single-GPU box)
        self._local = self.world == 1 and not (os.environ.get("EWDML_FORCE_PG") == "1"
                                               and self.backend != "local")
        self.rccl = None  # handle of the stream-ordered RCCL communicator (see module doc)
        self.watchdog = None  # native step watchdog (arm_watchdog)
        self.probe = None  # outcome of the first-contact collective probe (parallel/probe.py)
        if (self.backend == "nccl" and not self._local and group is None
                and os.environ.get("EWDML_COMM", "rccl") != "pg"):
            self.rccl = self._make_rccl()
            if self.rccl is not None and os.environ.get("EWDML_COMM_PROBE", "1") != "0":
                self._verify_rccl()

    def _verify_rccl(self):
        """Probe the own communicator (eager and graph-captured collectives against their closed
        forms, all ranks agreeing); on any failure every rank destroys it and the data plane
        falls back to the process group (whose collectives the trainer keeps outside its graphs:
        split graphs)."""
        import logging

        from .probe import probe_collectives

        log = logging.getLogger("ewdml")
        res = probe_collectives(self, torch.device("cuda", torch.cuda.current_device()))
        self.probe = res
        if res["ok"]:
            return
        log.warning(f"RCCL communicator probe failed on at least one rank (this rank: eager="
                    f"{res['eager']} graph={res['graph']} error={res['error']}): collectives "
                    "fall back to the process group on every rank")
        torch.cuda.synchronize()
        try:
            self._rc().rccl_destroy(self.rccl)
        except Exception as e:  # noqa: BLE001 - the handle is dropped either way
            log.warning(f"destroying the failed communicator: {e!r}")
        self.rccl = None

    def _make_rccl(self):
        """Create the RCCL communicator (collective over the process group: rank 0's unique id
        is broadcast as an object).  Every rank must end up with one or none alike."""
        import logging

        from .. import ops

        log = logging.getLogger("ewdml")
        # every rank issues the same process-group collectives whatever fails where: rank 0
        # always broadcasts (the unique id, or None after a local failure) and everyone skips
        # ncclCommInitRank on None, then all agree on the outcome
        uid = None
        if self.rank == 0:
            try:
                uid = ops.require().rccl_unique_id()
            except Exception as e:  # noqa: BLE001 - fall back to the process group everywhere
                log.warning(f"RCCL unique id unavailable ({e!r})")
        uid = self.broadcast_object(uid, src=0)
        h, ok = None, 0.0
        if uid is not None:
            try:
                h = ops.require().rccl_init(uid, self.world, self.rank,
                                            torch.cuda.current_device())
                ok = 1.0
            except Exception as e:  # noqa: BLE001
                log.warning(f"RCCL communicator init failed ({e!r})")
        if self.all_reduce_scalars([ok], op="min")[0] < 1.0:
            if h is not None:
                ops.require().rccl_destroy(h)
            log.warning("RCCL communicator unavailable: collectives stay on the process group")
            return None
        return h

    def _rc(self):
        from .. import ops

        return ops.require()

    # -- failure detection on the data plane -------------------------------------
    def arm_watchdog(self, timeout_s: float, exit_code: int = 3, force: bool = False):
        """Start the native step watchdog (``ops/csrc/rccl_comm.hip``): after :meth:`watch`
        records a step's completion event, a host thread aborts the RCCL communicator and ends the
        process with ``exit_code`` if that event is still pending after ``timeout_s`` (a dead or
        stalled peer).  Armed only when the own communicator carries the collectives (the
        process group has its own watchdog) unless ``force``."""
        if self.watchdog is not None or not timeout_s or timeout_s <= 0:
            return self.watchdog
        if self.rccl is None and not force:
            return None
        self.watchdog = self._rc().rccl_watchdog_start(self.rccl or 0,
                                                       torch.cuda.current_device(),
                                                       float(timeout_s), int(exit_code))
        return self.watchdog

    def watch(self):
        """Record the current stream's position for the watchdog (call after a step's last
        collective was enqueued; never inside a graph capture)."""
        if self.watchdog is not None:
            from ..ops import _stream

            self._rc().rccl_watch(self.watchdog, _stream())

    def abort(self):
        """ncclCommAbort of the own communicator (peers blocked in a collective return)."""
        if self.rccl is not None:
            self._rc().rccl_abort(self.rccl)
            self.rccl = None

    def close(self):
        """Stop the watchdog and destroy the own communicator (the process group stays)."""
        if self.watchdog is None and self.rccl is None:
            return
        torch.cuda.synchronize()  # pending watch marks write the watchdog's host memory
        if self.watchdog is not None:
            self._rc().rccl_watchdog_stop(self.watchdog)
            self.watchdog = None
        if self.rccl is not None:
            self._rc().rccl_destroy(self.rccl)
            self.rccl = None

    @staticmethod
    def _dt(t):
        return _RC_DT[t.dtype]

    @property
    def kind(self) -> str:
        """Where the step's data-plane collectives run: ``rccl-stream`` (own communicator on the
        caller's stream), ``process-group`` (torch.distributed), or ``local`` (world of one)."""
        if self._local:
            return "local"
        return "rccl-stream" if self.rccl is not None else "process-group"

    @property
    def distributed(self) -> bool:
        return self.world > 1

    # -- collectives (return a Work handle or None when already complete) --------------------
    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """``out`` [world * n] <- concat of every rank's ``inp`` [n] (``inp`` may be this rank's
        slot of ``out``: in-place)."""
        if self._local:
            if inp.data_ptr() != out.data_ptr():
                out[:inp.numel()].copy_(inp)
            return None
        if self.rccl is not None and out.is_cuda:
            from ..ops import _ptr, _stream

            self._rc().rccl_all_gather(self.rccl, _ptr(inp), _ptr(out), inp.numel(),
                                       self._dt(inp), _stream())
            return None
        if self._gloo_ag:
            chunks = list(out.view(self.world, -1).unbind(0))
            if inp.data_ptr() == chunks[self.rank].data_ptr():
                inp = inp.clone()  # gloo copies its input into the output slot: no aliasing
            return dist.all_gather(chunks, inp, group=self.group, async_op=async_op)
        return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM, async_op: bool = False):
        if self._local:
            return None
        if self.rccl is not None and t.is_cuda and op in _RC_OP:
            from ..ops import _ptr, _stream

            self._rc().rccl_all_reduce(self.rccl, _ptr(t), _ptr(t), t.numel(), self._dt(t),
                                       _RC_OP[op], _stream())
            return None
        return dist.all_reduce(t, op=op, group=self.group, async_op=async_op)

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False):
        if self._local:
            return None
        if self.rccl is not None and t.is_cuda and t.is_contiguous():
            from ..ops import _ptr, _stream

            self._rc().rccl_broadcast(self.rccl, _ptr(t), _ptr(t), t.numel(), self._dt(t), src,
                                      _stream())
            return None
        return dist.broadcast(t, src=src, group=self.group, async_op=async_op)

    def gather(self, t: torch.Tensor, out: torch.Tensor = None, dst: int = 0):
        """Rank ``dst`` receives every rank's ``t`` into ``out`` [world, *t.shape]."""
        if self.world == 1:
            out[0].copy_(t)
            return
        if self.backend == "gloo" and t.is_cuda:  # Gloo gathers host tensors only
            h = t.cpu()
            ho = torch.empty(out.shape, dtype=out.dtype) if self.rank == dst else None
            dist.gather(h, list(ho.unbind(0)) if ho is not None else None, dst=dst,
                        group=self.group)
            if ho is not None:
                out.copy_(ho)
            return
        if self.rank == dst:
            dist.gather(t, list(out.unbind(0)), dst=dst, group=self.group)
        else:
            dist.gather(t, None, dst=dst, group=self.group)

    def isend(self, t: torch.Tensor, dst: int, tag: int = 0):
        """Point-to-point send (RCCL / Gloo); returns the Work to wait on."""
        return dist.isend(t, dst=dst, group=self.group, tag=tag)

    def irecv(self, t: torch.Tensor, src: int, tag: int = 0):
        return dist.irecv(t, src=src, group=self.group, tag=tag)

    def batch_p2p(self, sends=(), recvs=()):
        """Post point-to-point sends ``[(tensor, dst)]`` and receives ``[(tensor, src)]`` as ONE
        group (``dist.batch_isend_irecv``) and return the Works.  With RCCL, p2p ops of one rank
        pair share a communicator and stream: ungrouped, a recv posted before the matching send
        on both sides waits for a send queued behind it (deadlock); grouped, RCCL pairs them."""
        ops = [dist.P2POp(dist.irecv, t, src, group=self.group) for t, src in recvs]
        ops += [dist.P2POp(dist.isend, t, dst, group=self.group) for t, dst in sends]
        return dist.batch_isend_irecv(ops) if ops else []

    def recv_any(self, t: torch.Tensor, tag: int = 0) -> int:
        """Blocking receive from whichever rank sends first (Gloo); returns the sender."""
        return dist.recv(t, src=None, group=self.group, tag=tag)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        if self.world == 1:
            out.copy_(inp)
            return
        if self.rccl is not None and out.is_cuda:
            from ..ops import _ptr, _stream

            self._rc().rccl_all_to_all(self.rccl, _ptr(inp), _ptr(out), inp.numel() // self.world,
                                       self._dt(inp), self.world, _stream())
            return
        dist.all_to_all_single(out, inp, group=self.group)

    def barrier(self):
        if self.world > 1:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)

    def all_reduce_scalars(self, values, op="sum", device=None):
        """All-reduce a short list of Python floats (metrics averaging, ``horvod_pytorch.py:84``)."""
        if device is None:  # RCCL only reduces device tensors
            device = torch.cuda.current_device() if self.backend == "nccl" else "cpu"
        t = torch.tensor(values, dtype=torch.float64, device=device)
        if self.world > 1:
            rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                   "min": dist.ReduceOp.MIN}[op]
            dist.all_reduce(t, op=rop, group=self.group)
        return t.tolist()

    def all_gather_object(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def broadcast_object(self, obj, src=0):
        if self.world == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]


_RC_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.uint8: 3,
          torch.int8: 3, torch.int32: 4, torch.float64: 5, torch.int64: 6}
_RC_OP = {dist.ReduceOp.SUM: 0, dist.ReduceOp.MAX: 1, dist.ReduceOp.MIN: 2}


def shutdown(comm: "Comm" = None):
    if comm is not None:
        comm.close()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
