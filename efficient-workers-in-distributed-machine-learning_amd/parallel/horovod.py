"""Horovod-style API on top of the ewdml engine (no Horovod, no MPI).

Parity with what ``horvod_pytorch.py`` uses (``:119-205``): ``init``, ``rank``/``size``/
``local_rank``/``local_size``, ``allreduce`` (metric averaging, ``:84-87``),
``broadcast_parameters`` / ``broadcast_optimizer_state`` (``:187-188``), and
``DistributedOptimizer(optimizer, named_parameters, compression, op=Average|Sum|Adasum,
gradient_predivide_factor, backward_passes_per_step)`` (``:197-201``) with pluggable compression
(``Compression.none/fp16`` and the project's QSGD compressor, ``horovod_compression.py``).

How it maps: the wrapped optimizer's parameters become views of a flat bucketed buffer; gradient
buckets are exchanged with backward overlap by :class:`GradientExchange` (RCCL all-reduce for
none/fp16/bf16, packed all-gather for qsgd/topk/topk_qsgd -- the fusion buffer of
``horovodrun --fusion-threshold-mb`` is ``bucket_mb``); ``step()`` writes the averaged gradient into
``p.grad`` and calls the wrapped optimizer.  Unlike the reference's Horovod QSGD (which *averages
levels* across ranks and decodes with the local norm), every rank's payload
is decoded with its own scale before averaging.

``Adasum`` (``--use-adasum``, ``horvod_pytorch.py:35-36``): the dense gradients are combined with the
Adasum rule in a fixed binary tree over ranks by pairwise exchanges between the tree's groups
(``adasum_tree``: D log2 N bytes per rank), identical on every rank.
"""
import os

import torch

from ..compress.codecs import Codec
from .comm import Comm, init_distributed
from .engine import GradientExchange
from .flat import FlatModel

Average = "average"
Sum = "sum"
Adasum = "adasum"

_COMM = None


def init(backend: str = None, timeout_s: float = None):
    global _COMM
    if torch.cuda.is_available() and backend != "gloo":
        torch.cuda.set_device(local_rank())
        dev = torch.device("cuda", local_rank())
    else:
        dev = None
    _COMM = init_distributed(backend, timeout_s, device=dev)
    return _COMM


def _comm() -> Comm:
    global _COMM
    if _COMM is None:
        _COMM = Comm()
    return _COMM


def rank() -> int:
    return _comm().rank


def size() -> int:
    return _comm().world


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def local_size() -> int:
    return int(os.environ.get("LOCAL_WORLD_SIZE", str(size())))


def allreduce(tensor: torch.Tensor, name: str = None, op: str = Average) -> torch.Tensor:
    out = tensor.detach().clone()
    c = _comm()
    if c.world > 1:
        c.all_reduce(out)
        if op == Average:
            out /= c.world
    return out


def broadcast_parameters(params, root_rank: int = 0):
    """``params``: a state_dict, a list of (name, tensor) or of tensors."""
    c = _comm()
    items = params.values() if isinstance(params, dict) else \
        [p[1] if isinstance(p, tuple) else p for p in params]
    for t in items:
        if torch.is_tensor(t):
            c.broadcast(t.data, src=root_rank)


def broadcast_optimizer_state(optimizer, root_rank: int = 0):
    """Every rank ends with the root's optimizer state and hyper-parameters.  State the root has
    but a rank has not created yet (a fresh optimizer has empty ``state``) is first allocated
    from the root's description, so every rank issues the same sequence of broadcasts."""
    c = _comm()
    if c.world == 1:
        return
    inner = getattr(optimizer, "optimizer", optimizer)
    params = [p for g in inner.param_groups for p in g["params"]]
    spec = None
    if c.rank == root_rank:
        spec = []
        for p in params:
            st = inner.state.get(p, {})
            spec.append([(k, tuple(v.shape), str(v.dtype), v.device.type)
                         for k, v in sorted(st.items()) if torch.is_tensor(v)])
    spec = c.broadcast_object(spec, src=root_rank)
    for p, entries in zip(params, spec):
        st = inner.state.setdefault(p, {})
        for k, shape, dt, devtype in entries:
            v = st.get(k)
            if not (torch.is_tensor(v) and tuple(v.shape) == tuple(shape)):
                dtype = getattr(torch, dt.replace("torch.", ""))
                v = torch.zeros(shape, dtype=dtype, device=p.device if devtype != "cpu" else "cpu")
                st[k] = v
            if v.numel() == 0:
                continue
            if v.device.type == "cpu" and c.backend not in ("gloo", "local"):
                t = v.to(p.device)  # RCCL broadcasts device memory only
                c.broadcast(t, src=root_rank)
                v.copy_(t.cpu())
            else:
                c.broadcast(v.data, src=root_rank)
    hp = c.broadcast_object([{k: v for k, v in g.items() if k != "params"}
                             for g in inner.param_groups], src=root_rank)
    for g, h in zip(inner.param_groups, hp):
        g.update(h)


class Compression:
    """Compression choices (``hvd.Compression.none`` / ``.fp16`` plus the project's codecs)."""

    none = "none"
    fp16 = "fp16"
    bf16 = "bf16"

    @staticmethod
    def qsgd(levels: int = 127, bits: int = 8, norm: str = "l2"):
        return Codec("qsgd", levels=levels, bits=bits, norm=norm)

    @staticmethod
    def topk(ratio: float = 0.01):
        return Codec("topk", ratio=ratio)

    @staticmethod
    def topk_qsgd(ratio: float = 0.01, levels: int = 127, bits: int = 8, norm: str = "max"):
        return Codec("topk_qsgd", ratio=ratio, levels=levels, bits=bits, norm=norm)


def _as_codec(compression) -> Codec:
    if isinstance(compression, Codec):
        return compression
    if isinstance(compression, str):
        return Codec(compression)
    name = getattr(compression, "__name__", str(compression)).lower()
    if "qsgd" in name:  # e.g. the reference's horovod_compression.QSGDCompressor class
        return Compression.qsgd()
    if "fp16" in name:
        return Codec("fp16")
    return Codec("none")


class _OptAdapter:
    """Lets GradientExchange drive a torch optimizer (non-fused path)."""

    fusable = False

    def __init__(self):
        self.steps = 0

    def end_step(self):
        self.steps += 1


def adasum_pair(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """The Adasum rule for two gradients (a: the lower-rank group's, b: the higher one's), in
    float64: ``(1 - a.b / 2|a|^2) a + (1 - a.b / 2|b|^2) b`` (a zero vector keeps weight 1)."""
    a, b = a.double(), b.double()
    dot = torch.dot(a, b)
    na, nb = torch.dot(a, a), torch.dot(b, b)
    one = torch.ones((), dtype=a.dtype, device=a.device)
    ca = torch.where(na > 0, 1 - dot / (2 * torch.where(na > 0, na, one)), one)
    cb = torch.where(nb > 0, 1 - dot / (2 * torch.where(nb > 0, nb, one)), one)
    return (ca * a + cb * b).float()


def adasum_combine(grads: torch.Tensor) -> torch.Tensor:
    """Adasum of ``grads`` [N, D] over a fixed binary tree (rank order): at level l the groups of
    2^l consecutive ranks combine pairwise, a trailing unpaired group passes through."""
    vs = list(grads.unbind(0))
    while len(vs) > 1:
        nxt = [adasum_pair(vs[i], vs[i + 1]) for i in range(0, len(vs) - 1, 2)]
        if len(vs) % 2:
            nxt.append(vs[-1])
        vs = nxt
    return vs[0]


def adasum_tree(comm, g: torch.Tensor) -> torch.Tensor:
    """The same tree as :func:`adasum_combine`, run distributed by point-to-point exchanges:
    at level l every rank holds its group's combined vector; it swaps it with one rank of the
    partner group (group index xor 1) and both combine (lower group first), so after
    ceil(log2 N) levels every rank holds the root.  O(D) memory and D * log2 N bytes per rank on
    the wire, instead of all-gathering N vectors (N * D), and bitwise the same result on every
    rank (the same operands in the same order).  A trailing partner group smaller than the
    group serves several ranks: each of its members sends to the ranks that map to it."""
    rank, n = comm.rank, comm.world
    v = g.detach().clone()
    level = 0
    while (1 << level) < n:
        size = 1 << level
        grp = rank // size
        pg = grp ^ 1
        lo, hi = pg * size, min(n, (pg + 1) * size)  # partner group's ranks
        if lo >= n:  # no partner group: pass through
            level += 1
            continue

        def src_of(r):  # the partner-group rank that serves rank r
            q = (r // size ^ 1) * size + r % size
            return min(q, min(n, ((r // size ^ 1) + 1) * size) - 1)

        other = torch.empty_like(v)
        # the partner ranks that take their vector from me; the level's sends and receive are
        # posted as one group (separate isend / irecv to one peer deadlock on RCCL)
        sends = [(v, r) for r in range(lo, hi) if src_of(r) == rank]
        for q in comm.batch_p2p(sends=sends, recvs=[(other, src_of(rank))]):
            q.wait()
        v = adasum_pair(v, other) if grp < pg else adasum_pair(other, v)
        level += 1
    return v


class _DistributedOptimizer:
    def __init__(self, optimizer, named_parameters=None, compression=Compression.none,
                 backward_passes_per_step: int = 1, op: str = Average,
                 gradient_predivide_factor: float = 1.0, bucket_mb: float = 32.0):
        self.optimizer = optimizer
        self.comm = _comm()
        params = [p for g in optimizer.param_groups for p in g["params"] if p.requires_grad]
        self.flat = FlatModel(params, bucket_bytes=int(bucket_mb * (1 << 20)))
        self.op = op
        self.bpps = max(1, int(backward_passes_per_step))
        codec = Codec("none") if op == Adasum else _as_codec(compression)
        self.exchange = GradientExchange(self.flat, self.comm, codec, _OptAdapter(),
                                         overlap=(self.bpps == 1 and op != Adasum),
                                         predivide=gradient_predivide_factor)
        self._synced = False
        self.exchange.begin()

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()
        self.flat.reattach_grads()

    def synchronize(self):
        """Finish the gradient exchange; ``p.grad`` then holds the averaged gradient."""
        if self._synced:
            return
        if self.op == Adasum and self.comm.world > 1:
            g = self.flat.grad
            g.copy_(adasum_tree(self.comm, g))  # pairwise tree exchange (horvod_pytorch.py:35-36)
            self.exchange._active = False
        else:
            self.exchange.finish(apply=False)
            self.exchange.decode_average()
            if self.op == Sum:
                self.flat.grad.mul_(self.comm.world)
        self._synced = True

    def step(self, closure=None):
        """Reduce the gradients accumulated over the preceding ``backward_passes_per_step``
        backward passes (autograd sums them in place) and apply the wrapped optimizer, as
        Horovod's ``backward_passes_per_step`` prescribes: N backward passes, then one step."""
        self.synchronize()
        out = self.optimizer.step(closure) if closure is not None else self.optimizer.step()
        self._synced = False
        self.exchange.begin()
        return out

    def state_dict(self):
        return self.optimizer.state_dict()

    def load_state_dict(self, sd):
        self.optimizer.load_state_dict(sd)


def DistributedOptimizer(optimizer, named_parameters=None, compression=Compression.none,
                         backward_passes_per_step=1, op=Average, gradient_predivide_factor=1.0,
                         bucket_mb=32.0):
    return _DistributedOptimizer(optimizer, named_parameters, compression,
                                 backward_passes_per_step, op, gradient_predivide_factor,
                                 bucket_mb)
