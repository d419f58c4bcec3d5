"""Data parallelism: communicator, flat buckets, overlap engine, PS topology, local SGD,
and the Horovod-style ``DistributedOptimizer`` API."""
from .comm import Comm, init_distributed, shutdown
from .engine import GradientExchange, Stopwatch, sync_buffers, sync_params
from .flat import FlatModel
from .local_sgd import LocalSGDExchange
from .ps import PSExchange

__all__ = ["Comm", "init_distributed", "shutdown", "GradientExchange", "Stopwatch",
           "sync_buffers", "sync_params", "FlatModel", "LocalSGDExchange", "PSExchange"]
