"""ewdml -- MI355X-native gradient-compressed data-parallel training.

A from-scratch re-design of the capabilities of "Efficient Workers in Distributed Machine
Learning" (PyTorch parameter server + Horovod, QSGD and top-k gradient compression) for AMD
Instinct MI355X: one process per GPU over RCCL/xGMI, flat bucketed gradients with
backward-overlapped compressed exchange, and hand-written CDNA4 (gfx950) HIP kernels for top-k
selection, QSGD quantisation, packing, fused decode + average + SGD, and the flat optimizers.

Layout (see README.md):
  models/    LeNet, VGG-11/13/16/19(+BN), ResNet-18..152 (CIFAR + ImageNet stems), Horovod MnistNet
  compress/  bucket plans, packed payload layouts, codecs, torch oracle, counter RNG
  ops/       gfx950 HIP kernels (csrc/) + validated Python launchers
  parallel/  communicator, flat buckets, overlap engine, PS topology, local SGD, Horovod-style API
  optim/     flat SGD / Adam with explicit gradients
  data/      device-resident datasets (MNIST/CIFAR/SVHN readers, synthetic), sharded loader
  runtime/   trainer (worker / server roles), evaluator
  utils/     metrics + byte accounting, atomic checkpoints
"""
__version__ = "0.1.0"

import os as _os

# Kernel arguments in device memory rather than host-coherent memory.  Must be set before the HIP
# runtime initialises (first device call), which importing this package precedes.  Unprofiled
# this matches the runtime default on MI355X (=0 costs ResNet-50 5-7 %); pinning it keeps it so
# under rocprofv3, where the VGG-11 step graph otherwise shows a ~55 us mid-backward dispatch
# stall that the unprofiled run does not have (profiles/ab/device_kernargs.txt).
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

from .config import Config, build_parser, parse_args  # noqa: E402
from .parallel.horovod import (Adasum, Average, Compression, DistributedOptimizer,  # noqa: E402
                               Sum, allreduce, broadcast_optimizer_state,
                               broadcast_parameters, init, local_rank, local_size, rank, size)

__all__ = [
    "Config", "build_parser", "parse_args", "init", "rank", "size", "local_rank", "local_size",
    "allreduce", "broadcast_parameters", "broadcast_optimizer_state", "DistributedOptimizer",
    "Compression", "Average", "Sum", "Adasum",
]
