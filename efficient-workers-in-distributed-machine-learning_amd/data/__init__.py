"""Datasets and loaders.

Parity: ``PyTorch-parameter-server/src/util.py:20-106`` (``prepare_data``: MNIST, CIFAR-10/100 with
reflect-pad-4 + random-crop-32 + h-flip, SVHN) and ``src/data/data_prepare.py``.

MI355X-first differences:
  * torchvision is not required: MNIST IDX, CIFAR binary and SVHN .mat files are parsed directly
    (numpy / scipy.io -- no pickle), and ``synthetic`` datasets of the same shapes are generated
    on the device for benchmarks (there is no network to download anything);
  * the whole dataset is kept resident in HBM (CIFAR-10 is 150 MB of uint8; the MI355X has 288 GB)
    and batches are gathered + augmented on the GPU, so the input pipeline never stalls a step;
  * the sampler shards the permutation across ranks and gives every rank the same number of
    steps (the reference iterates the full set on every worker with no sampler and deadlocks
    when worker and master step counts differ: SURVEY Appendix B #2, #3).
"""
from .datasets import DATASETS, dataset_info, load_dataset
from .loader import DeviceLoader, augment_cifar

__all__ = ["DATASETS", "dataset_info", "load_dataset", "DeviceLoader", "augment_cifar"]
