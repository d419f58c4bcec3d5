"""Dataset readers (uint8 images + int64 labels, kept as tensors).

Formats (all parsed without executing anything from the file):
  * MNIST: IDX files ``{train,t10k}-{images-idx3,labels-idx1}-ubyte[.gz]`` under
    ``<root>/MNIST/raw`` or ``<root>`` (the layout ``torchvision.datasets.MNIST`` downloads).
  * CIFAR-10/100: the *binary* distributions (``cifar-10-batches-bin/data_batch_{1..5}.bin``,
    ``cifar-100-binary/{train,test}.bin``).  The python-pickle distribution is deliberately not
    supported (unpickling is code execution).
  * SVHN: ``{train,test}_32x32.mat`` via ``scipy.io.loadmat``.
  * ``synthetic``: class-conditional images of the dataset's shape generated on the device (a fixed
    random template per class plus Gaussian noise), so a run on it really learns.
"""
import gzip
import os

import numpy as np
import torch

# name -> (shape C,H,W, classes, normalisation mean, std)  (util.py:23-104)
DATASETS = {
    "mnist": ((1, 28, 28), 10, (0.1307,), (0.3081,)),
    "cifar10": ((3, 32, 32), 10, (125.3 / 255, 123.0 / 255, 113.9 / 255),
                (63.0 / 255, 62.1 / 255, 66.7 / 255)),
    "cifar100": ((3, 32, 32), 100, (125.3 / 255, 123.0 / 255, 113.9 / 255),
                 (63.0 / 255, 62.1 / 255, 66.7 / 255)),
    "svhn": ((3, 32, 32), 10, (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)),
    "imagenet": ((3, 224, 224), 1000, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),
}
_ALIASES = {"cifar": "cifar10", "cifar-10": "cifar10", "cifar-100": "cifar100"}


def canonical(name: str) -> str:
    k = name.strip().lower()
    k = _ALIASES.get(k, k)
    if k not in DATASETS:
        raise ValueError(f"unknown dataset {name!r}; known: {sorted(DATASETS)}")
    return k


def dataset_info(name: str):
    return DATASETS[canonical(name)]


def _open(path):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def read_idx(path) -> np.ndarray:
    """Parse an IDX file (MNIST): magic 0x00000803 (images) or 0x00000801 (labels)."""
    with _open(path) as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    if magic >> 8 != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file (magic {magic:#x})")
    ndim = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(ndim)]
    arr = np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim)
    if arr.size != int(np.prod(dims)):
        raise ValueError(f"{path}: truncated ({arr.size} of {int(np.prod(dims))} bytes)")
    return arr.reshape(dims)


def _mnist(root, train):
    split = "train" if train else "t10k"
    for d in (os.path.join(root, "MNIST", "raw"), root):
        try:
            x = read_idx(os.path.join(d, f"{split}-images-idx3-ubyte"))
            y = read_idx(os.path.join(d, f"{split}-labels-idx1-ubyte"))
            return torch.from_numpy(x.copy()).unsqueeze(1), torch.from_numpy(y.astype(np.int64))
        except FileNotFoundError:
            continue
    raise FileNotFoundError(f"MNIST {split} IDX files not found under {root}")


def _cifar_bin(root, train, coarse_fine):
    if coarse_fine is None:  # CIFAR-10: <1 label byte><3072 image bytes>
        d = os.path.join(root, "cifar-10-batches-bin")
        files = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
        rec, lab = 3073, 0
    else:  # CIFAR-100: <coarse><fine><3072>
        d = os.path.join(root, "cifar-100-binary")
        files = ["train.bin" if train else "test.bin"]
        rec, lab = 3074, 1
    xs, ys = [], []
    for f in files:
        raw = np.fromfile(os.path.join(d, f), dtype=np.uint8).reshape(-1, rec)
        ys.append(raw[:, lab].astype(np.int64))
        xs.append(raw[:, rec - 3072:].reshape(-1, 3, 32, 32))
    return torch.from_numpy(np.concatenate(xs)), torch.from_numpy(np.concatenate(ys))


def _svhn(root, train):
    from scipy.io import loadmat

    m = loadmat(os.path.join(root, "train_32x32.mat" if train else "test_32x32.mat"))
    x = np.transpose(m["X"], (3, 2, 0, 1)).copy()  # HWCN -> NCHW
    y = m["y"].astype(np.int64).flatten()
    y[y == 10] = 0
    return torch.from_numpy(x), torch.from_numpy(y)


def synthetic(shape, num_classes, size, seed=0, device="cpu", noise=0.6, chunk=2048):
    """Learnable synthetic uint8 images: per-class template + noise, labels uniform.  Generated on
    ``device`` in chunks (a 224x224 set never materialises in fp32 all at once)."""
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(1234 + seed)
    templates = torch.rand((num_classes,) + tuple(shape), generator=g, device=dev)
    y = torch.randint(0, num_classes, (size,), generator=g, device=dev)
    x = torch.empty((size,) + tuple(shape), dtype=torch.uint8, device=dev)
    for s in range(0, size, chunk):
        yy = y[s:s + chunk]
        v = templates[yy] + (noise * 0.25) * torch.randn((yy.numel(),) + tuple(shape),
                                                         generator=g, device=dev)
        x[s:s + chunk] = (v.clamp_(0, 1) * 255).to(torch.uint8)
    return x, y


def load_dataset(name: str, root: str = None, train: bool = True, synthetic_size: int = 0,
                 seed: int = 0, device="cpu"):
    """Returns (x uint8 [N,C,H,W], y int64 [N], info).  ``root=None`` or ``'synthetic'`` (or a
    missing root) -> synthetic data of the dataset's shape."""
    key = canonical(name)
    shape, ncls, mean, std = DATASETS[key]
    use_syn = root in (None, "", "synthetic") or synthetic_size > 0
    if not use_syn:
        if key == "mnist":
            x, y = _mnist(root, train)
        elif key == "cifar10":
            x, y = _cifar_bin(root, train, None)
        elif key == "cifar100":
            x, y = _cifar_bin(root, train, True)
        elif key == "svhn":
            x, y = _svhn(root, train)
        else:
            raise FileNotFoundError(f"no reader for real {key} data; use synthetic")
    else:
        n = synthetic_size or (50000 if key != "mnist" else 60000)
        if not train:
            n = max(1000, n // 5)
        x, y = synthetic(shape, ncls, n, seed=seed + (0 if train else 1), device=device)
    return x.to(device), y.to(device), {"name": key, "shape": shape, "classes": ncls,
                                        "mean": mean, "std": std, "synthetic": use_syn}
