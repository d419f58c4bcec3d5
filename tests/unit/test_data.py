"""Dataset readers and the sharded device loader."""
import os

import numpy as np
import pytest
import torch

from ewdml.data import DeviceLoader, augment_cifar, load_dataset
from ewdml.data.datasets import DATASETS, _cifar_bin, read_idx

REF_LABELS = "/root/reference/PyTorch-parameter-server/mnist_data/MNIST/raw/train-labels-idx1-ubyte"


@pytest.mark.skipif(not os.path.exists(REF_LABELS), reason="reference checkout not mounted")
def test_idx_reader_on_reference_labels():
    y = read_idx(REF_LABELS)
    assert y.shape == (60000,)
    assert np.bincount(y).tolist() == [5923, 6742, 5958, 6131, 5842, 5421, 5918, 6265, 5851, 5949]
    yz = read_idx(REF_LABELS[:-len("train-labels-idx1-ubyte")] + "t10k-labels-idx1-ubyte")
    assert yz.shape == (10000,)


def test_idx_roundtrip(tmp_path):
    imgs = np.random.randint(0, 255, (7, 28, 28), dtype=np.uint8)
    hdr = (0x00000803).to_bytes(4, "big") + b"".join(d.to_bytes(4, "big") for d in imgs.shape)
    (tmp_path / "t10k-images-idx3-ubyte").write_bytes(hdr + imgs.tobytes())
    lab = np.arange(7, dtype=np.uint8)
    (tmp_path / "t10k-labels-idx1-ubyte").write_bytes(
        (0x00000801).to_bytes(4, "big") + (7).to_bytes(4, "big") + lab.tobytes())
    x, y, info = load_dataset("MNIST", str(tmp_path), train=False)
    assert x.shape == (7, 1, 28, 28) and torch.equal(x[:, 0], torch.from_numpy(imgs))
    assert y.tolist() == list(range(7)) and not info["synthetic"]


def test_cifar10_binary(tmp_path):
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rec = np.zeros((3, 3073), dtype=np.uint8)
    rec[:, 0] = [3, 1, 4]
    rec[:, 1:] = np.arange(3072) % 251
    rec.tofile(d / "test_batch.bin")
    x, y = _cifar_bin(str(tmp_path), False, None)
    assert x.shape == (3, 3, 32, 32) and y.tolist() == [3, 1, 4]
    assert int(x[0, 1, 0, 0]) == 1024 % 251


def test_svhn_mat(tmp_path):
    sio = pytest.importorskip("scipy.io")
    X = np.random.randint(0, 255, (32, 32, 3, 5), dtype=np.uint8)
    sio.savemat(tmp_path / "test_32x32.mat", {"X": X, "y": np.array([[10], [1], [2], [3], [4]])})
    x, y, _ = load_dataset("SVHN", str(tmp_path), train=False)
    assert x.shape == (5, 3, 32, 32) and y.tolist() == [0, 1, 2, 3, 4]
    assert torch.equal(x[1, 2], torch.from_numpy(X[:, :, 2, 1].copy()))


def test_synthetic_shapes():
    for name in ("MNIST", "Cifar10", "Cifar100", "SVHN"):
        x, y, info = load_dataset(name, None, synthetic_size=64)
        assert tuple(x.shape[1:]) == DATASETS[info["name"]][0]
        assert int(y.max()) < info["classes"] and x.dtype == torch.uint8


def test_sharded_loader_equal_steps_and_disjoint():
    x = torch.arange(103, dtype=torch.uint8).view(103, 1, 1, 1).expand(103, 1, 2, 2).contiguous()
    y = torch.arange(103)
    info = {"mean": (0.0,), "std": (1.0,)}
    seen = []
    lens = []
    for r in range(3):
        ld = DeviceLoader(x, y, info, 8, rank=r, world=3, seed=5)
        lens.append(len(ld))
        seen.append(torch.cat([b[1] for b in ld]))
    assert len(set(lens)) == 1 and lens[0] == 103 // 3 // 8
    allv = torch.cat(seen)
    assert allv.unique().numel() == allv.numel()  # no sample on two ranks


def test_augment_shapes_and_flip():
    x = torch.arange(2 * 3 * 32 * 32, dtype=torch.float32).view(2, 3, 32, 32)
    out = augment_cifar(x, torch.Generator().manual_seed(0))
    assert out.shape == x.shape
