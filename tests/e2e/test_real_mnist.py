"""Accuracy on real data: the reference checkout ships the 10K MNIST *test* images
(``data/MNIST/raw/t10k-images-idx3-ubyte.gz``).  LeNet is trained on 9K of them and scored on the
held-out 1K, per codec.  The report's LeNet accuracies are 96.5-98 %; top-1 % without
error feedback is expected a few points lower (the reference's Method 5 used K = 0.4, also tested)."""
import os

import pytest
import torch
import torch.nn.functional as F

from ewdml.compress import make_codec
from ewdml.data import DeviceLoader
from ewdml.data.datasets import DATASETS, _mnist
from ewdml.models import build_model
from ewdml.optim import FlatSGD
from ewdml.parallel import Comm, FlatModel, GradientExchange

ROOT = "/root/reference/data"
pytestmark = [pytest.mark.slow,
              pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "MNIST", "raw",
                                                                 "t10k-images-idx3-ubyte.gz")),
                                 reason="reference MNIST test images not mounted")]


# floors: the report's lowest LeNet accuracy (Method 5, 96.5 %) for every accuracy-preserving
# configuration; top-1 % without error feedback (132x fewer bytes, no residual) loses ~3 points
@pytest.mark.parametrize("kind,ef,norm,ratio,floor", [("none", False, "max", 0.01, 96.5),
                                                      ("topk_qsgd", False, "max", 0.01, 93.0),
                                                      ("topk_qsgd", True, "max", 0.01, 96.5),
                                                      ("topk_qsgd", False, "l2", 0.4, 96.5),
                                                      ("qsgd", False, "l2", 0.01, 96.5)])
def test_lenet_real_mnist_holdout(kind, ef, norm, ratio, floor):
    torch.manual_seed(0)
    x, y = _mnist(ROOT, train=False)
    info = {"mean": DATASETS["mnist"][2], "std": DATASETS["mnist"][3]}
    tr = DeviceLoader(x[:9000], y[:9000], info, 64, seed=1)
    te = DeviceLoader(x[9000:], y[9000:], info, 1000, shuffle=False, drop_last=False)
    m = build_model("LeNet")
    flat = FlatModel(m)
    opt = FlatSGD(flat, lr=0.01, momentum=0.9)
    ex = GradientExchange(flat, Comm(), make_codec(kind, ratio=ratio, norm=norm), opt,
                          error_feedback=ef)
    for _ in range(1500):
        xb, yb = tr.next()
        flat.zero_grad()
        ex.begin()
        F.cross_entropy(m(xb), yb).backward()
        ex.finish()
    with torch.no_grad():
        xb, yb = next(iter(te))
        acc = 100 * (m(xb).argmax(1) == yb).float().mean().item()
    assert acc >= floor, f"{kind} ef={ef}: holdout accuracy {acc:.1f}% < {floor}%"
