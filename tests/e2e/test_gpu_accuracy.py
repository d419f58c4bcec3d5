"""Accuracy of the GPU training path (HIP codecs, fused kernels, full HIP-graph steps).

* LeNet on real MNIST: the reference ships only the 10K test images (``tests/fixtures/mnist``,
  copied from its ``data/MNIST/raw/t10k-*``); train on 9K, score the held-out 1K.  Floors: the
  report's Method 5 LeNet figure, 96.5 % (``Report.zip:Top1 Accuracy.png``), for the
  dense exchange, for top-1 % + 8-bit QSGD with error feedback (the bench codec) and for the
  report's Method 5 codec itself (top-40 % + QSGD), in fp32 and in bf16.
* VGG-11-BN on a learnable synthetic CIFAR-shaped set (class prototypes + noise): the fused bf16
  stack (MFMA convs, fused BN / head kernels, HIP graph) and the fp32 fused stack must track the
  module-by-module fp32 path (MIOpen, PyTorch BN / head) over 300 steps.  Real CIFAR is absent from
  the reference checkout, so CIFAR accuracy parity stays unpinned.
"""
import os

import pytest
import torch

import ewdml
from ewdml import ops

pytestmark = pytest.mark.gpu

MNIST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fixtures",
                     "mnist")


def _train(flags, steps):
    from ewdml.runtime import Trainer

    torch.manual_seed(0)
    tr = Trainer(ewdml.parse_args(flags + ["--max-steps", str(steps)]))
    losses = []
    for _ in range(steps):
        loss, _ = tr.train_step()
        losses.append(loss)
    torch.cuda.synchronize()
    return tr, [float(v.detach()) for v in losses]


LENET = ["--network", "LeNet", "--dataset", "MNIST", "--data-dir", MNIST,
         "--holdout-from-test", "1000", "--batch-size", "64", "--lr", "0.01", "--momentum", "0.9",
         "--eval-freq", "0", "--quiet", "--device", "cuda", "--hip-graph", "full",
         "--graph-warmup", "2", "--test-batch-size", "1000"]


@pytest.mark.parametrize("amp", ["none", "bf16", "bf16_autocast"])
@pytest.mark.parametrize("codec", ["dense", "topk1_qsgd_ef", "method5"])
def test_lenet_real_mnist_gpu(codec, amp, monkeypatch):
    """``bf16``: --amp bf16 keeps LeNet's fused fp32 step (faster and more precise: the trainer's
    amp_kept_fp32); ``bf16_autocast`` (EWDML_AMP_FUSED_FP32=0): the bf16 autocast path itself."""
    ops.require()
    if amp == "bf16_autocast":
        monkeypatch.setenv("EWDML_AMP_FUSED_FP32", "0")
    extra = {"dense": ["--compress", "none"],
             "topk1_qsgd_ef": ["--compress", "topk_qsgd", "--topk-ratio", "0.01",
                               "--error-feedback"],
             "method5": ["--compress", "topk_qsgd", "--topk-ratio", "0.4", "--qsgd-norm", "l2",
                         "--no-error-feedback"]}
    tr, losses = _train(LENET + ["--amp", amp.split("_")[0]] + extra[codec], 1500)
    assert tr.graph_mode == "full" and tr._graphs is not None
    assert tr.compute_dtype == ("bf16" if amp == "bf16_autocast" else "fp32")
    ev = tr.evaluate()
    assert ev["samples"] == 1000
    assert ev["top1"] >= 96.5, f"{codec}/{amp}: holdout top-1 {ev['top1']:.1f}% < 96.5%"


VGG = ["--network", "VGG11", "--dataset", "Cifar10", "--batch-size", "64", "--synthetic-size",
       "4096", "--lr", "0.02", "--momentum", "0.9", "--eval-freq", "0", "--quiet", "--device",
       "cuda", "--compress", "topk_qsgd", "--topk-ratio", "0.01", "--error-feedback",
       "--graph-warmup", "2"]


def test_vgg11_fused_stack_tracks_unfused_fp32():
    ops.require()
    steps = 300
    _, ref = _train(VGG + ["--fused-nn", "off", "--amp", "none", "--hip-graph", "off"], steps)
    _, f32 = _train(VGG + ["--fused-nn", "on", "--amp", "none", "--hip-graph", "full"], steps)
    _, b16 = _train(VGG + ["--fused-nn", "on", "--amp", "bf16", "--hip-graph", "full"], steps)

    def tail(v):
        return sum(v[-50:]) / 50

    # learnable: the loss falls well below chance (ln 10 = 2.30)
    assert tail(ref) < 1.0, tail(ref)
    # the fused stacks converge like the reference composition (stated band: 0.15 nats on the
    # mean of the last 50 losses; dropout masks and codec rounding differ between the paths)
    assert abs(tail(f32) - tail(ref)) < 0.15, (tail(f32), tail(ref))
    assert abs(tail(b16) - tail(ref)) < 0.15, (tail(b16), tail(ref))
