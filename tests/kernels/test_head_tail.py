"""The fused VGG classifier tail (ops/csrc/head_tail.hip: fc2 + ReLU + fc3 + cross-entropy in one
launch, its backward in one more) against a float64 reference on the CPU (dropout off), and with
dropout on against head.hip's per-Linear kernels + the cross-entropy kernel (the same counter
masks: the first Linear and its dropouts run the same kernels on both paths)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _cls(seed=3):
    from ewdml import ops
    from ewdml.models import build_model

    ops.require()
    torch.manual_seed(seed)
    return build_model("vgg11", 10).cuda().classifier


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("B", [128, 37])
def test_tail_matches_fp64_without_dropout(B):
    from ewdml.ops import head

    cls = _cls()
    for mod in cls:
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = torch.randn(B, 512, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    xa = x.clone().requires_grad_(True)
    tail, head._TAIL = head._TAIL, True
    try:
        assert head.tail_supported(cls, xa, y)
    finally:
        head._TAIL = tail
    loss, logits = head.vgg_loss(cls, xa, y)
    loss.backward()
    ga = [p.grad.clone() for p in cls.parameters()]
    ref = copy.deepcopy(cls).double().cpu()
    xb = x.double().cpu().requires_grad_(True)
    rl = F.cross_entropy(ref(xb), y.cpu())
    rl.backward()
    assert abs(float(loss) - float(rl)) <= 1e-5 * abs(float(rl))
    assert _rel(logits, ref(xb)) < 1e-5
    assert _rel(xa.grad, xb.grad) < 1e-4
    for a, p in zip(ga, ref.parameters()):
        assert a.shape == p.shape
        assert _rel(a, p.grad) < 1e-4, _rel(a, p.grad)


def test_tail_matches_head_kernels_with_dropout():
    from ewdml.ops import head
    from ewdml.ops.nn import cross_entropy

    cls = _cls(5)
    cls.train()
    ref = copy.deepcopy(cls)
    x = torch.randn(128, 512, device="cuda")
    y = torch.randint(0, 10, (128,), device="cuda")
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    loss, logits = head.vgg_loss(cls, xa, y)
    loss.backward()
    out = head.vgg_head(ref, xb)  # fresh counters on both copies: the same masks
    rl = cross_entropy(out, y)
    rl.backward()
    assert abs(float(loss) - float(rl)) <= 1e-5 * abs(float(rl))
    assert _rel(logits, out) < 1e-5
    assert _rel(xa.grad, xb.grad) < 1e-4
    for a, b in zip(cls.parameters(), ref.parameters()):
        assert _rel(a.grad, b.grad) < 1e-4


def test_vgg_fused_loss_in_trainer_step():
    """VGG.fused_loss is what the trainer runs (fp32, fused kernels): the loss falls over a few
    steps and the head tail launched."""
    import ewdml
    from ewdml.ops import head
    from ewdml.runtime import Trainer

    calls = []
    orig = head._HeadTail.apply

    def spy(*a):
        calls.append(1)
        return orig(*a)

    head._HeadTail.apply = spy
    tail = head._TAIL
    head._TAIL = True  # opt-in path
    try:
        tr = Trainer(ewdml.parse_args([
            "--network", "VGG11", "--dataset", "Cifar10", "--synthetic-size", "256",
            "--batch-size", "32", "--device", "cuda", "--hip-graph", "off", "--quiet",
            "--eval-freq", "0", "--compress", "none", "--amp", "none", "--max-steps", "3"]))
        losses = [float(tr.train_step()[0]) for _ in range(3)]
    finally:
        head._HeadTail.apply = orig
        head._TAIL = tail
    assert len(calls) == 3
    assert all(v == v for v in losses)
