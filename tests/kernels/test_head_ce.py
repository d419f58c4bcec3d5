"""The cross-entropy riding in the VGG classifier's last Linear (ops/csrc/head.hip HdCe, ops/head.py
_HeadLinearCE) against head.hip's Linear kernel + the cross-entropy kernel (ops/nn.py
cross_entropy): the same loss, logits and gradients bit for bit (k_ce_fwd's expressions and its
summation order), with the trainer's unit seed and with an arbitrary upstream gradient."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cls(dtype, seed=3):
    from ewdml import ops
    from ewdml.models import build_model

    ops.require()
    torch.manual_seed(seed)
    return build_model("vgg11", 10).cuda().to(dtype).classifier


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B", [128, 37])
@pytest.mark.parametrize("unit", [True, False])
def test_head_ce_matches_linear_plus_cross_entropy(dtype, B, unit):
    from ewdml.ops import head
    from ewdml.ops import nn as fnn

    cls = _cls(dtype)
    cls.train()
    saved, head._HEAD_CE = head._HEAD_CE, True  # opt-in path
    ref = copy.deepcopy(cls)
    x = torch.randn(B, 512, device="cuda").to(dtype)
    y = torch.randint(0, 10, (B,), device="cuda")
    seed = torch.ones((), device="cuda")
    fnn.set_unit_grad(seed if unit else None)
    try:
        g = seed if unit else torch.full((), 0.37, device="cuda")
        xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
        assert head.head_ce_supported(cls, xa, y)
        loss, logits = head.vgg_head_loss(cls, xa, y)
        loss.backward(g)
        out = head.vgg_head(ref, xb)  # fresh dropout counters on both copies: the same masks
        rl = fnn.cross_entropy(out, y)
        rl.backward(g)
    finally:
        fnn.set_unit_grad(None)
        head._HEAD_CE = saved
    assert torch.equal(loss, rl)
    assert torch.equal(logits, out.detach())
    assert torch.equal(xa.grad, xb.grad)
    for a, b in zip(cls.parameters(), ref.parameters()):
        assert torch.equal(a.grad, b.grad)


def test_vgg_trainer_step_runs_head_ce():
    """With EWDML_HEAD_CE on, VGG.fused_loss takes the loss-carrying head in the trainer's fp32
    step: it launches each step and the loss is finite."""
    import ewdml
    from ewdml.ops import head
    from ewdml.runtime import Trainer

    calls = []
    orig = head._HeadLinearCE.apply

    def spy(*a):
        calls.append(1)
        return orig(*a)

    head._HeadLinearCE.apply = spy
    saved, head._HEAD_CE = head._HEAD_CE, True  # opt-in path
    try:
        tr = Trainer(ewdml.parse_args([
            "--network", "VGG11", "--dataset", "Cifar10", "--synthetic-size", "256",
            "--batch-size", "32", "--device", "cuda", "--hip-graph", "off", "--quiet",
            "--eval-freq", "0", "--compress", "none", "--amp", "none", "--max-steps", "3"]))
        losses = [float(tr.train_step()[0]) for _ in range(3)]
    finally:
        head._HeadLinearCE.apply = orig
        head._HEAD_CE = saved
    assert len(calls) == 3
    assert all(v == v for v in losses)


@pytest.mark.parametrize("B", [128, 64])
@pytest.mark.parametrize("cbias", [False, True])
def test_bn_backward_rides_in_head_input_gradient(B, cbias):
    """The backward statistics + finalisation of the BN + ReLU + 2x2 pool layer feeding VGG's
    classifier, formed in the first Linear's input-gradient blocks (ops/csrc/head.hip HdBnB),
    against its own statistics + finalize launches (EWDML_HEAD_BN=0): the same gradients up to
    the order of the fp32 sums."""
    from ewdml.ops import head
    from ewdml.ops import nn as fnn

    cls0 = _cls(torch.float32, seed=7)
    cls0.train()
    bn0 = torch.nn.BatchNorm2d(512).cuda()
    with torch.no_grad():
        bn0.weight.uniform_(0.5, 1.5)
        bn0.bias.uniform_(-0.3, 0.3)
    h0 = torch.randn(B, 512, 2, 2, device="cuda").contiguous(memory_format=torch.channels_last)
    cb0 = torch.randn(512, device="cuda") * 0.1
    g = torch.randn(B, 10, device="cuda")
    res = []
    saved = head._HEAD_BN
    try:
        for on in (True, False):
            head._HEAD_BN = on
            rides, used = head.BN_RIDES, fnn.PRE_BWD_USED
            cls, bn = copy.deepcopy(cls0), copy.deepcopy(bn0)
            h = h0.clone().requires_grad_(True)
            cb = cb0.clone().requires_grad_(True) if cbias else None
            feat = fnn.bn_act(h, bn, "relu", pool=True, cbias=cb)
            out = head.vgg_head(cls, feat.flatten(1), getattr(feat, "_ew_bn_node", None))
            out.backward(g)
            assert (head.BN_RIDES > rides) == on and (fnn.PRE_BWD_USED > used) == on
            # (a conv bias feeding BN has an exact gradient of 0: its fp32 value is rounding
            # noise, no comparison)
            res.append([h.grad, bn.weight.grad, bn.bias.grad] + [p.grad for p in cls.parameters()])
    finally:
        head._HEAD_BN = saved
    for a, b in zip(*res):
        a, b = a.double(), b.double()
        assert float((a - b).norm() / (b.norm() + 1e-30)) < 1e-5
