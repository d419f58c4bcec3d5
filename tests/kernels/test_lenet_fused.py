"""LeNet's fused fp32 training step (ops/csrc/lenet_f32.hip, four launches) against a float64
PyTorch reference of ``models.LeNet`` + mean cross-entropy on the CPU.

The kernels accumulate in fp32 in their own orders; the bound is a relative error of 1e-5 on the
loss / logits and 1e-4 (norm-wise) on every gradient.  Inputs come from fixed seeds: a 2x2 max-pool
window whose two largest values sit within fp32 rounding of each other could route a gradient
differently from float64, and fixed data makes such a case (none occurs for these seeds)
reproducible rather than a flake.  Batches cover whole 16-row fc tiles (64) and a ragged one (37).
"""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _setup(B, seed=0, K=10):
    from ewdml import ops
    from ewdml.models.lenet import LeNet

    ops.require()
    torch.manual_seed(seed)
    m = LeNet(num_classes=K).cuda()
    x = torch.randn(B, 1, 28, 28, device="cuda")
    y = torch.randint(0, K, (B,), device="cuda")
    return m, x, y


def _ref(m, x, y, scale=1.0):
    r = copy.deepcopy(m).double().cpu()
    out = r(x.double().cpu())
    loss = F.cross_entropy(out, y.cpu())
    (loss * scale).backward()
    return loss, out, [p.grad for p in r.parameters()]


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("B", [64, 37])
def test_lenet_fused_step_vs_fp64(B):
    from ewdml.ops import lenet

    m, x, y = _setup(B)
    assert lenet.supported(m, x, y)
    loss, out = m.fused_loss(x, y)
    loss.backward()
    torch.cuda.synchronize()
    rl, rout, rgrads = _ref(m, x, y)
    assert abs(float(loss) - float(rl)) <= 1e-5 * abs(float(rl)), (float(loss), float(rl))
    assert _rel(out, rout) < 1e-5
    names = [n for n, _ in m.named_parameters()]
    for n, p, g in zip(names, m.parameters(), rgrads):
        assert p.grad is not None and p.grad.shape == p.shape, n
        assert _rel(p.grad, g) < 1e-4, (n, _rel(p.grad, g))


def test_lenet_fused_repeat_is_bitwise_and_scales_with_the_loss_gradient():
    m, x, y = _setup(64, seed=1)
    runs = []
    for scale in (1.0, 1.0, 2.5):
        for p in m.parameters():
            p.grad = None
        loss, _ = m.fused_loss(x, y)
        (loss * scale).backward()
        torch.cuda.synchronize()
        runs.append((loss.detach().clone(), [p.grad.clone() for p in m.parameters()]))
    (l0, g0), (l1, g1), (l2, g2) = runs
    # the tickets re-arm: the second step is the first one bit for bit
    assert torch.equal(l0, l1)
    assert all(torch.equal(a, b) for a, b in zip(g0, g1))
    # d(loss)/d(loss) = 2.5: every gradient scales (the conv gradients sum products of the scaled
    # d(a2), so up to rounding)
    for a, c in zip(g0, g2):
        assert _rel(c, a * 2.5) < 1e-6


def test_lenet_trainer_uses_the_fused_step():
    import ewdml
    from ewdml.ops import lenet
    from ewdml.runtime import Trainer

    calls = []
    orig = lenet._LeNetStep.apply

    def spy(*a):
        calls.append(1)
        return orig(*a)

    lenet._LeNetStep.apply = spy
    try:
        tr = Trainer(ewdml.parse_args([
            "--network", "LeNet", "--dataset", "MNIST", "--synthetic-size", "512",
            "--batch-size", "64", "--device", "cuda", "--hip-graph", "off", "--quiet",
            "--eval-freq", "0", "--compress", "none", "--max-steps", "3"]))
        losses = [float(tr.train_step()[0]) for _ in range(3)]
    finally:
        lenet._LeNetStep.apply = orig
    assert len(calls) == 3
    assert all(v == v and v > 0 for v in losses)
