"""Numerics of the model-side HIP kernels (ops/csrc/nn.hip) against plain PyTorch fp32.

* fused NHWC BatchNorm(+conv bias)+ReLU(+2x2 max pool): forward output, running statistics,
  num_batches_tracked, and the gradients of the input, gamma, beta and the conv bias;
* 2x2 max pool (NCHW and channels_last): exact values, exact gradient routing (ties included);
* VGG-11 with the fused feature stack vs the module-by-module stack.
"""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ops():
    from ewdml import ops
    from ewdml.ops import nn as fnn

    ops.require()
    return fnn


def _ref(h32, cb, bn, pool):
    z = h32 + cb.view(1, -1, 1, 1) if cb is not None else h32
    y = F.relu(bn(z))
    return F.max_pool2d(y, 2, 2) if pool else y


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _rel64(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("shape,pool", [((8, 64, 32, 32), True), ((8, 64, 16, 16), False),
                                        ((4, 512, 2, 2), True), ((6, 24, 6, 10), False),
                                        ((2, 2048, 4, 4), False)])
@pytest.mark.parametrize("momentum", [0.1, None])
def test_bn_relu_fp32_matches_torch(shape, pool, momentum):
    fnn = _ops()
    torch.manual_seed(0)
    dev = "cuda"
    N, C, H, W = shape
    h = (torch.randn(shape, device=dev) * 2 + 0.5).contiguous(memory_format=torch.channels_last)
    cb = torch.randn(C, device=dev) * 0.1
    bn = nn.BatchNorm2d(C, momentum=momentum).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.9, 1.1)
    bn_ref = copy.deepcopy(bn)
    hh = h.clone().requires_grad_(True)
    cbb = cb.clone().requires_grad_(True)
    y = fnn.bn_relu(hh, cbb, bn, pool)
    hr = h.clone().contiguous().requires_grad_(True)
    cbr = cb.clone().requires_grad_(True)
    yr = _ref(hr, cbr, bn_ref, pool)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, yr) < 1e-5
    assert torch.allclose(bn.running_mean, bn_ref.running_mean, atol=1e-5, rtol=1e-5)
    assert torch.allclose(bn.running_var, bn_ref.running_var, atol=1e-5, rtol=1e-5)
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked) == 1
    dy = torch.randn_like(yr)
    y.backward(dy.contiguous(memory_format=torch.channels_last))
    yr.backward(dy)
    assert _rel(hh.grad, hr.grad) < 1e-4
    assert _rel(bn.weight.grad, bn_ref.weight.grad) < 1e-4
    assert _rel(bn.bias.grad, bn_ref.bias.grad) < 1e-4
    # the conv bias cancels in batch-norm: both gradients are rounding noise around 0
    scale = float(hr.grad.abs().sum())
    assert float(cbb.grad.abs().max()) < 1e-3 * scale / C + 1e-3
    assert float(cbr.grad.abs().max()) < 1e-3 * scale / C + 1e-3


@pytest.mark.parametrize("pool", [False, True])
def test_bn_relu_bf16_close_to_fp32(pool):
    fnn = _ops()
    torch.manual_seed(1)
    dev = "cuda"
    shape = (16, 128, 16, 16)
    C = shape[1]
    h32 = torch.randn(shape, device=dev) * 3 - 1
    h = h32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(C).to(dev)
    bn_ref = copy.deepcopy(bn)
    hh = h.clone().requires_grad_(True)
    y = fnn.bn_relu(hh, None, bn, pool)
    assert y.dtype == torch.bfloat16
    hr = h.float().contiguous().requires_grad_(True)
    yr = _ref(hr, None, bn_ref, pool)
    assert _rel(y, yr) < 1e-2
    assert torch.allclose(bn.running_mean, bn_ref.running_mean, atol=1e-4, rtol=1e-4)
    assert torch.allclose(bn.running_var, bn_ref.running_var, atol=1e-4, rtol=1e-4)
    if not pool:  # pooled bf16 argmax may differ from fp32 on bf16 ties; see the next test
        dy = torch.randn_like(yr)
        y.backward(dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        yr.backward(dy.to(torch.bfloat16).float())
        assert _rel(hh.grad, hr.grad) < 2e-2
        assert _rel(bn.weight.grad, bn_ref.weight.grad) < 1e-2
        assert _rel(bn.bias.grad, bn_ref.bias.grad) < 1e-2


def test_bn_relu_pool_equals_unpooled_then_pool_bf16():
    """The fused pool is exactly max_pool2d of the fused unpooled output (same bf16 values, same
    first-max routing), and its gradient matches routing dy through torch's max-pool backward."""
    fnn = _ops()
    torch.manual_seed(2)
    dev = "cuda"
    shape = (8, 64, 8, 8)
    h = (torch.randn(shape, device=dev)).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    bn1 = nn.BatchNorm2d(64).to(dev)
    bn2 = copy.deepcopy(bn1)
    a = h.clone().requires_grad_(True)
    yp = fnn.bn_relu(a, None, bn1, True)
    b = h.clone().requires_grad_(True)
    yf = fnn.bn_relu(b, None, bn2, False)
    yfp = F.max_pool2d(yf, 2, 2)
    assert torch.equal(yp.float(), yfp.float())
    dy = torch.randn(yp.shape, device=dev).to(torch.bfloat16)
    yp.backward(dy.contiguous(memory_format=torch.channels_last))
    yfp.backward(dy.contiguous(memory_format=torch.channels_last))
    assert _rel(a.grad, b.grad) < 1e-2


def test_bn_relu_eval_mode():
    fnn = _ops()
    torch.manual_seed(3)
    dev = "cuda"
    h = torch.randn(4, 32, 8, 8, device=dev).contiguous(memory_format=torch.channels_last)
    cb = torch.randn(32, device=dev)
    bn = nn.BatchNorm2d(32).to(dev)
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-1, 1)
    bn.eval()
    for pool in (False, True):
        with torch.no_grad():
            y = fnn.bn_relu(h, cb, bn, pool)
            yr = _ref(h.contiguous(), cb, bn, pool)
        assert _rel(y, yr) < 1e-5


@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_maxpool2x2_exact(layout, dtype):
    fnn = _ops()
    torch.manual_seed(4)
    x = torch.randint(-3, 4, (4, 16, 12, 10), device="cuda").to(dtype)  # many ties
    x[0, 0, 0, 0] = float("nan")
    if layout == "nhwc":
        x = x.contiguous(memory_format=torch.channels_last)
    a = x.clone().requires_grad_(True)
    y = fnn.maxpool2x2(a)
    b = x.clone().requires_grad_(True)
    yr = F.max_pool2d(b, 2, 2)
    assert torch.equal(torch.nan_to_num(y.float(), 99.0), torch.nan_to_num(yr.float(), 99.0))
    dy = torch.randn(yr.shape, device="cuda").to(dtype)
    y.backward(dy)
    yr.backward(dy)
    assert torch.equal(a.grad.float(), b.grad.float())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hw", [(12, 10), (13, 9), (112, 112)])
def test_maxpool3x3s2_matches_torch(dtype, hw):
    """3x3 / stride 2 / pad 1 max pool (the ImageNet ResNet stem's): values and tap choice as
    F.max_pool2d (first maximum in (kh, kw) order, NaN wins; ties included), gradient gathered
    from every window whose winner is the pixel -- against PyTorch's CPU pool in float64 (its
    scatter adds the same terms; overlapping windows share a pixel)."""
    fnn = _ops()
    torch.manual_seed(5)
    H, W = hw
    N = 2 if H > 64 else 4
    x = torch.randint(-3, 4, (N, 16, H, W), device="cuda").to(dtype)  # many ties
    x[0, 0, 0, 0] = float("nan")
    x = x.contiguous(memory_format=torch.channels_last)
    a = x.clone().requires_grad_(True)
    y = fnn.maxpool3x3s2(a)
    assert y.grad_fn is not None and "MaxPool3s2" in type(y.grad_fn).__name__
    b = x.detach().cpu().double().requires_grad_(True)
    yr = F.max_pool2d(b, 3, 2, 1)
    assert torch.equal(torch.nan_to_num(y.double().cpu(), 99.0), torch.nan_to_num(yr, 99.0))
    dy = torch.randn(yr.shape).to(dtype)
    y.backward(dy.cuda().contiguous(memory_format=torch.channels_last))
    yr.backward(dy.double())
    torch.testing.assert_close(a.grad.double().cpu(), b.grad, rtol=1e-2 if dtype ==
                               torch.bfloat16 else 1e-6, atol=1e-2 if dtype == torch.bfloat16
                               else 1e-6)


def _vgg_run(model, x, y, fused_on, amp):
    from ewdml.models import fused

    fused.set_enabled(fused_on)
    torch.manual_seed(7)  # same dropout masks in every run
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = model(x)
        F.cross_entropy(out.float(), y).backward()
    finally:
        fused.set_enabled(True)
    grads = {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}
    return out.detach().float(), grads


def test_vgg11_fused_matches_modules():
    """fp32: the fused feature stack equals the module stack to fp32 rounding.  bf16 autocast: the
    fused stack is no further from the fp32 gradients than the module stack is."""
    from ewdml.models import build_model

    _ops()
    torch.manual_seed(5)
    base = build_model("vgg11", 10).cuda().to(memory_format=torch.channels_last)
    for mod in base.modules():  # dropout draws differ between fp32 and bf16 kernels
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    runs = {}
    for key in [(True, False), (False, False), (True, True), (False, True)]:
        m = copy.deepcopy(base)
        runs[key] = _vgg_run(m, x, y, *key) + (m,)
    conv_bias = {n + ".bias" for n, mod in base.named_modules() if isinstance(mod, nn.Conv2d)
                 and n.startswith("features")}
    (o_f, g_f, m_f), (o_m, g_m, m_m) = runs[(True, False)], runs[(False, False)]
    assert _rel(o_f, o_m) < 1e-4
    for n in g_m:
        if n in conv_bias:  # cancels in batch-norm: rounding noise around 0 in both
            continue
        assert _rel(g_f[n], g_m[n]) < 1e-2, n  # 8 BN backwards of fp32 rounding-order noise
    for (n, b1), (_, b2) in zip(m_f.named_buffers(), m_m.named_buffers()):
        assert torch.allclose(b1.float(), b2.float(), rtol=1e-4, atol=1e-5), n
    (ob_f, gb_f, _), (ob_m, gb_m, _) = runs[(True, True)], runs[(False, True)]
    assert _rel(ob_f, o_m) < 5e-2 and _rel(ob_m, o_m) < 5e-2
    errs = {n: (_rel(gb_f[n], g_m[n]), _rel(gb_m[n], g_m[n])) for n in g_m if n not in conv_bias}
    print("bf16 grad error vs fp32 (fused, modules):",
          {n: (round(a, 4), round(b, 4)) for n, (a, b) in errs.items()})
    err_f = sum(a for a, _ in errs.values())
    err_m = sum(b for _, b in errs.values())
    assert err_f < 1.5 * err_m + 1e-2, (err_f, err_m)


@pytest.mark.parametrize("mode", ["none", "add_relu"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_act_modes_match_torch(mode, dtype):
    fnn = _ops()
    torch.manual_seed(6)
    dev = "cuda"
    shape = (8, 256, 8, 8)
    C = shape[1]
    h = (torch.randn(shape, device=dev) * 1.5 + 0.3).to(dtype).contiguous(
        memory_format=torch.channels_last)
    r = torch.randn(shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    bn_ref = copy.deepcopy(bn)
    hh = h.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True) if mode == "add_relu" else None
    y = fnn.bn_act(hh, bn, mode, res=rr)
    hr = h.float().contiguous().requires_grad_(True)
    rrr = r.float().contiguous().requires_grad_(True) if mode == "add_relu" else None
    yr = fnn.bn_act_reference(hr, None, bn_ref, False, mode, rrr)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(y, yr) < tol
    assert torch.allclose(bn.running_mean, bn_ref.running_mean, atol=1e-4, rtol=1e-4)
    dy = torch.randn_like(yr).to(dtype)
    y.backward(dy.contiguous(memory_format=torch.channels_last))
    yr.backward(dy.float())
    gtol = 1e-4 if dtype == torch.float32 else 3e-2
    assert _rel(hh.grad, hr.grad) < gtol
    assert _rel(bn.weight.grad, bn_ref.weight.grad) < gtol
    assert _rel(bn.bias.grad, bn_ref.bias.grad) < gtol
    if mode == "add_relu":
        assert _rel(rr.grad, rrr.grad) < gtol


def test_resnet18_fused_matches_modules_fp32():
    from ewdml.models import build_model

    _ops()
    torch.manual_seed(8)
    base = build_model("resnet18", 10).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    runs = {}
    for on in (True, False):
        m = copy.deepcopy(base)
        runs[on] = _vgg_run(m, x, y, on, False) + (m,)
    (o_f, g_f, m_f), (o_m, g_m, m_m) = runs[True], runs[False]
    assert _rel(o_f, o_m) < 1e-4
    for n in g_m:  # 18 layers of fp32 rounding-order differences reach the stem
        assert _rel(g_f[n], g_m[n]) < 1e-2, n
    for (n, b1), (_, b2) in zip(m_f.named_buffers(), m_m.named_buffers()):
        assert torch.allclose(b1.float(), b2.float(), rtol=1e-4, atol=1e-5), n


@pytest.mark.parametrize("B,K,dtype", [(128, 10, torch.bfloat16), (64, 1000, torch.bfloat16),
                                       (7, 10, torch.float32), (300, 37, torch.float32)])
def test_cross_entropy_matches_torch(B, K, dtype):
    fnn = _ops()
    g = torch.Generator(device="cuda").manual_seed(B + K)
    logits = (3 * torch.randn(B, K, device="cuda", generator=g)).to(dtype)
    y = torch.randint(0, K, (B,), device="cuda", generator=g)
    a = logits.clone().requires_grad_(True)
    loss = fnn.cross_entropy(a, y)
    (2.5 * loss).backward()
    r = logits.clone().float().requires_grad_(True)
    ref = F.cross_entropy(r, y)
    (2.5 * ref).backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * max(1.0, abs(ref.item()))
    assert a.grad.dtype == dtype
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert _rel(a.grad, r.grad) < tol, _rel(a.grad, r.grad)


@pytest.mark.parametrize("B,K", [(128, 10), (64, 1000)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cross_entropy_unit_seed_grad_formed_in_forward(B, K, dtype):
    """With the trainer's all-ones loss seed registered, the forward kernel writes d(loss)/d(logits)
    and the backward launches nothing: bitwise the gradient of the backward kernel; any other
    upstream gradient still takes the backward kernel."""
    fnn = _ops()
    g = torch.Generator(device="cuda").manual_seed(B * K)
    logits = (3 * torch.randn(B, K, device="cuda", generator=g)).to(dtype)
    y = torch.randint(0, K, (B,), device="cuda", generator=g)
    seed = torch.ones((), device="cuda")
    ref = logits.clone().requires_grad_(True)
    fnn.cross_entropy(ref, y).backward(seed.clone())  # not the registered seed: kernel path
    try:
        fnn.set_unit_grad(seed)
        a = logits.clone().requires_grad_(True)
        loss = fnn.cross_entropy(a, y)
        loss.backward(seed)
        assert torch.equal(a.grad, ref.grad)
        b = logits.clone().requires_grad_(True)
        fnn.cross_entropy(b, y).backward(2 * seed)
        torch.testing.assert_close(b.grad.float(), 2 * ref.grad.float(), rtol=1e-2, atol=1e-6)
        with torch.no_grad():  # an eval forward: no backward can follow, no dx is formed
            fnn.cross_entropy(logits, y)
        seed.fill_(1.0)  # written since it was registered: no longer trusted as the unit seed
        c = logits.clone().requires_grad_(True)
        fnn.cross_entropy(c, y).backward(seed)
        assert torch.equal(c.grad, ref.grad)  # the backward kernel's (identical) bits
    finally:
        fnn.set_unit_grad(None)


def _head_model():
    from ewdml.models import build_model

    torch.manual_seed(3)
    m = build_model("vgg11", 10).cuda()
    for p in m.classifier.parameters():
        p.data = p.data.to(torch.bfloat16)
    return m.classifier


def test_vgg_head_matches_torch_without_dropout():
    from ewdml.ops import head

    _ops()
    cls = _head_model()
    for mod in cls:
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = torch.randn(128, 512, device="cuda").to(torch.bfloat16)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    assert head.supported(cls, xa)
    out = head.vgg_head(cls, xa)
    gout = torch.randn_like(out)
    out.backward(gout)
    ga = [p.grad.clone() for p in cls.parameters()]
    for p in cls.parameters():
        p.grad = None
    ref = cls(xb)
    ref.backward(gout)
    assert _rel(out, ref) < 1e-2
    assert _rel(xa.grad, xb.grad) < 2e-2
    for a, p in zip(ga, cls.parameters()):
        assert a.dtype == p.dtype
        assert _rel(a, p.grad) < 2e-2, _rel(a, p.grad)


def test_vgg_head_dropout_masks():
    from ewdml.ops import head

    fnn = _ops()
    cls = _head_model()
    x = torch.randn(128, 512, device="cuda").to(torch.bfloat16).requires_grad_(True)
    d0 = cls[0]
    z1 = head._ActDropout.apply(x, 0.5, False, head._ctr(d0, x.device))
    kept = (z1 != 0) & (x != 0)
    frac = float(kept.float().mean())
    assert 0.47 < frac < 0.53, frac
    assert torch.equal(z1[kept].float(), (2 * x[kept].float()).to(torch.bfloat16).float())
    g = torch.ones_like(z1)
    z1.backward(g)
    # backward recomputes the forward's mask: grad 2 where kept, 0 where dropped
    assert torch.equal(x.grad[kept].float(), torch.full_like(x.grad[kept].float(), 2.0))
    assert float(x.grad[~kept & (x != 0)].abs().max()) == 0.0
    z2 = head._ActDropout.apply(x.detach(), 0.5, False, head._ctr(d0, x.device))
    assert not torch.equal(z1.detach(), z2)  # the device counter advanced: a new mask
    del fnn


@pytest.mark.parametrize("rows,C,p", [(37, 24, 0.0), (300, 40, 0.3), (128, 512, 0.5),
                                      (128, 10, 0.0)])
def test_head_linear_backward_edges(rows, C, p):
    """Head Linear + ReLU + output dropout (ops/csrc/head.hip): forward and the one-launch
    backward (mask recomputed, bias gradient fused) on row counts and widths off the 32 x 32
    tiling, against the same mask applied in PyTorch fp32."""
    from ewdml.ops import head

    _ops()
    lin = nn.Linear(64, C).cuda().to(torch.bfloat16)
    x = torch.randn(rows, 64, device="cuda").to(torch.bfloat16).requires_grad_(True)
    ctr = head._ctr(lin, x.device)
    spec = (ctr, 1234, p) if p > 0 else None
    z = head.head_linear(x, lin, relu=True, dout=spec)
    y = torch.addmm(lin.bias.float(), x.detach().float(), lin.weight.float().t())
    # the forward: bf16(relu(bf16(y)) * mask)
    keep = (z.float() != 0) | (y.to(torch.bfloat16).float() <= 0)
    if p == 0.0:
        assert bool(keep.all())
    else:
        frac = float(keep[y > 0.05].float().mean())
        assert abs(frac - (1 - p)) < 0.08, frac
    scale = 1.0 / (1.0 - p)
    zr = torch.relu(y.to(torch.bfloat16).float()) * keep.float() * scale
    assert _rel(z, zr) < 1e-2
    assert int(ctr[0]) == 0
    g = torch.randn_like(z)
    z.backward(g)
    if p > 0:
        assert int(ctr[0]) == 1 and int(ctr[1:].abs().sum()) == 0  # advanced once, tickets reset
    dyr = (g.float() * (y.to(torch.bfloat16).float() > 0).float() * keep.float() * scale)
    dyr = dyr.to(torch.bfloat16).float()
    assert lin.bias.grad.dtype == torch.bfloat16
    assert torch.allclose(lin.bias.grad.float(), dyr.sum(0), rtol=1e-2, atol=1e-2)
    assert _rel(x.grad, dyr @ lin.weight.detach().float()) < 1e-2
    assert _rel(lin.weight.grad, dyr.t() @ x.detach().float()) < 1e-2


def test_head_linear_input_dropout():
    """The input dropout applied on the GEMM's operand load: with W = I the output shows the
    mask; the input gradient carries the same mask and scale."""
    from ewdml.ops import head

    _ops()
    K = 64
    lin = nn.Linear(K, K).cuda().to(torch.bfloat16)
    with torch.no_grad():
        lin.weight.copy_(torch.eye(K))
        lin.bias.zero_()
    x = torch.ones(96, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    ctr = head._ctr(nn.Dropout(), x.device)
    z = head.head_linear(x, lin, relu=False, din=(ctr, 77, 0.5))
    kept = z.float() != 0
    assert 0.4 < float(kept.float().mean()) < 0.6
    assert torch.equal(z.float()[kept], torch.full_like(z.float()[kept], 2.0))
    z.backward(torch.ones_like(z))
    assert torch.equal(x.grad.float(), kept.float() * 2.0)
    assert int(ctr[0]) == 1
    z2 = head.head_linear(x.detach(), lin, relu=False, din=(ctr, 77, 0.5))
    assert not torch.equal(z2, z.detach())  # next step: new mask


def test_vgg_head_fp32_matches_float64():
    """fp32 head kernels (eight v_mfma_f32_16x16x4_f32 per 32-deep step): forward and all
    gradients against float64 PyTorch, no dropout."""
    from ewdml.models import build_model
    from ewdml.ops import head

    _ops()
    cls = build_model("vgg11", 10).cuda().classifier
    for mod in cls:
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = torch.randn(128, 512, device="cuda")
    xa = x.clone().requires_grad_(True)
    assert head.supported(cls, xa)
    out = head.vgg_head(cls, xa)
    assert out.dtype == torch.float32 and out.grad_fn is not None
    assert "Head" in type(out.grad_fn).__name__
    gout = torch.randn_like(out)
    out.backward(gout)
    c64 = copy.deepcopy(cls).double().cpu()
    xr = x.double().cpu().requires_grad_(True)
    ref = c64(xr)
    ref.backward(gout.double().cpu())
    assert _rel64(out, ref) < 1e-5, _rel64(out, ref)
    assert _rel64(xa.grad, xr.grad) < 1e-5, _rel64(xa.grad, xr.grad)
    for p, q in zip(cls.parameters(), c64.parameters()):
        assert p.grad.dtype == torch.float32
        assert _rel64(p.grad, q.grad) < 1e-5, _rel64(p.grad, q.grad)


@pytest.mark.parametrize("rows,C,p", [(37, 24, 0.0), (300, 40, 0.3), (128, 512, 0.5)])
def test_head_linear_fp32_dropout_edges(rows, C, p):
    """fp32 head Linear + ReLU + output dropout on off-tile shapes: the forward's mask applied in
    float64 reproduces output and gradients to fp32 accuracy."""
    from ewdml.ops import head

    _ops()
    lin = nn.Linear(64, C).cuda()
    x = torch.randn(rows, 64, device="cuda").requires_grad_(True)
    ctr = head._ctr(lin, x.device)
    spec = (ctr, 4321, p) if p > 0 else None
    z = head.head_linear(x, lin, relu=True, dout=spec)
    y = torch.addmm(lin.bias.double(), x.detach().double(), lin.weight.double().t())
    keep = (z.double() != 0) | (y <= 0)
    scale = 1.0 / (1.0 - p)
    zr = torch.relu(y) * keep.double() * scale
    assert _rel64(z, zr) < 1e-5
    g = torch.randn_like(z)
    z.backward(g)
    dyr = g.double() * (y > 0).double() * keep.double() * scale
    assert torch.allclose(lin.bias.grad.double(), dyr.sum(0), rtol=1e-5, atol=1e-5)
    assert _rel64(x.grad, dyr @ lin.weight.detach().double()) < 1e-5
    assert _rel64(lin.weight.grad, dyr.t() @ x.detach().double()) < 1e-5


@pytest.mark.parametrize("shape", [(128, 2048, 4, 4), (6, 64, 7, 5), (3, 512, 1, 1)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_global_avg_pool_matches_torch(shape, dtype):
    """ResNet head pool (NHWC HIP kernels) against the fp32 torch reference, both directions."""
    fnn = _ops()
    torch.manual_seed(4)
    x = torch.randn(shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    xx = x.clone().requires_grad_(True)
    y = fnn.global_avg_pool(xx)
    xr = x.float().clone().requires_grad_(True)
    yr = F.adaptive_avg_pool2d(xr, 1).flatten(1)
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert y.shape == yr.shape and y.dtype == dtype
    assert _rel(y, yr) < tol
    dy = torch.randn(yr.shape, device="cuda")
    y.backward(dy.to(dtype))
    yr.backward(dy)
    assert xx.grad.is_contiguous(memory_format=torch.channels_last)
    assert _rel(xx.grad, xr.grad) < tol
