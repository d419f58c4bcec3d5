"""MFMA implicit-GEMM 3x3 / 1x1 convolution (ops/csrc/conv.hip) against plain PyTorch fp32.

Inputs and weights are bf16; the reference is ``F.conv2d`` / its autograd in fp32 on the same
(bf16-valued) tensors.  The kernels accumulate in fp32 and round the result to bf16 once, so the
relative error is ~bf16 resolution (2^-8).  Shapes cover every tiling path: 128x128 tiles (M*N
large), 64x64 tiles, split-K with the slab reduction (small M), H != W, and the VGG-11 layers.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _conv():
    from ewdml import ops
    from ewdml.ops import conv

    ops.require()
    conv.set_enabled(True)
    return conv


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _data(N, C, Nc, H, W, seed=0, k=3):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(Nc, C, k, k, device="cuda", generator=g) / (k * C ** 0.5)).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    w = w.contiguous(memory_format=torch.channels_last)
    return x, w


SHAPES = [
    (128, 64, 128, 16, 16),   # VGG conv2: 128x128 tiles
    (16, 128, 256, 8, 8),     # 64x64 tiles
    (128, 256, 512, 4, 4),    # VGG conv5
    (128, 512, 512, 2, 2),    # VGG conv7: split-K fwd / bwd-data
    (2, 64, 128, 8, 16),      # H != W, small
    (4, 192, 128, 4, 8),      # C not a power of two
    (512, 64, 128, 16, 16),   # one k-group per block (many tiles)
    (8, 128, 64, 8, 8),       # C_out = 64
    (8, 64, 128, 8, 5),       # odd width (row pairs cross image rows)
]
SHAPES = [s + (3,) for s in SHAPES] + [
    (16, 64, 256, 32, 32, 1),     # ResNet bottleneck 1x1 expand
    (16, 256, 64, 32, 32, 1),     # 1x1 reduce, C_out = 64
    (32, 512, 2048, 4, 4, 1),     # stage 4 expand (small M: split-K)
    (8, 128, 128, 8, 6, 1),
]


@pytest.mark.parametrize("N,C,Nc,H,W,k", SHAPES)
def test_conv_forward(N, C, Nc, H, W, k):
    conv = _conv()
    x, w = _data(N, C, Nc, H, W, k=k)
    assert conv.supported(x, w)
    y = conv.conv(x, w)
    ref = F.conv2d(x.float(), w.float(), padding=k // 2)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 6e-3, _rel(y, ref)
    # bf16 rounding of an fp32 result: every element within one bf16 ulp of the reference
    err = (y.float() - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -7 + 1e-3).all()), float(err.max())


@pytest.mark.parametrize("N,C,Nc,H,W,k", SHAPES)
def test_conv_backward(N, C, Nc, H, W, k):
    conv = _conv()
    x, w = _data(N, C, Nc, H, W, seed=1, k=k)
    g = torch.Generator(device="cuda").manual_seed(7)
    dy = torch.randn(N, Nc, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    conv.conv(xa, wa).backward(dy)
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    F.conv2d(xr, wr, padding=k // 2).backward(dy.float())
    assert xa.grad.dtype == torch.bfloat16 and wa.grad.dtype == torch.bfloat16
    assert _rel(xa.grad, xr.grad) < 6e-3, _rel(xa.grad, xr.grad)
    assert _rel(wa.grad, wr.grad) < 6e-3, _rel(wa.grad, wr.grad)


def test_conv3x3_deterministic_and_fallback():
    conv = _conv()
    x, w = _data(128, 512, 512, 2, 2, seed=3)
    a = conv.conv3x3(x, w)
    b = conv.conv3x3(x, w)
    assert torch.equal(a, b)  # split-K slabs are summed in a fixed order
    # unsupported shapes (3 input channels, fp32) take F.conv2d
    x3 = torch.randn(2, 3, 8, 8, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w3 = torch.randn(128, 3, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    assert not conv.supported(x3, w3)
    assert torch.allclose(conv.conv3x3(x3, w3).float(), F.conv2d(x3, w3, padding=1).float())


def test_vgg11_mfma_conv_matches_miopen_step():
    """One bf16 training step of VGG-11-BN through the MFMA convs and through MIOpen, both against
    the same step in fp32: the MFMA path's error must be no worse than MIOpen's (bf16 rounding
    compounds through 8 conv+BN layers, so the two bf16 paths differ from each other by about as
    much as each differs from fp32)."""
    import copy

    from ewdml.models import build_model

    conv = _conv()
    torch.manual_seed(0)
    m0 = build_model("vgg11", 10).cuda().to(memory_format=torch.channels_last)
    for mod in m0.modules():  # dropout masks would differ between the runs
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    mref, m1 = copy.deepcopy(m0), copy.deepcopy(m0)
    x = torch.randn(64, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda")
    outs = []
    for m, on, bf in ((mref, False, False), (m0, True, True), (m1, False, True)):
        conv.set_enabled(on)
        if bf:
            for p in m.parameters():
                p.data = p.data.to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last if p.dim() == 4 else torch.contiguous_format)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf):
            out = m(x.to(torch.bfloat16) if bf else x)
        F.cross_entropy(out.float(), y).backward()
        outs.append((out.float(), [p.grad.float() for p in m.parameters()]))
    conv.set_enabled(True)
    (o_ref, g_ref), (o_hip, g_hip), (o_mio, g_mio) = outs
    assert _rel(o_hip, o_ref) <= 1.5 * _rel(o_mio, o_ref) + 1e-3
    e_hip = sum(_rel(a, b) for a, b in zip(g_hip, g_ref)) / len(g_ref)
    e_mio = sum(_rel(a, b) for a, b in zip(g_mio, g_ref)) / len(g_ref)
    assert e_hip <= 1.5 * e_mio + 1e-3, (e_hip, e_mio)


def test_resnet50_mfma_conv_matches_miopen_step():
    """ResNet-50 (CIFAR) bf16 step through the MFMA 3x3/1x1 convs vs MIOpen, both against fp32."""
    import copy

    from ewdml.models import build_model

    conv = _conv()
    torch.manual_seed(0)
    m0 = build_model("resnet50", 10).cuda().to(memory_format=torch.channels_last)
    mref, m1 = copy.deepcopy(m0), copy.deepcopy(m0)
    x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    outs = []
    for m, on, bf in ((mref, False, False), (m0, True, True), (m1, False, True)):
        conv.set_enabled(on)
        if bf:
            for p in m.parameters():
                p.data = p.data.to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last if p.dim() == 4 else torch.contiguous_format)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf):
            out = m(x.to(torch.bfloat16) if bf else x)
        F.cross_entropy(out.float(), y).backward()
        outs.append((out.float(), [p.grad.float() for p in m.parameters()]))
    conv.set_enabled(True)
    (o_ref, g_ref), (o_hip, g_hip), (o_mio, g_mio) = outs
    assert _rel(o_hip, o_ref) <= 1.5 * _rel(o_mio, o_ref) + 1e-3
    e_hip = sum(_rel(a, b) for a, b in zip(g_hip, g_ref)) / len(g_ref)
    e_mio = sum(_rel(a, b) for a, b in zip(g_mio, g_ref)) / len(g_ref)
    assert e_hip <= 1.5 * e_mio + 1e-3, (e_hip, e_mio)


@pytest.mark.parametrize("N,C,Nc,H,W,k", [(128, 64, 128, 16, 16, 3), (16, 128, 256, 8, 8, 3),
                                          (128, 512, 512, 2, 2, 3), (16, 64, 256, 32, 32, 1),
                                          (128, 3, 64, 32, 32, 3)])
def test_conv_epilogue_bn_statistics(N, C, Nc, H, W, k):
    """The forward epilogue's BatchNorm partial sums (consumed by the fused BN, which then skips
    its statistics pass) give the same normalisation and running statistics as the BN kernels'
    own statistics pass over the stored output."""
    import copy

    from ewdml.ops import nn as fnn

    conv = _conv()
    x, w = _data(N, C, Nc, H, W, seed=5, k=k)
    bn0 = torch.nn.BatchNorm2d(Nc).cuda()
    bn1 = copy.deepcopy(bn0)
    h = conv.conv(x, w.clone().requires_grad_(True))
    # every launch hands its partials over (split-K ones from the slab reduction)
    assert hasattr(h, "_ew_bn_part")
    y0 = fnn.bn_act(h, bn0, "relu")
    h2 = h.detach().clone()  # same values, no partials attached
    y1 = fnn.bn_act(h2, bn1, "relu")
    assert _rel(y0, y1) < 1e-3
    assert torch.allclose(bn0.running_mean, bn1.running_mean, rtol=1e-4, atol=1e-6)
    assert torch.allclose(bn0.running_var, bn1.running_var, rtol=1e-4, atol=1e-6)
    assert int(bn0.num_batches_tracked) == int(bn1.num_batches_tracked) == 1


STEM_SHAPES = [
    (128, 64, 32, 32),   # VGG conv1 / CIFAR ResNet stem at batch 128
    (8, 128, 16, 16),    # two output-channel tiles
    (4, 64, 8, 8),       # M = 256: one weight-gradient block
    (2, 64, 16, 24),     # H != W
]


@pytest.mark.parametrize("N,Nc,H,W", STEM_SHAPES)
def test_conv_stem_forward_backward(N, Nc, H, W):
    """3-input-channel stem kernels: forward and weight gradient against fp32 PyTorch; the input
    gradient (MIOpen) when requested."""
    conv = _conv()
    x, w = _data(N, 3, Nc, H, W, seed=11)
    assert conv.stem_supported(x, w) and conv.supported(x, w)
    g = torch.Generator(device="cuda").manual_seed(12)
    dy = torch.randn(N, Nc, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = conv.conv(xa, wa)
    assert y.grad_fn is not None and "Stem" in type(y.grad_fn).__name__
    y.backward(dy)
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    ref = F.conv2d(xr, wr, padding=1)
    ref.backward(dy.float())
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    err = (y.float() - ref.detach()).abs()
    assert bool((err <= ref.detach().abs() * 2 ** -7 + 1e-3).all()), float(err.max())
    assert wa.grad.dtype == torch.bfloat16
    assert _rel(wa.grad, wr.grad) < 6e-3, _rel(wa.grad, wr.grad)
    assert _rel(xa.grad, xr.grad) < 1e-2, _rel(xa.grad, xr.grad)
    # the network-input case: no input gradient, weight gradient only
    wb = w.clone().requires_grad_(True)
    conv.conv(x, wb).backward(dy)
    assert torch.equal(wb.grad, wa.grad)  # fixed-order partial reduction: deterministic


@pytest.mark.parametrize("mode,pool", [("relu", True), ("relu", False), ("none", False)])
@pytest.mark.parametrize("N,HW", [(64, 16), (32, 4)])
def test_bn_backward_sums_in_bwd_data_epilogue(mode, pool, N, HW):
    """conv -> BN(+ReLU)(+pool) -> conv: the second conv's backward-data epilogue (or, for the
    small maps, its split-K slab reduction) sums the BN's backward statistics (the BN skips its
    own pass); every gradient matches the unfused path."""
    import copy

    from ewdml.ops import nn as fnn

    conv = _conv()
    # 64 x 16 x 16: the second conv's backward-data has >= 128 output tiles (epilogue sums);
    # 32 x 4 x 4: a split-K launch (sums in the slab reduction)
    x0, w0 = _data(N, 64, 128, HW, HW, seed=21)
    _, w1 = _data(8, 128, 64, 8, 8, seed=22)
    bn0 = torch.nn.BatchNorm2d(128).cuda()
    with torch.no_grad():
        bn0.weight.uniform_(0.5, 1.5)
        bn0.bias.uniform_(-0.3, 0.3)
    g = None
    grads = []
    for fused in (True, False):
        conv.set_bn_bwd_fusion(fused)
        used = fnn.PRE_BWD_USED
        bn = copy.deepcopy(bn0)
        xa, wa, wb = (t.clone().requires_grad_(True) for t in (x0, w0, w1))
        h = conv.conv(xa, wa)
        y = fnn.bn_act(h, bn, mode, pool=pool)
        z = conv.conv(y, wb)
        if g is None:
            g = torch.randn(z.shape, device="cuda").to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
        z.backward(g)
        assert (fnn.PRE_BWD_USED > used) == fused
        grads.append([xa.grad, wa.grad, wb.grad, bn.weight.grad, bn.bias.grad])
    conv.set_bn_bwd_fusion(True)
    for a, b in zip(*grads):
        assert _rel(a, b) < 2e-3, _rel(a, b)


@pytest.mark.parametrize("net", ["resnet18", "resnet50"])
def test_resnet_residual_grad_sink_and_bn_sums_match_autograd_sum(net):
    """Identity-residual gradients handed to the block's first conv (added in its backward-data
    epilogue) and BN backward sums from the epilogues: one bf16 ResNet step is as close to the
    fp32 step as the bf16 step with autograd summing the residual gradients and the BN kernels'
    own statistics passes."""
    import copy

    from ewdml.models import build_model, resnet
    from ewdml.ops import nn as fnn

    conv = _conv()
    torch.manual_seed(0)
    m0 = build_model(net, 10).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    res = []
    for run in ("fp32", "fused", "unfused"):
        fused = run == "fused"
        resnet.set_residual_sink(fused)
        conv.set_bn_bwd_fusion(fused)
        m = copy.deepcopy(m0)
        xx = x
        conv.set_enabled(run != "fp32")  # fp32 reference: MIOpen, not the fp32 MFMA kernels
        if run != "fp32":
            for p in m.parameters():
                p.data = p.data.to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last if p.dim() == 4 else torch.contiguous_format)
            xx = x.to(torch.bfloat16)
        used = fnn.PRE_BWD_USED
        try:
            out = m(xx)
            torch.nn.functional.cross_entropy(out.float(), y).backward()
        finally:
            resnet.set_residual_sink(True)
            conv.set_bn_bwd_fusion(True)
            conv.set_enabled(True)
        if fused:
            assert fnn.PRE_BWD_USED > used
        res.append((out.float(), [p.grad.float() for p in m.parameters()]))
    (o_ref, g_ref), (o_f, g_f), (o_u, g_u) = res
    assert _rel(o_f, o_ref) <= 1.25 * _rel(o_u, o_ref) + 1e-3
    e_f = sum(_rel(a, b) for a, b in zip(g_f, g_ref)) / len(g_ref)
    e_u = sum(_rel(a, b) for a, b in zip(g_u, g_ref)) / len(g_ref)
    assert e_f <= 1.25 * e_u + 1e-3, (e_f, e_u)
