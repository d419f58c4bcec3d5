"""fp32 MFMA implicit-GEMM convolutions (ops/csrc/conv_f32.hip, v_mfma_f32_16x16x4_f32) and the
Winograd F(2x2, 3x3) path (ops/csrc/winograd_f32.hip) against a float64 PyTorch reference on the
CPU.

The kernels multiply and accumulate in fp32 with no reduced-precision operand step, so the
relative error is a few fp32 ulps times the reduction length's growth: the bound used is 1e-5
(bf16 would be ~4e-3, xf32/tf32 ~5e-4).  Shapes cover every tiling path: 128x128, 128x64, 64x128
and 64x64 tiles, split-K slab reductions, H != W, odd widths, 1x1 and the 3-channel stem.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _conv(wino=False, min_c=64, tile="auto", sm=False):
    """The conv module with the Winograd path off (direct implicit GEMM for every shape) or on
    for every layer with at least ``min_c`` channels, tile m = 2, 4 or auto; ``sm``: the 2x2-map
    dense position GEMMs (ops/csrc/smallmap_f32.hip) for the layers they take."""
    from ewdml import ops
    from ewdml.ops import conv

    ops.require()
    conv.set_enabled(True)
    conv.set_winograd(wino, min_c, tile)
    conv.set_smallmap(sm)
    return conv


@pytest.fixture(autouse=True)
def _restore_winograd():
    from ewdml.ops import conv

    saved = (conv._WINO, conv._WINO_MIN_C, conv._WINO_TILE)
    s2, sm = conv._S2, conv._SMALLMAP
    yield
    conv.set_winograd(*saved)
    conv.set_stride2(s2)
    conv.set_smallmap(sm)


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _data(N, C, Nc, H, W, seed=0, k=3):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(N, C, H, W, device="cuda", generator=g)
    w = torch.randn(Nc, C, k, k, device="cuda", generator=g) / (k * C ** 0.5)
    return (x.contiguous(memory_format=torch.channels_last),
            w.contiguous(memory_format=torch.channels_last))


def _ref64(x, w, k, dy=None):
    """float64 CPU forward (and grads for dy)."""
    xr = x.detach().double().cpu().requires_grad_(dy is not None)
    wr = w.detach().double().cpu().requires_grad_(dy is not None)
    y = F.conv2d(xr, wr, padding=k // 2)
    if dy is not None:
        y.backward(dy.detach().double().cpu())
        return y.detach(), xr.grad, wr.grad
    return y.detach()


SHAPES = [
    (128, 64, 128, 16, 16, 3),   # VGG conv2: 128x128 tiles, no split
    (128, 128, 256, 8, 8, 3),    # VGG conv3: 128x128, split 2
    (64, 256, 512, 4, 4, 3),     # 128x128 split-K
    (128, 512, 512, 2, 2, 3),    # VGG conv7: 64x64 split-K
    (2, 64, 128, 8, 16, 3),      # H != W, small
    (4, 192, 128, 4, 8, 3),      # C not a power of two
    (8, 128, 64, 8, 8, 3),       # C_out = 64
    (8, 64, 128, 8, 5, 3),       # odd width
    (16, 64, 256, 32, 32, 1),    # 1x1 expand
    (16, 256, 64, 32, 32, 1),    # 1x1 reduce
    (32, 512, 2048, 4, 4, 1),    # 1x1, small M
    (32, 256, 64, 32, 32, 1),    # ResNet layer-1 1x1 reduce: 64x256 weight-gradient tile, split-K
]


@pytest.mark.parametrize("N,C,Nc,H,W,k", SHAPES)
def test_conv_f32_forward(N, C, Nc, H, W, k):
    conv = _conv()
    x, w = _data(N, C, Nc, H, W, k=k)
    assert conv.supported(x, w)
    y = conv.conv(x, w)
    assert y.grad_fn is None or "Conv" in type(y.grad_fn).__name__
    assert y.dtype == torch.float32 and y.is_contiguous(memory_format=torch.channels_last)
    ref = _ref64(x, w, k)
    assert _rel(y, ref) < TOL, _rel(y, ref)


@pytest.mark.parametrize("N,C,Nc,H,W,k", SHAPES)
def test_conv_f32_forward_lds_dma_staging(N, C, Nc, H, W, k):
    """The forward GEMM with LDS-DMA operand staging (buffer_load ... lds, swizzle on the source
    address, three stage images) writes bitwise what the register-staged kernel writes: the same
    LDS images, the same MFMA order; padding taps read zeros through out-of-range offsets."""
    from ewdml import ops

    conv = _conv()
    C_ = ops.require()
    x, w = _data(N, C, Nc, H, W, seed=3, k=k)
    prev = C_.cf_set_glds(0)
    try:
        y0 = conv.conv(x, w)
        C_.cf_set_glds(1)
        y1 = conv.conv(x, w)
        torch.cuda.synchronize()
    finally:
        C_.cf_set_glds(prev)
    torch.testing.assert_close(y1, y0, rtol=0, atol=0)
    assert _rel(y1, _ref64(x, w, k)) < TOL


@pytest.mark.parametrize("N,C,Nc,H,W,k", SHAPES)
def test_conv_f32_backward(N, C, Nc, H, W, k):
    conv = _conv()
    x, w = _data(N, C, Nc, H, W, seed=1, k=k)
    g = torch.Generator(device="cuda").manual_seed(7)
    dy = torch.randn(N, Nc, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = conv.conv(xa, wa)
    assert "Conv" in type(y.grad_fn).__name__  # the HIP autograd function, not MIOpen
    y.backward(dy)
    _, gx, gw = _ref64(x, w, k, dy)
    assert xa.grad.dtype == torch.float32 and wa.grad.dtype == torch.float32
    assert _rel(xa.grad, gx) < TOL, _rel(xa.grad, gx)
    assert _rel(wa.grad, gw) < TOL, _rel(wa.grad, gw)


@pytest.mark.parametrize("N,C,Nc,H,W,k", [(128, 64, 128, 16, 16, 3), (32, 256, 64, 32, 32, 1),
                                          (64, 256, 512, 4, 4, 3), (128, 512, 512, 2, 2, 3)])
def test_conv_f32_inlaunch_split_reduction_bitwise(N, C, Nc, H, W, k):
    """Split-K GEMMs reduced by each tile's last split inside the launch (k_cf_gemm epilogue,
    write-through slabs + ticket) give bitwise what the separate k_cf_slab_reduce launch gives:
    forward, backward data and weight gradient."""
    from ewdml import ops

    conv = _conv()
    C_ = ops.require()
    x, w = _data(N, C, Nc, H, W, seed=9, k=k)
    dy = torch.randn(N, Nc, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    res = []
    prev = C_.cf_set_inred(1)
    try:
        for on in (1, 0):
            C_.cf_set_inred(on)
            xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
            y = conv.conv(xa, wa)
            y.backward(dy)
            torch.cuda.synchronize()
            res.append((y.detach(), xa.grad, wa.grad))
    finally:
        C_.cf_set_inred(prev)
    for a, b in zip(*res):
        assert torch.equal(a, b)
    assert _rel(res[0][2], _ref64(x, w, k, dy)[2]) < TOL


def test_conv_f32_deterministic():
    conv = _conv()
    x, w = _data(128, 512, 512, 2, 2, seed=3)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    a = conv.conv(xa, wa)
    b = conv.conv(x, w)
    assert torch.equal(a, b)  # split-K slabs are summed in a fixed order
    dy = torch.randn_like(a)
    a.backward(dy)
    g1 = (xa.grad.clone(), wa.grad.clone())
    xa.grad = wa.grad = None
    conv.conv(xa, wa).backward(dy)
    assert torch.equal(g1[0], xa.grad) and torch.equal(g1[1], wa.grad)


@pytest.mark.parametrize("N,Nc,H,W", [(128, 64, 32, 32), (8, 128, 16, 16), (4, 64, 8, 8),
                                      (2, 64, 16, 24)])
def test_conv_f32_stem(N, Nc, H, W):
    conv = _conv()
    x, w = _data(N, 3, Nc, H, W, seed=11)
    assert conv.stem_supported(x, w)
    g = torch.Generator(device="cuda").manual_seed(12)
    dy = torch.randn(N, Nc, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    wa = w.clone().requires_grad_(True)
    y = conv.conv(x, wa)
    assert "Stem" in type(y.grad_fn).__name__
    y.backward(dy)
    ref, _, gw = _ref64(x, w, 3, dy)
    assert y.dtype == torch.float32
    assert _rel(y, ref) < TOL, _rel(y, ref)
    assert _rel(wa.grad, gw) < TOL, _rel(wa.grad, gw)
    wb = w.clone().requires_grad_(True)
    conv.conv(x, wb).backward(dy)
    assert torch.equal(wb.grad, wa.grad)


@pytest.mark.parametrize("N,C,Nc,H,W,k", [(128, 64, 128, 16, 16, 3), (16, 128, 256, 8, 8, 3),
                                          (128, 512, 512, 2, 2, 3), (16, 64, 256, 32, 32, 1),
                                          (128, 3, 64, 32, 32, 3)])
def test_conv_f32_epilogue_bn_statistics(N, C, Nc, H, W, k):
    """BatchNorm partial sums from the fp32 epilogue / slab reduction give the BN kernels' own
    statistics."""
    from ewdml.ops import nn as fnn

    conv = _conv()
    x, w = _data(N, C, Nc, H, W, seed=5, k=k)
    bn0 = torch.nn.BatchNorm2d(Nc).cuda()
    bn1 = copy.deepcopy(bn0)
    h = conv.conv(x, w.clone().requires_grad_(True))
    assert hasattr(h, "_ew_bn_part")
    y0 = fnn.bn_act(h, bn0, "relu")
    y1 = fnn.bn_act(h.detach().clone(), bn1, "relu")
    assert _rel(y0, y1) < 1e-5
    assert torch.allclose(bn0.running_mean, bn1.running_mean, rtol=1e-5, atol=1e-7)
    assert torch.allclose(bn0.running_var, bn1.running_var, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("mode,pool", [("relu", True), ("relu", False), ("none", False)])
@pytest.mark.parametrize("N,HW", [(64, 16), (32, 4)])
def test_conv_f32_bn_backward_sums_in_bwd_data_epilogue(mode, pool, N, HW):
    from ewdml.ops import nn as fnn

    conv = _conv()
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
            g = torch.randn(z.shape, device="cuda").contiguous(memory_format=torch.channels_last)
        z.backward(g)
        assert (fnn.PRE_BWD_USED > used) == fused
        grads.append([xa.grad, wa.grad, wb.grad, bn.weight.grad, bn.bias.grad])
    conv.set_bn_bwd_fusion(True)
    for a, b in zip(*grads):
        assert _rel(a, b) < 1e-5, _rel(a, b)


S2_SHAPES = [  # (N, C, Nc, H, W, k): stride 2, H x W the input map
    (128, 128, 128, 32, 32, 3),   # ResNet-50 CIFAR layer2.0 conv2
    (128, 256, 256, 16, 16, 3),   # layer3.0 conv2
    (128, 512, 512, 8, 8, 3),     # layer4.0 conv2: split-K forward / weight gradient
    (128, 256, 512, 32, 32, 1),   # layer2.0 shortcut
    (128, 1024, 2048, 8, 8, 1),   # layer4.0 shortcut
    (4, 64, 128, 16, 32, 3),      # H != W, small
    (16, 64, 64, 8, 8, 1),        # 1x1, small
]


@pytest.mark.parametrize("N,C,Nc,H,W,k", S2_SHAPES)
def test_conv_f32_stride2(N, C, Nc, H, W, k):
    """Stride-2 3x3 / 1x1 kernels (phase-split backward data) against float64, through
    ``conv2d_module`` as the ResNets call them."""
    conv = _conv()
    conv.set_stride2(True)
    x, w = _data(N, C, Nc, H, W, seed=31, k=k)
    m = torch.nn.Conv2d(C, Nc, k, 2, k // 2, bias=False).cuda()
    with torch.no_grad():
        m.weight.copy_(w)
    m = m.to(memory_format=torch.channels_last)
    assert conv.s2_supported(x, m.weight, m.stride, m.padding, m.dilation, m.groups)
    g = torch.Generator(device="cuda").manual_seed(32)
    dy = torch.randn(N, Nc, H // 2, W // 2, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    xa = x.clone().requires_grad_(True)
    y = conv.conv2d_module(m, xa)
    assert "ConvS2" in type(y.grad_fn).__name__  # the HIP kernels, not MIOpen
    assert y.shape == (N, Nc, H // 2, W // 2)
    assert hasattr(y, "_ew_bn_part")
    y.backward(dy)
    xr = x.detach().double().cpu().requires_grad_(True)
    wr = w.detach().double().cpu().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=2, padding=k // 2)
    yr.backward(dy.detach().double().cpu())
    assert _rel(y, yr) < TOL, _rel(y, yr)
    assert _rel(xa.grad, xr.grad) < TOL, _rel(xa.grad, xr.grad)
    assert _rel(m.weight.grad, wr.grad) < TOL, _rel(m.weight.grad, wr.grad)
    # deterministic (fixed-order split sums) and BN partials consistent with the BN kernels
    xb = x.clone().requires_grad_(True)
    gw = m.weight.grad.clone()
    m.weight.grad = None
    y2 = conv.conv2d_module(m, xb)
    y2.backward(dy)
    assert torch.equal(y, y2) and torch.equal(xa.grad, xb.grad) and torch.equal(gw, m.weight.grad)


def test_conv_f32_stride2_bn_partials():
    from ewdml.ops import nn as fnn

    conv = _conv()
    x, w = _data(64, 128, 256, 16, 16, seed=33)
    bn0 = torch.nn.BatchNorm2d(256).cuda()
    bn1 = copy.deepcopy(bn0)
    h = conv.conv_s2(x, w.clone().requires_grad_(True))
    assert hasattr(h, "_ew_bn_part")
    y0 = fnn.bn_act(h, bn0, "relu")
    y1 = fnn.bn_act(h.detach().clone(), bn1, "relu")
    assert _rel(y0, y1) < 1e-5
    assert torch.allclose(bn0.running_var, bn1.running_var, rtol=1e-5, atol=1e-7)


WINO_SHAPES = [  # (N, C, Nc, H, W, m)
    (128, 128, 256, 8, 8, 2),    # VGG conv3
    (128, 256, 256, 8, 8, 2),    # VGG conv4
    (128, 512, 512, 4, 4, 2),    # VGG conv6
    (128, 512, 512, 2, 2, 2),    # VGG conv8: one tile per image, mostly padding
    (8, 64, 128, 16, 16, 2),     # 64 input channels
    (2, 128, 64, 8, 16, 2),      # H != W, 64 output channels
    (16, 1024, 128, 4, 4, 2),    # wide input
    (128, 128, 256, 8, 8, 4),    # F(4x4, 3x3): VGG conv3
    (128, 256, 256, 8, 8, 4),    # VGG conv4
    (128, 256, 512, 4, 4, 4),    # VGG conv5: one tile per image
    (256, 512, 512, 4, 4, 4),    # VGG conv6
    (8, 64, 128, 16, 16, 4),
    (4, 128, 64, 8, 32, 4),      # H != W, 64 output channels
]
# relative error bound vs float64 by tile: m = 4's transforms (coefficients up to 8 and 1/24)
# cost ~10x the rounding of m = 2 (tools/probes/conv_f32_probe.py --err; still ~100x below tf32)
WINO_TOL = {2: TOL, 4: 2e-5}


@pytest.mark.parametrize("N,C,Nc,H,W,m", WINO_SHAPES)
def test_conv_f32_winograd_forward_backward(N, C, Nc, H, W, m):
    conv = _conv(wino=True, tile=m)
    x, w = _data(N, C, Nc, H, W, seed=31)
    assert conv.supported(x, w) and conv.wino_tile(x, w) == m
    TOL = WINO_TOL[m]
    g = torch.Generator(device="cuda").manual_seed(32)
    dy = torch.randn(N, Nc, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = conv.conv(xa, wa)
    y.backward(dy)
    ref, gx, gw = _ref64(x, w, 3, dy)
    assert y.dtype == torch.float32 and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < TOL, _rel(y, ref)
    assert _rel(xa.grad, gx) < TOL, _rel(xa.grad, gx)
    assert _rel(wa.grad, gw) < TOL, _rel(wa.grad, gw)
    # bit-for-bit repeatable (fixed-order transforms and split sums)
    xb, wb = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y2 = conv.conv(xb, wb)
    y2.backward(dy)
    assert torch.equal(y, y2) and torch.equal(xa.grad, xb.grad) and torch.equal(wa.grad, wb.grad)
    # and close to the direct kernels (both within rounding of float64)
    d = _conv(wino=False)
    assert not d.wino_ok(x, w)
    assert _rel(d.conv(x, w), y) < 2 * TOL


def test_conv_f32_winograd_tile_choice():
    conv = _conv(wino=True, min_c=128, tile="auto")
    x, w = _data(128, 256, 256, 8, 8)
    assert conv.wino_tile(x, w) == 4
    x, w = _data(128, 512, 512, 2, 2)
    assert conv.wino_tile(x, w) == 2  # a 2x2 map does not tile by 4
    x, w = _data(16, 1024, 128, 4, 4)
    assert conv.wino_tile(x, w) == 2  # F(4x4) output kernel takes C_out <= 512; tiles % 64
    conv.set_winograd(True, 128, 2)
    x, w = _data(128, 256, 256, 8, 8)
    assert conv.wino_tile(x, w) == 2
    conv.set_winograd(True, 128, "size")  # m = 4 only with >= 2048 output tiles
    assert conv.wino_tile(x, w) == 2  # 128 x 2 x 2 = 512 tiles
    x, w = _data(128, 128, 128, 16, 16)
    assert conv.wino_tile(x, w) == 4  # 128 x 4 x 4 = 2048 tiles


def test_conv_f32_winograd_only_where_chosen():
    conv = _conv(wino=True, min_c=128)
    x, w = _data(8, 64, 128, 16, 16)
    assert not conv.wino_ok(x, w)  # 64 input channels < min_c
    x, w = _data(8, 128, 128, 16, 16)
    assert conv.wino_ok(x, w)
    x, w = _data(8, 128, 128, 16, 16, k=1)
    assert not conv.wino_ok(x, w)  # 1x1
    x, w = _data(8, 128, 128, 8, 5)
    assert not conv.wino_ok(x, w)  # odd width
    x, w = _data(8, 192, 128, 8, 8)
    assert not conv.wino_ok(x, w)  # C not a power of two


@pytest.mark.parametrize("N,C,Nc,H,W,m", [(16, 128, 256, 8, 8, 2), (128, 512, 512, 2, 2, 2),
                                          (32, 256, 512, 4, 4, 2), (64, 128, 256, 8, 8, 4),
                                          (128, 256, 512, 4, 4, 4)])
def test_conv_f32_winograd_bn_statistics(N, C, Nc, H, W, m):
    """BatchNorm partial sums from the Winograd output transform give the BN kernels' own
    statistics."""
    from ewdml.ops import nn as fnn

    conv = _conv(wino=True, tile=m)
    x, w = _data(N, C, Nc, H, W, seed=35)
    assert conv.wino_tile(x, w) == m
    bn0 = torch.nn.BatchNorm2d(Nc).cuda()
    bn1 = copy.deepcopy(bn0)
    h = conv.conv(x, w.clone().requires_grad_(True))
    assert hasattr(h, "_ew_bn_part")
    y0 = fnn.bn_act(h, bn0, "relu")
    y1 = fnn.bn_act(h.detach().clone(), bn1, "relu")
    assert _rel(y0, y1) < 1e-5
    assert torch.allclose(bn0.running_mean, bn1.running_mean, rtol=1e-5, atol=1e-7)
    assert torch.allclose(bn0.running_var, bn1.running_var, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("m", [2, 4])
@pytest.mark.parametrize("mode,pool", [("relu", True), ("relu", False), ("none", False)])
def test_conv_f32_winograd_bn_backward_sums(mode, pool, m):
    """The Winograd backward-data output transform produces the producing BN layer's backward
    sums (and the BN backward then skips its statistics pass): same gradients as unfused."""
    from ewdml.ops import nn as fnn

    conv = _conv(wino=True, tile=m)
    N, HW = 32, 16
    x0, w0 = _data(N, 128, 128, HW, HW, seed=41)
    _, w1 = _data(8, 128, 128, 8, 8, seed=42)
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
        assert conv.wino_ok(y, wb)
        z = conv.conv(y, wb)
        if g is None:
            g = torch.randn(z.shape, device="cuda").contiguous(memory_format=torch.channels_last)
        z.backward(g)
        assert (fnn.PRE_BWD_USED > used) == fused
        grads.append([xa.grad, wa.grad, wb.grad, bn.weight.grad, bn.bias.grad])
    conv.set_bn_bwd_fusion(True)
    for a, b in zip(*grads):
        assert _rel(a, b) < 1e-5, _rel(a, b)


@pytest.mark.parametrize("wino,m,k,C", [(True, 2, 3, 128), (True, 4, 3, 128), (False, 2, 3, 64),
                                        (False, 2, 1, 512)])
@pytest.mark.parametrize("mode,pool", [("relu", True), ("relu", False)])
def test_bn_finalize_rides_in_wgrad_launch(wino, m, k, C, mode, pool):
    """The BN backward finalisation riding in the next conv's weight-gradient GEMM launch (extra
    blocks, ops/csrc/bn_fin.h) gives bitwise the gradients of its own launch, Winograd and direct
    convs, with the lazy BN backward (coef read by the first conv's input transform) and without."""
    from ewdml.ops import conv as cmod
    from ewdml.ops import nn as fnn

    _conv(wino=wino, tile=m)
    N, HW = 32, 16
    x0, w0 = _data(N, C, C, HW, HW, seed=51, k=k)
    _, w1 = _data(8, C, C, 8, 8, seed=52, k=k)
    bn0 = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn0.weight.uniform_(0.5, 1.5)
        bn0.bias.uniform_(-0.3, 0.3)
    g = None
    grads = []
    saved = cmod._FIN_RIDE
    try:
        for ride in (True, False):
            cmod._FIN_RIDE = ride
            rides = cmod.FIN_RIDES
            bn = copy.deepcopy(bn0)
            xa, wa, wb = (t.clone().requires_grad_(True) for t in (x0, w0, w1))
            y = fnn.bn_act(cmod.conv(xa, wa), bn, mode, pool=pool)
            z = cmod.conv(y, wb)
            if g is None:
                g = torch.randn(z.shape, device="cuda").contiguous(
                    memory_format=torch.channels_last)
            z.backward(g)
            assert (cmod.FIN_RIDES > rides) == ride
            grads.append([xa.grad, wa.grad, wb.grad, bn.weight.grad, bn.bias.grad])
    finally:
        cmod._FIN_RIDE = saved
    for a, b in zip(*grads):
        assert torch.equal(a, b), _rel(a, b)


def test_fp32_vgg11_step_vs_fp64():
    """One fp32 VGG-11-BN training step (fused NHWC path, fp32 MFMA convs, lazy BN through the
    Winograd convs) against the same step in float64 on the CPU, and no worse than the step
    through MIOpen's fp32 convolutions.  The conv biases that feed a BatchNorm are left out: their
    exact gradient is 0 (BN removes them), so any fp32 value is pure rounding noise."""
    from ewdml.models import build_model

    conv = _conv(wino=True, min_c=128, tile=2, sm=True)  # the production choice
    torch.manual_seed(0)
    m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last)
    for mod in m0.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    # batch 32 (the 2x2-map layers run Winograd here; the small-map GEMMs need N % 64 == 0:
    # test_fp32_vgg11_convs_in_situ).  At larger batches a single fp32-vs-fp64 flip of a near-tie
    # in a BN-ReLU-max-pool window re-routes one gradient element and moves every earlier
    # layer's gradient by ~1e-3, MIOpen's path included (tools/probes/vgg_bn6_debug.py: batch
    # 128 -> 3e-3 on the HIP path, 6e-3 on MIOpen's), so whole-network gradients are no oracle
    x = torch.randn(32, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,))
    m64 = copy.deepcopy(m0).double()
    out64 = m64(x.double())
    F.cross_entropy(out64, y).backward()
    g64 = [p.grad for p in m64.parameters()]
    res = []
    for on in (True, False):
        m = copy.deepcopy(m0).cuda()
        conv.set_enabled(on)
        try:
            out = m(x.cuda())
            F.cross_entropy(out, y.cuda()).backward()
        finally:
            conv.set_enabled(True)
        feat = dict(m.features.named_children())
        zero = {f"features.{k}.bias" for k, v in feat.items()
                if isinstance(v, torch.nn.Conv2d) and isinstance(feat.get(str(int(k) + 1)),
                                                                 torch.nn.BatchNorm2d)}
        big = [(p.grad, r, n) for (n, p), r in zip(m.named_parameters(), g64)
               if float(r.norm()) > 1e-6 and n not in zero]
        worst = max(big, key=lambda t: _rel(t[0], t[1]))
        res.append((_rel(out, out64), _rel(worst[0], worst[1]), worst[2]))
    (o_h, e_h, n_h), (o_m, e_m, n_m) = res
    assert o_h < 1e-5 and e_h < 1e-4, (o_h, e_h, n_h, e_m, n_m)
    assert o_h <= 2 * o_m + 1e-6 and e_h <= 2 * e_m + 1e-5, (o_h, o_m, e_h, e_m)


def test_vgg11_step_with_deferred_reduction_bitwise():
    """Two fp32 VGG-11 training steps (production path) with conv2's split-K weight-gradient
    reduction left to the stem's reduction launch (ops/csrc/conv_f32.hip k_cf_reduce2) and with
    its own launch (EWDML_BN_FIN_RIDE off for it): bitwise the same weights and losses."""
    from ewdml.models import build_model
    from ewdml.ops import conv as cmod

    _conv(wino=True, min_c=128, tile=2, sm=True)
    torch.manual_seed(0)
    m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last).cuda()
    for mod in m0.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    x = torch.randn(128, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (128,), device="cuda")
    runs = []
    saved = cmod._FIN_RIDE
    try:
        for ride in (True, False):
            cmod._FIN_RIDE = ride
            m = copy.deepcopy(m0)
            hs = _opt_in(list(m.parameters()))  # the engine's hooks: deferral allowed
            opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
            losses = []
            defers = cmod.STEM_RED_DEFERS
            for _ in range(2):
                opt.zero_grad()
                cmod.new_pass()
                loss = F.cross_entropy(m(x), y)
                loss.backward()  # (a pending reduction is run by the end-of-backward callback)
                assert not cmod._STEM_RED[0]
                opt.step()
                losses.append(float(loss.detach()))
            assert (cmod.STEM_RED_DEFERS > defers) == ride
            _opt_out(list(m.parameters()), hs)
            runs.append((m, losses))
    finally:
        cmod._FIN_RIDE = saved
    (ma, la), (mb, lb) = runs
    assert la == lb
    for (k, a), b in zip(ma.state_dict().items(), mb.state_dict().values()):
        assert torch.equal(a, b), k


def test_vgg11_flat_view_grads_never_defer_reduction():
    """With the gradients pre-attached as views of one flat buffer (FlatModel(attach_grads=True),
    the PS / sharded topologies) AccumulateGrad adds dw into .grad as soon as the conv's backward
    returns it, so conv2's split-K reduction must not be left for the stem's launch: the
    gradients (NaN-poisoned dw) are bitwise those of the run without any rider."""
    from ewdml.models import build_model
    from ewdml.ops import conv as cmod
    from ewdml.parallel.flat import FlatModel

    _conv(wino=True, min_c=128, tile=2, sm=True)
    torch.manual_seed(0)
    m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last).cuda()
    for mod in m0.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    x = torch.randn(128, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (128,), device="cuda")
    grads = []
    saved = cmod._FIN_RIDE
    try:
        for ride in (True, False):
            cmod._FIN_RIDE = ride
            cmod._POISON_DW = True
            m = copy.deepcopy(m0)
            params = list(m.parameters())
            flat = FlatModel(params, attach_grads=True)
            hs = _opt_in(params)
            flat.zero_grad()
            cmod.new_pass()
            defers = cmod.STEM_RED_DEFERS
            F.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            assert cmod.STEM_RED_DEFERS == defers  # .grad was not None: no deferral
            _opt_out(params, hs)
            grads.append(flat.grad.clone())
    finally:
        cmod._FIN_RIDE = saved
        cmod._POISON_DW = False
    assert not torch.isnan(grads[0]).any()
    assert torch.equal(grads[0], grads[1])


def test_fp32_vgg11_convs_in_situ():
    """Every MFMA conv backward of one fp32 VGG-11 step at batch 64 (the production path: lazy BN,
    Winograd conv3-6, small-map GEMMs for the 2x2 conv7 / conv8) against float64 on the tensors it
    actually received."""
    from ewdml.models import build_model
    from ewdml.ops import conv as cmod

    _conv(wino=True, min_c=128, tile=2, sm=True)
    recs = []
    orig = cmod._Conv.backward
    defer, cmod._DEFER_WOUT = cmod._DEFER_WOUT, False

    def bwd(ctx, dy):
        from ewdml.ops.nn import materialize

        materialize(dy)
        x, w = ctx.saved_tensors
        materialize(x)
        sm = ctx.sm is not None
        dx, dw, a, b = orig(ctx, dy)
        recs.append((sm, x.detach().clone(), w.detach().clone(), dy.detach().clone(),
                     None if dx is None else dx.detach().clone(), dw.detach().clone()))
        return dx, dw, a, b

    cmod._Conv.backward = staticmethod(bwd)
    try:
        torch.manual_seed(0)
        m = build_model("vgg11", 10).to(memory_format=torch.channels_last).cuda()
        x = torch.randn(64, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (64,), device="cuda")
        F.cross_entropy(m(x), y).backward()
    finally:
        cmod._Conv.backward = orig
        cmod._DEFER_WOUT = defer
    assert sum(r[0] for r in recs) == 2  # conv7 and conv8 took the small-map GEMMs
    for sm, x, w, dy, dx, dw in recs:
        _, gx, gw = _ref64(x, w, 3, dy)
        assert _rel(dw, gw) < TOL, (sm, tuple(x.shape), _rel(dw, gw))
        if dx is not None:
            assert _rel(dx, gx) < TOL, (sm, tuple(x.shape), _rel(dx, gx))


def test_fp32_resnet18_step_convs_in_situ():
    """Every MFMA conv backward of one fp32 ResNet-18 step (BN-backward sums and residual sinks
    on) against float64 on the tensors it actually received.  (The whole-network gradient is not
    a usable oracle here: the BN bias gradients are sums with ~1e4x cancellation, so any two fp32
    runs -- MIOpen against itself included -- differ by up to ~1e-3 after a few blocks.)"""
    from ewdml.models import build_model
    from ewdml.ops import conv as cmod

    _conv(wino=True, min_c=128, tile=2)  # the production choice
    recs = []
    orig = cmod._Conv.backward
    # dw is read right after each backward: its output transform must not be deferred
    defer, cmod._DEFER_WOUT = cmod._DEFER_WOUT, False

    def bwd(ctx, dy):
        from ewdml.ops.nn import materialize

        materialize(dy)  # a lazily formed BN input gradient (ops/nn.py): record its values
        x, w = ctx.saved_tensors
        # a lazily applied BN output (the Winograd conv's forward transformed it on the fly, its
        # backward never reads it): write it for the float64 reference
        materialize(x)
        had_sink = ctx.sink is not None and getattr(ctx.sink, "grad", None) is not None
        dx, dw, a, b = orig(ctx, dy)
        recs.append((x.detach().clone(), w.detach().clone(), dy.detach().clone(),
                     None if (dx is None or had_sink) else dx.detach().clone(), dw.detach().clone()))
        return dx, dw, a, b

    cmod._Conv.backward = staticmethod(bwd)
    try:
        torch.manual_seed(0)
        m = build_model("resnet18", 10).to(memory_format=torch.channels_last).cuda()
        x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (32,), device="cuda")
        F.cross_entropy(m(x), y).backward()
    finally:
        cmod._Conv.backward = orig
        cmod._DEFER_WOUT = defer
    assert len(recs) >= 12
    for x, w, dy, dx, dw in recs:
        _, gx, gw = _ref64(x, w, w.shape[-1], dy)
        assert _rel(dw, gw) < TOL, (tuple(x.shape), _rel(dw, gw))
        if dx is not None:
            assert _rel(dx, gx) < TOL, (tuple(x.shape), _rel(dx, gx))


@pytest.mark.parametrize("steps", [3])
def test_lazy_bn_through_winograd_matches_materialised(steps):
    """VGG-11 fp32 training steps with the BN layers in front of / behind the Winograd convs
    applied inside the convs' input transforms (ops/nn.py lazy BN, winograd_f32.hip WgSrc) equal
    the materialised path bit for bit: losses, weights, running statistics, batch counters.
    The lazy run also leaves the BN backward applies to the producing convs (ops/nn.py
    _LAZY_BWD: the Winograd backward input transforms and the stem's weight gradient)."""
    from ewdml.models import build_model
    from ewdml.models import fused
    from ewdml.ops import nn as onn

    _conv(wino=True, min_c=128, tile=2, sm=True)  # the production choice
    torch.manual_seed(0)
    m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last).cuda()
    for mod in m0.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    x = torch.randn(64, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda")
    runs = []
    lazy_bwd = onn._LAZY_BWD
    for lazy in (True, False):
        fused._LAZY = lazy
        onn._LAZY_BWD = lazy
        try:
            m = copy.deepcopy(m0)
            opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
            losses = []
            for _ in range(steps):
                opt.zero_grad()
                loss = F.cross_entropy(m(x), y)
                loss.backward()
                opt.step()
                losses.append(float(loss.detach()))
            runs.append((m, losses))
        finally:
            fused._LAZY = True
            onn._LAZY_BWD = lazy_bwd
    (ml, ll), (me, le) = runs
    # the input transforms evaluate the BN kernels' own expressions: bit-identical training
    assert ll == le
    for (k, a), b in zip(ml.state_dict().items(), me.state_dict().values()):
        assert torch.equal(a, b), k  # incl. num_batches_tracked: counted once per step


@pytest.mark.parametrize("m", [2, 4])
def test_winograd_deferred_wgrad_output_transform(m):
    """A Winograd layer's weight-gradient output transform is deferred (ops/conv.py _PENDING) and
    rides in the next same-m backward-data input launch, or is flushed at the end of the backward
    pass: the gradients are bitwise those of the immediate transform, also when a second backward
    accumulates into existing .grad tensors (no deferral then) and through the exchange engine's
    flush (conv.flush_pending)."""
    conv = _conv(True, 64, str(m))
    torch.manual_seed(0)
    N, H = 16, 8
    chans = [64, 128, 128, 64]
    ws = [torch.nn.Parameter((torch.randn(co, ci, 3, 3, device="cuda") / (3 * ci ** 0.5))
                             .contiguous(memory_format=torch.channels_last))
          for ci, co in zip(chans[:-1], chans[1:])]
    x = torch.randn(N, chans[0], H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    dy = torch.randn(N, chans[-1], H, H, device="cuda").contiguous(
        memory_format=torch.channels_last)
    handles = _opt_in(ws)

    def run(defer, passes=1):
        conv._DEFER_WOUT = defer
        conv._POISON_DW = True  # a read of dw before its transform ran would show as NaN
        for w in ws:
            w.grad = None
        x.grad = None
        seen = []
        for _ in range(passes):
            y = x
            for w in ws:
                assert conv.wino_tile(y, w) == m
                y = conv.conv(y, w)
            y.backward(dy)
            seen.append(conv._PENDING is None)  # flushed by the end-of-backward callback
        torch.cuda.synchronize()
        return [w.grad.clone() for w in ws] + [x.grad.clone()], seen

    try:
        ref, _ = run(False)
        got, seen = run(True)
        assert all(seen)
        for a, b in zip(got, ref):
            assert not torch.isnan(a).any()
            assert torch.equal(a, b)
        ref2, _ = run(False, passes=2)
        got2, seen2 = run(True, passes=2)
        assert all(seen2)
        for a, b in zip(got2, ref2):
            assert torch.equal(a, b)
        # the engine's explicit flush after the pass's own callback: idempotent
        conv._DEFER_WOUT = True
        conv._POISON_DW = True
        for w in ws:
            w.grad = None
        y = x
        for w in ws:
            y = conv.conv(y, w)
        y.backward(dy)
        conv.flush_pending()
        torch.cuda.synchronize()
        for w, r in zip(ws, ref):
            assert torch.equal(w.grad, r)
    finally:
        conv._DEFER_WOUT = True
        conv._POISON_DW = False
        _opt_out(ws, handles)


@pytest.mark.parametrize("k0", [3, 1])
def test_winograd_deferred_transform_rides_in_direct_bwd_data(k0):
    """The deferred weight-gradient output transform of a Winograd layer rides in the direct
    (non-Winograd) conv's backward-data GEMM launch behind it (ops/csrc/conv_f32.hip WgOut rider):
    bitwise the immediate transform."""
    conv = _conv(True, 128, "2")
    torch.manual_seed(1)
    N, H = 128, 16  # VGG-11's conv2 -> conv3 (the bwd-data GEMM takes 128-row tiles)
    w0 = torch.nn.Parameter((torch.randn(128, 64, k0, k0, device="cuda") / (k0 * 8.0))
                            .contiguous(memory_format=torch.channels_last))
    w1 = torch.nn.Parameter((torch.randn(128, 128, 3, 3, device="cuda") / 34.0)
                            .contiguous(memory_format=torch.channels_last))
    ws = [w0, w1]
    x = torch.randn(N, 64, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    dy = torch.randn(N, 128, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    handles = _opt_in(ws)

    def run(defer):
        conv._DEFER_WOUT = defer
        conv._POISON_DW = True
        conv.new_pass()  # the exchange engine's begin: not a second (tied) use of the weights
        for w in ws:
            w.grad = None
            w._ew_tied = False
        x.grad = None
        rides = conv.WO_RIDES
        h = conv.conv(x, w0)
        assert conv.wino_tile(x, w0) == 0 and conv.wino_tile(h, w1) == 2
        conv.conv(h, w1).backward(dy)
        torch.cuda.synchronize()
        return [w.grad.clone() for w in ws] + [x.grad.clone()], conv.WO_RIDES - rides

    try:
        ref, r0 = run(False)
        got, r1 = run(True)
        assert r0 == 0 and r1 == 1
        for a, b in zip(got, ref):
            assert not torch.isnan(a).any()
            assert torch.equal(a, b)
    finally:
        conv._DEFER_WOUT = True
        conv._POISON_DW = False
        _opt_out(ws, handles)


def _opt_in(ws):
    """Mark parameters the way parallel/engine.py does (a post-accumulate hook it owns, counted
    in _ew_engine_hooks): only those defer their weight-gradient output transform."""
    hs = []
    for w in ws:
        hs.append(w.register_post_accumulate_grad_hook(lambda p: None))
        w._ew_engine_hooks = 1
    return hs


def _opt_out(ws, hs):
    for w, h in zip(ws, hs):
        h.remove()
        w._ew_engine_hooks = 0


@pytest.mark.parametrize("opt_in", [False, True])
def test_winograd_autograd_grad_matches_fp64(opt_in):
    """torch.autograd.grad never installs .grad: a deferred transform must still land in the dw
    tensor it returns (the job writes dw's own memory at the end-of-backward callback), and a
    foreign post-accumulate hook disables deferral."""
    conv = _conv(True, 64, "2")
    torch.manual_seed(3)
    N, H, C, Nc = 16, 8, 128, 128
    x, w0 = _data(N, C, Nc, H, H, seed=4)
    ws = [torch.nn.Parameter(w0.clone())]
    hs = _opt_in(ws) if opt_in else []
    g = torch.Generator(device="cuda").manual_seed(9)
    dy = torch.randn(N, Nc, H, H, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    try:
        conv._POISON_DW = True
        xa = x.clone().requires_grad_(True)
        y = conv.conv(xa, ws[0])
        gx, gw = torch.autograd.grad(y, [xa, ws[0]], dy)
        assert conv._PENDING is None
        torch.cuda.synchronize()
        _, rx, rw = _ref64(x, w0, 3, dy)
        assert not torch.isnan(gw).any()
        assert _rel(gw, rw) < TOL and _rel(gx, rx) < TOL
        assert ws[0].grad is None
        # a foreign hook on an opted-in parameter: no deferral, .backward() still exact
        extra = ws[0].register_post_accumulate_grad_hook(lambda p: None)
        y = conv.conv(x, ws[0])
        y.backward(dy)
        extra.remove()
        torch.cuda.synchronize()
        assert _rel(ws[0].grad, rw) < TOL
    finally:
        conv._POISON_DW = False
        _opt_out(ws, hs)


def test_exchange_tied_winograd_weights():
    """A Winograd conv weight used twice in one pass under the exchange engine, which opts its
    parameters into deferred weight-gradient transforms (pointer-mode gradients: .grad is None
    when backward starts, as in the trainer): autograd sums the two dw contributions in its input
    buffer before any hook runs, so that weight must not defer; the exchanged gradient equals the
    float64 reference on every pass."""
    conv = _conv(True, 64, "2")
    from ewdml.compress.codecs import make_codec
    from ewdml.optim.flat import FlatSGD
    from ewdml.parallel.comm import Comm
    from ewdml.parallel.engine import GradientExchange
    from ewdml.parallel.flat import FlatModel

    torch.manual_seed(5)
    N, H, C = 16, 8, 128
    w = torch.nn.Parameter((torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5))
                           .contiguous(memory_format=torch.channels_last))
    other = torch.nn.Parameter((torch.randn(C, C, 3, 3, device="cuda") / (3 * C ** 0.5))
                               .contiguous(memory_format=torch.channels_last))
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    flat = FlatModel([w, other], attach_grads=False)
    ex = GradientExchange(flat, Comm(), make_codec("none"), FlatSGD(flat, lr=0.0))
    try:
        conv._POISON_DW = True
        for it in range(2):
            flat.zero_grad()
            ex.begin()
            assert conv.wino_tile(x, w) == 2
            y = conv.conv(conv.conv(conv.conv(x, w), other), w)
            y.backward(dy)
            ex.finish(apply=False)
            ex.decode_average()
            torch.cuda.synchronize()
            xr = x.double().cpu()
            wr = w.detach().double().cpu().requires_grad_(True)
            orr = other.detach().double().cpu().requires_grad_(True)
            yr = F.conv2d(F.conv2d(F.conv2d(xr, wr, padding=1), orr, padding=1), wr, padding=1)
            yr.backward(dy.double().cpu())
            def gview(p):  # the parameter's slot of the flat gradient, in its own layout
                o = flat.offsets[next(i for i, q in enumerate(flat.params) if q is p)]
                return flat.grad[o:o + p.numel()].as_strided(p.shape, p.stride())

            assert not torch.isnan(flat.grad).any()
            assert _rel(gview(w), wr.grad) < TOL, (it, _rel(gview(w), wr.grad))
            assert _rel(gview(other), orr.grad) < TOL, (it, _rel(gview(other), orr.grad))
        assert getattr(w, "_ew_tied", False) and not getattr(other, "_ew_tied", False)
    finally:
        conv._POISON_DW = False
        ex.close()


@pytest.mark.parametrize("s2", [True, False])
def test_projection_shortcut_gradient_sink_matches_autograd_sum(s2):
    """ResNet-50 projection shortcuts (stride 1 in layer 1 on the MFMA conv; stride 2 on our
    stride-2 kernels or MIOpen) hand the block input's shortcut gradient to conv1's backward-data
    epilogue through a GradSink (models/resnet.py): one fp32 step with the sinks matches the step
    where autograd sums the two input gradients (bitwise forward on our kernels; MIOpen's fp32
    solvers are not run-to-run deterministic)."""
    from ewdml.models import build_model, resnet
    from ewdml.ops import conv as cmod

    _conv(wino=True, min_c=128, tile="size")
    cmod.set_stride2(s2)
    torch.manual_seed(0)
    m0 = build_model("resnet50", 10).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    # MIOpen (the stride-2 convs) picks its solvers on the first call: settle them first
    F.cross_entropy(copy.deepcopy(m0)(x), y).backward()
    res = []
    # MIOpen: a second run without sinks measures the run-to-run noise (BN's cancellations
    # amplify fp32 solver differences to ~1e-2 in the gradients after 50 layers)
    for sink in (True, False) if s2 else (True, False, False):
        resnet.set_residual_sink(sink)
        m = copy.deepcopy(m0)
        adds = cmod.SINK_ADDS
        try:
            out = m(x)
            F.cross_entropy(out, y).backward()
        finally:
            resnet.set_residual_sink(True)
        n = cmod.SINK_ADDS - adds
        # 16 blocks: 12 identity + 4 projection sinks; none with the sinks off
        assert n == (16 if sink else 0), n
        res.append((out.detach(), [p.grad.detach().clone() for p in m.parameters()]))
    (o_a, g_a), (o_b, g_b) = res[:2]
    errs = [_rel(a, b) for a, b in zip(g_a, g_b)]
    e = sum(errs) / len(errs)
    if s2:
        assert torch.equal(o_a, o_b)
        assert e < 1e-5, (e, max(errs))
    else:
        g_c = res[2][1]
        noise = [_rel(a, b) for a, b in zip(g_c, g_b)]
        e_n = sum(noise) / len(noise)
        assert _rel(o_a, o_b) < 1e-4, _rel(o_a, o_b)
        assert e <= 3 * e_n + 1e-5 and max(errs) <= 3 * max(noise) + 1e-5, (e, e_n, max(errs),
                                                                             max(noise))


# ---- 2x2-map dense position GEMMs (ops/csrc/smallmap_f32.hip) ----
SM_SHAPES = [  # (N, C, Nc) on 2x2 maps
    (128, 512, 512),   # VGG-11 conv7 / conv8: tile counts multiples of 8 (XCD-grouped splits)
    (64, 256, 128),
    (64, 64, 192),     # 12 forward / 4 backward tiles: plain split mapping
    (192, 128, 64),
]


@pytest.mark.parametrize("N,C,Nc", SM_SHAPES)
def test_conv_f32_smallmap_forward_backward(N, C, Nc):
    """Forward, input and weight gradient of the 2x2-map GEMMs against float64; bitwise
    repeatable (in-launch split-K reduced in split order); close to the direct kernels."""
    conv = _conv(sm=True)
    x, w = _data(N, C, Nc, 2, 2, seed=51)
    assert conv.smallmap_for(tuple(x.shape), x.dtype, w)
    g = torch.Generator(device="cuda").manual_seed(52)
    dy = torch.randn(N, Nc, 2, 2, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = conv.conv(xa, wa)
    assert getattr(y.grad_fn, "sm", None) is not None  # the small-map path ran
    y.backward(dy)
    ref, gx, gw = _ref64(x, w, 3, dy)
    assert _rel(y, ref) < TOL, _rel(y, ref)
    assert _rel(xa.grad, gx) < TOL, _rel(xa.grad, gx)
    assert _rel(wa.grad, gw) < TOL, _rel(wa.grad, gw)
    xb, wb = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y2 = conv.conv(xb, wb)
    y2.backward(dy)
    assert torch.equal(y, y2) and torch.equal(xa.grad, xb.grad) and torch.equal(wa.grad, wb.grad)
    d = _conv(sm=False)
    assert _rel(d.conv(x, w), y) < 2 * TOL
    # only one of the gradients requested
    xc = x.clone().requires_grad_(True)
    _conv(sm=True).conv(xc, w).backward(dy)
    assert torch.equal(xc.grad, xa.grad)
    wc = w.clone().requires_grad_(True)
    _conv(sm=True).conv(x, wc).backward(dy)
    assert torch.equal(wc.grad, wa.grad)


@pytest.mark.parametrize("N,C,Nc", SM_SHAPES[:2])
def test_conv_f32_smallmap_fenced_handoff_bitwise(N, C, Nc):
    """The small-map split-K hand-off has two forms (ops/csrc/smallmap_f32.hip sm_reduce): the
    default write-through one (sc1 stores and loads, no fences: MI355X_MICROARCH.md's hand-off
    table, row 1) and the fenced one (plain stores, agent release before the ticket, acquire
    after it: the HIP memory model's own form, EWDML_SM_FENCE=1).  Both give the same bits, so
    the fenced path stays a drop-in should the write-through form ever stop holding."""
    from ewdml import ops

    conv = _conv(sm=True)
    C_ = ops.require()
    x, w = _data(N, C, Nc, 2, 2, seed=57)
    g = torch.Generator(device="cuda").manual_seed(58)
    dy = torch.randn(N, Nc, 2, 2, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    outs = []
    prev = C_.sm_set_fence(0)
    try:
        for fence in (0, 1):
            C_.sm_set_fence(fence)
            xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
            y = conv.conv(xa, wa)
            y.backward(dy)
            torch.cuda.synchronize()
            outs.append((y.detach(), xa.grad, wa.grad))
    finally:
        C_.sm_set_fence(prev)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_conv_f32_smallmap_bn_statistics():
    """The split-K reducer's BatchNorm partial sums (8 rows) give the BN kernels' own statistics."""
    from ewdml.ops import nn as fnn

    conv = _conv(sm=True)
    x, w = _data(128, 512, 512, 2, 2, seed=53)
    bn0 = torch.nn.BatchNorm2d(512).cuda()
    bn1 = copy.deepcopy(bn0)
    h = conv.conv(x, w.clone().requires_grad_(True))
    part, rows = h._ew_bn_part
    assert rows == 8
    y0 = fnn.bn_act(h, bn0, "relu")
    y1 = fnn.bn_act(h.detach().clone(), bn1, "relu")
    assert _rel(y0, y1) < 1e-5
    assert torch.allclose(bn0.running_mean, bn1.running_mean, rtol=1e-5, atol=1e-7)
    assert torch.allclose(bn0.running_var, bn1.running_var, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("front_pool", [False, True])
@pytest.mark.parametrize("pool", [True, False])
def test_conv_f32_smallmap_lazy_bn_matches_materialised(pool, front_pool):
    """conv -> BN-ReLU -> 2x2-map conv -> BN-ReLU(-pool to 1x1): with the BN layers applied inside
    the small-map GEMM's operand loads (forward x, backward dy; ops/nn.py lazy BN) every output,
    gradient, running statistic and batch counter equals the materialised path bit for bit; the
    producing BN layer's backward sums come from the reducer (pooled: routed by the 4x4 -> 2x2
    window codes).  The 2x2-map conv's output is also checked against float64."""
    from ewdml.ops import nn as fnn

    conv = _conv(wino=True, min_c=64, tile=2, sm=True)
    N, C = 64, 128
    HW0 = 4 if front_pool else 2
    x0, w0 = _data(N, C, C, HW0, HW0, seed=61)
    _, w1 = _data(N, C, C, 2, 2, seed=62)
    bns = [torch.nn.BatchNorm2d(C).cuda() for _ in range(2)]
    with torch.no_grad():
        for bn in bns:
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.3, 0.3)
    gshape = (N, C, 1, 1) if pool else (N, C, 2, 2)
    g = torch.randn(gshape, device="cuda").contiguous(memory_format=torch.channels_last)
    lazy_bwd, sm_lazy = fnn._LAZY_BWD, conv._SM_LAZY_BWD
    runs = []
    try:
        for lazy in (True, False):
            fnn._LAZY_BWD = lazy
            conv._SM_LAZY_BWD = lazy  # the lazy dy path of the small-map backward (opt-in)
            b0, b1 = copy.deepcopy(bns[0]), copy.deepcopy(bns[1])
            xa, wa, wb = (t.clone().requires_grad_(True) for t in (x0, w0, w1))
            h = conv.conv(xa, wa)
            y = fnn.bn_relu(h, None, b0, pool=front_pool, lazy=lazy and not front_pool)
            z = conv.conv(y, wb)
            assert getattr(z.grad_fn, "sm", None) is not None
            if not lazy:
                zref = _ref64(fnn.materialize(y).detach(), w1, 3)
                assert _rel(z, zref) < TOL, _rel(z, zref)
            out = fnn.bn_act(z, b1, "relu", pool=pool)
            out.backward(g)
            runs.append([out, xa.grad, wa.grad, wb.grad] +
                        [t for b in (b0, b1) for t in (b.weight.grad, b.bias.grad,
                                                      b.running_mean, b.running_var,
                                                      b.num_batches_tracked)])
    finally:
        fnn._LAZY_BWD, conv._SM_LAZY_BWD = lazy_bwd, sm_lazy
    for i, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("N,C", [(64, 128), (128, 512)])
@pytest.mark.parametrize("pool", [True, False])
def test_bn_finalize_rides_in_smallmap_backward(N, C, pool):
    """The BN backward finalisation formed by each channel tile's last row tile of the 2x2-map
    backward launch (ops/csrc/smallmap_f32.hip, bn_fin.h ew_bn_bwd_fin_chan) gives bitwise the
    gradients of the finalize launch."""
    from ewdml.ops import conv as cmod
    from ewdml.ops import nn as fnn

    _conv(wino=True, min_c=64, tile=2, sm=True)
    HW = 4 if pool else 2
    x0, w0 = _data(N, C, C, HW, HW, seed=81)
    _, w1 = _data(N, C, C, 2, 2, seed=82)
    bn0 = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn0.weight.uniform_(0.5, 1.5)
        bn0.bias.uniform_(-0.3, 0.3)
    g = torch.randn(N, C, 2, 2, device="cuda").contiguous(memory_format=torch.channels_last)
    grads = []
    saved = cmod._FIN_RIDE
    try:
        for ride in (True, False):
            cmod._FIN_RIDE = ride
            rides = cmod.FIN_RIDES
            bn = copy.deepcopy(bn0)
            xa, wa, wb = (t.clone().requires_grad_(True) for t in (x0, w0, w1))
            z = cmod.conv(fnn.bn_act(cmod.conv(xa, wa), bn, "relu", pool=pool), wb)
            assert getattr(z.grad_fn, "sm", None) is not None
            z.backward(g)
            assert (cmod.FIN_RIDES > rides) == ride
            grads.append([xa.grad, wa.grad, wb.grad, bn.weight.grad, bn.bias.grad])
    finally:
        cmod._FIN_RIDE = saved
    for a, b in zip(*grads):
        assert torch.equal(a, b), _rel(a, b)


@pytest.mark.parametrize("mode,pool", [("relu", True), ("relu", False), ("none", False)])
def test_conv_f32_smallmap_bn_backward_sums(mode, pool):
    """The 2x2-map backward-data reducer's BN backward sums (the producing BN layer's sum dz and
    sum dz * (h - mean), routed through its 4x4 -> 2x2 pool codes) give the gradients of the BN
    layer's own statistics pass."""
    from ewdml.ops import nn as fnn

    conv = _conv(wino=True, min_c=64, tile=2, sm=True)
    N, C = 64, 128
    HW = 4 if pool else 2
    x0, w0 = _data(N, C, C, HW, HW, seed=71)
    _, w1 = _data(N, C, C, 2, 2, seed=72)
    bn0 = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn0.weight.uniform_(0.5, 1.5)
        bn0.bias.uniform_(-0.3, 0.3)
    g = torch.randn(N, C, 2, 2, device="cuda").contiguous(memory_format=torch.channels_last)
    grads = []
    for fused in (True, False):
        conv.set_bn_bwd_fusion(fused)
        used = fnn.PRE_BWD_USED
        bn = copy.deepcopy(bn0)
        xa, wa, wb = (t.clone().requires_grad_(True) for t in (x0, w0, w1))
        h = conv.conv(xa, wa)
        y = fnn.bn_act(h, bn, mode, pool=pool)
        z = conv.conv(y, wb)
        assert getattr(z.grad_fn, "sm", None) is not None
        z.backward(g)
        assert (fnn.PRE_BWD_USED > used) == fused
        grads.append([xa.grad, wa.grad, wb.grad, bn.weight.grad, bn.bias.grad])
    conv.set_bn_bwd_fusion(True)
    for i, (a, b) in enumerate(zip(*grads)):
        assert _rel(a, b) < 1e-5, (i, _rel(a, b))


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,Nc,HW", [(64, 64, 256, 8), (32, 128, 512, 4), (16, 512, 2048, 4)])
def test_conv_f32_1x1_lazy_bn_matches_materialised(N, C, Nc, HW):
    """ResNet bottleneck tail: 1x1 conv -> BN-ReLU -> 1x1 conv -> BN.  With the middle BN layer
    applied in the second conv's GEMM operand staging (forward A rows and weight-gradient x rows
    formed from h, conv_f32.hip CfLz; ops/nn.py lazy BN) every output, gradient, running
    statistic and batch counter equals the materialised path bit for bit, and the lazy conv's
    output matches float64."""
    from ewdml.ops import nn as fnn

    conv = _conv()
    x0, w0 = _data(N, C, C, HW, HW, seed=71, k=1)
    _, w1 = _data(N, C, Nc, HW, HW, seed=72, k=1)
    bns = [torch.nn.BatchNorm2d(C).cuda(), torch.nn.BatchNorm2d(Nc).cuda()]
    with torch.no_grad():
        for bn in bns:
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.3, 0.3)
    g = torch.randn(N, Nc, HW, HW, device="cuda").contiguous(memory_format=torch.channels_last)
    runs = []
    uses = conv.LAZY_1X1_USES
    for lazy in (True, False):
        b0, b1 = copy.deepcopy(bns[0]), copy.deepcopy(bns[1])
        xa, wa, wb = (t.clone().requires_grad_(True) for t in (x0, w0, w1))
        h = conv.conv(xa, wa)
        y = fnn.bn_act(h, b0, "relu", lazy=lazy)
        assert conv.lazy_input_ok(tuple(y.shape), y.dtype, wb)
        z = conv.conv(y, wb)
        if lazy:
            assert conv.LAZY_1X1_USES == uses + 1
            # materialised only now, after the conv consumed it lazily (no second batch count)
            zref = _ref64(fnn.materialize(y).detach(), w1, 1)
            assert _rel(z, zref) < TOL, _rel(z, zref)
        out = fnn.bn_act(z, b1, "none")
        out.backward(g)
        runs.append([out, xa.grad, wa.grad, wb.grad] +
                    [t for b in (b0, b1) for t in (b.weight.grad, b.bias.grad, b.running_mean,
                                                  b.running_var, b.num_batches_tracked)])
    for i, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), i


@pytest.mark.gpu
def test_resnet50_lazy_bn_into_conv3_bitwise():
    """ResNet-50 (CIFAR stem, our stride-2 kernels: deterministic): every bottleneck's conv3 reads
    relu(bn2(h)) through its GEMM operand staging instead of a written activation; one training
    step's output, parameter gradients and BN buffers equal the materialised step bit for bit."""
    from ewdml.models import build_model
    from ewdml.ops import conv as cmod

    _conv(wino=True, min_c=128, tile="size")
    cmod.set_stride2(True)
    torch.manual_seed(0)
    m0 = build_model("resnet50", 10).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    saved = cmod._LAZY_1X1
    res = []
    try:
        for on in (True, False):
            cmod._LAZY_1X1 = on
            m = copy.deepcopy(m0)
            uses = cmod.LAZY_1X1_USES
            out = m(x)
            F.cross_entropy(out, y).backward()
            assert cmod.LAZY_1X1_USES - uses == (16 if on else 0)
            res.append([out.detach()] + [p.grad.detach().clone() for p in m.parameters()]
                       + [b.clone() for b in m.buffers()])
    finally:
        cmod._LAZY_1X1 = saved
    for i, (a, b) in enumerate(zip(*res)):
        assert torch.equal(a, b), i
