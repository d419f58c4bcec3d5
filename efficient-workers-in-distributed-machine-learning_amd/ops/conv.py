"""Stride-1 3x3 (pad 1) and 1x1 convolutions on the gfx950 matrix cores, and the
3-input-channel 3x3 stem.

:func:`conv` is ``F.conv2d(x, w, padding=k // 2)`` (no bias: the fused BN kernels fold the conv
bias) for channels_last activations and weights, as an autograd function whose forward,
backward-data and backward-weight are hand-written MFMA implicit-GEMM kernels:

* bf16 operands (``ops/csrc/conv.hip``, ``v_mfma_f32_16x16x32_bf16``): fp32 accumulation, bf16
  results, like MIOpen's bf16 convolutions;
* fp32 operands (``ops/csrc/conv_f32.hip``, ``v_mfma_f32_16x16x4_f32``): exact fp32 products and
  accumulation, fp32 results -- the reference's precision.  fp32 3x3 layers with at least
  ``EWDML_WINO_MIN_C`` (default 128) input and output channels run as Winograd F(2x2, 3x3)
  (``ops/csrc/winograd_f32.hip``: 2.25x fewer MFMA FLOPs, fp32 transforms; F(4x4, 3x3) with
  ``EWDML_WINO_TILE=4|auto``, ``EWDML_WINOGRAD=0`` keeps the direct kernels) -- forward, backward data and weight gradient (the forward's transformed input
  is kept for it).

:func:`conv2d_module` dispatches an ``nn.Conv2d`` (VGG's and ResNet's stride-1 3x3 / 1x1 layers,
and with ``EWDML_CONV_S2=1`` ResNet's fp32 stride-2 3x3 / 1x1 down-sampling convs: :func:`conv_s2`).  Shapes the kernels
do not take (C_in or C_out not a multiple of 64, NCHW, other strides/padding) go to ``F.conv2d``
(MIOpen) -- e.g. the ImageNet ResNet's 7x7/2 stem.
``EWDML_CONV=miopen`` (or ``set_enabled(False)``) routes every call to MIOpen (A/B),
``EWDML_CONV_F32=miopen`` only the fp32 ones.

Parity: the reference's convolutions are ``nn.Conv2d(..., kernel_size=3, padding=1)`` in
``src/model_ops/vgg.py:46-59`` and ``resnet.py:14-36``; only the execution differs.
"""
import os

import torch
import torch.nn.functional as F

from . import _ptr, _stream, require

_ENABLED = os.environ.get("EWDML_CONV", "hip") != "miopen"
# operand dtypes the kernels take: bf16 (conv.hip) and fp32 (conv_f32.hip, reference precision);
# EWDML_CONV_F32=miopen sends fp32 convolutions to MIOpen (A/B)
_DTYPES = ((torch.bfloat16,) if os.environ.get("EWDML_CONV_F32", "hip") == "miopen"
           else (torch.bfloat16, torch.float32))
# BN-backward statistics of the producing layer in the backward-data epilogue (EWDML_CONV_BN_BWD=0:
# the BN backward's own statistics pass)
_BN_BWD = os.environ.get("EWDML_CONV_BN_BWD", "1") != "0"
# ... and the residual-gradient addend (GradSink), only for inputs of at most this many elements:
# the bf16 epilogue reads the extra operands with 2-byte loads in the MFMA output layout, which on
# large maps costs more than the separate, vectorised statistics / add kernels it replaces; the
# fp32 epilogue's 4-byte loads pay everywhere (ResNet-50 fp32 with no limit: CIFAR +1.0 %, 224 px
# +2.2 %; bf16 with it lifted: -0.2 % / -0.9 %: profiles/ab/epilogue_fusion_size_gate.txt)
_EPI_MAX = int(os.environ.get("EWDML_EPI_MAX", str(1 << 23)))  # bf16 inputs
_EPI_MAX_F32 = int(os.environ.get("EWDML_EPI_MAX_F32", str(1 << 62)))


# Winograd F(m x m, 3x3) for fp32 3x3 layers with min(C_in, C_out) >= _WINO_MIN_C (the deep layers,
# where the GEMM outweighs the transforms' activation traffic: tools/probes/conv_f32_probe.py --wino).
# m: EWDML_WINO_TILE = size (default, below), 2, 4 or auto (4 where the map tiles by 4 and C_out <=
# 512, else 2).  m = 4 measured only +1.5 % on the VGG-11 step (smaller, more numerous GEMMs; 36-point
# transforms) for ~4x m = 2's rounding error (5e-6 vs 1.3e-6 relative for MIOpen's fp32 on the
# whole-network forward): the default keeps m = 2 (profiles/conv/winograd_f32_probe_m4.txt)
_WINO = os.environ.get("EWDML_WINOGRAD", "1") != "0"
_WINO_MIN_C = int(os.environ.get("EWDML_WINO_MIN_C", "128"))
# "size" (default): m = 4 where it fits and leaves at least _WINO_M4_MIN_TILES output tiles (the
# batched GEMMs' rows), else m = 2 -- ResNet-50's 16x16 / 28x28 layers gain from m = 4 (+2.2 % /
# +1.6 % with every fitting layer at m = 4), VGG-11's 8x8 / 4x4 ones lose (few, short GEMMs)
_WINO_TILE = os.environ.get("EWDML_WINO_TILE", "size")
_WINO_M4_MIN_TILES = int(os.environ.get("EWDML_WINO_M4_MIN_TILES", "2048"))
# m = 4 for the layers with min(C_in, C_out) <= this many channels (and m = EWDML_WINO_TILE above),
# for layers below _WINO_MIN_C too: 0 = off
_WINO_M4_MAX_C = int(os.environ.get("EWDML_WINO_M4_MAX_C", "0"))
# most K-splits of a Winograd weight-gradient GEMM (slab memory: splits x a^2 x C_out x C_in floats)
_WINO_WG_SPLITS = int(os.environ.get("EWDML_WINO_WG_SPLITS", "4"))
# Deferred Winograd weight-gradient output transforms (dw = G^T dU G).  dw feeds only the
# optimizer / codec, so its transform rides in the next same-m Winograd backward-data input launch
# (ops/csrc/winograd_f32.hip WgOut) instead of a launch of its own.  Opt-in: deferred only for a
# leaf Parameter whose .grad is None when its conv's backward runs and whose only post-accumulate
# hooks are the exchange engine's (parallel/engine.py counts them in ``_ew_engine_hooks`` and
# flushes before it reads a bucket), so no foreign hook (e.g. one on the AccumulateGrad node) can
# read dw early.  The job writes into dw's own memory (it keeps dw's storage alive, not the tensor:
# an extra tensor reference would stop AccumulateGrad from adopting dw), so the result is right
# whoever ends up holding dw -- the adopted .grad, or the tensor torch.autograd.grad returns.  If
# autograd installed a copy as .grad before the flush, the copy is refreshed from dw afterwards.
# A job is never dropped: it is flushed as a launch of its own by a second deferral, at the end of
# the backward pass (an autograd final callback, run on the caller's current stream) and by the
# exchange engine before it encodes a bucket, so a bucket's gradients are complete when its
# encode starts.
_DEFER_WOUT = os.environ.get("EWDML_WINO_DEFER_WOUT", "1") != "0"
# weight gradients on a second stream: a conv's wgrad runs beside the backward-data chain of the
# layers before it (the chain is the backward's critical path).  Joined before any consumer reads
# a gradient (join_wgrad: flush_pending, the end of the backward).
_WGRAD_SIDE = False
# weight-gradient launches collected before one fork to the side stream: each fork is a
# cross-stream edge of the captured graph, which costs replay time of its own
_WGRAD_BATCH = int(os.environ.get("EWDML_WGRAD_BATCH", "1"))
_SIDE = {}
_SIDE_PENDING = set()
_SIDE_QUEUE = []  # (device index, launch closure, tensors it reads / writes)
SIDE_LAUNCHES = 0  # weight gradients issued on the side stream (tests)
# fp32 stride-2 3x3 / 1x1 convs (ResNet down-sampling) on the MFMA kernels: opt-in
# (EWDML_CONV_S2=1).  Measured slower than MIOpen's tuned (find-mode) solvers on every ResNet-50
# shape, 2078 vs 1740 us per step for the six layers, ResNet-50 CIFAR 8.38K vs 8.53K img/s
# (profiles/ab/conv_stride2_vs_miopen.txt), so MIOpen keeps them by default
_S2 = os.environ.get("EWDML_CONV_S2", "0") == "1"
# fp32 3x3 layers over 2x2 maps (VGG-11's conv7 / conv8) as dense position GEMMs
# (ops/csrc/smallmap_f32.hip): one forward launch and one backward launch (data + weight gradient)
# instead of Winograd's input / GEMM / output transform per pass.  EWDML_SMALLMAP=0: Winograd
_SMALLMAP = os.environ.get("EWDML_SMALLMAP", "1") != "0"
# the BN backward that follows a 2x2-map conv left to that conv's backward launch (KIND 2 dy formed
# on load, EWDML_SM_LAZY_BWD=1) or written by the BN backward apply and read plain (default): the
# lazy dy cost the two backward launches +14 / +18 us (every one of the conv's GEMM tiles re-forms
# it), more than the two apply launches it saves; 3 interleaved rounds 1.197 / 1.193 / 1.201 vs
# 1.217 / 1.212 / 1.214 ms per step (profiles/ab/README.md)
_SM_LAZY_BWD = os.environ.get("EWDML_SM_LAZY_BWD", "0") == "1"
# fp32 1x1 convs of a lazily applied BN + ReLU input (ResNet bottleneck conv3 of relu(bn2(h))):
# the GEMM's operand staging forms the input from h in the forward and the weight gradient
# (conv_f32.hip CfLz), so the BN apply never writes it.  EWDML_LAZY_1X1=0: materialised
_LAZY_1X1 = os.environ.get("EWDML_LAZY_1X1", "1") != "0"
LAZY_1X1_USES = 0  # forward passes that took it (tests / diagnostics)
# the same for the Winograd convs (their backward input transforms form the KIND 2 dy)
_WINO_LAZY_BWD = os.environ.get("EWDML_WINO_LAZY_BWD", "1") != "0"
# the backward finalisation of the BN layer whose input gradient a conv's backward-data launch
# produced (its partial sums come from that launch's epilogue) riding in the same conv's fp32
# weight-gradient GEMM launch as extra blocks (ops/csrc/bn_fin.h) instead of its own launch after
# it; EWDML_BN_FIN_RIDE=0: the BN backward launches it
_FIN_RIDE = os.environ.get("EWDML_BN_FIN_RIDE", "1") != "0"
FIN_RIDES = 0  # finalisations that rode in a weight-gradient launch (tests / diagnostics)
# deferred Winograd weight-gradient output transforms that rode in a direct conv's backward-data
# GEMM (same switch, EWDML_BN_FIN_RIDE)
WO_RIDES = 0
# whether a direct conv's split-K weight-gradient reduction was left pending for the stem's
# reduction launch (ops/csrc/conv_f32.hip ew_cf_defer_reduce: the conv fed by the stem's BN layer,
# whose backward runs next); flush_pending runs it before any gradient is read
_STEM_RED = [False]
STEM_RED_DEFERS = 0  # reductions left for the stem's launch (tests / diagnostics)
_SM_WS = {}


def set_stride2(on: bool):
    """Route fp32 stride-2 3x3 / 1x1 convs through :func:`conv_s2` (True) or MIOpen."""
    global _S2
    _S2 = bool(on)
_PENDING = None  # (src, split, param, Nc, C, m, keep-alive tensors, dw storage, shape, stride)
_POISON_DW = False  # tests: NaN-fill each fresh dw, so a read before its transform shows


def _job_fixup(job):
    """(dw pointer, copy) of a job: the transform writes dw's memory; if autograd installed a
    different tensor as the parameter's .grad (a copy of the unwritten dw), ``copy`` is the
    (grad, dw view) pair to refresh afterwards."""
    store, shape, stride = job[7], job[8], job[9]
    dst = store.data_ptr()
    g = job[2].grad
    if g is None or g.data_ptr() == dst:
        return dst, None
    dw = torch.empty(0, dtype=torch.float32, device=g.device).set_(store, 0, shape, stride)
    return dst, (g, dw)


def _dw_may_lag(ctx):
    """Whether this conv's dw may be written after the backward returns it (deferred transform,
    side-stream launch): its parameter's gradient is installed, not accumulated (grad None, no
    tied use), and nothing but the exchange engine's hooks (which join / flush before reading)
    looks at it during the backward."""
    p = getattr(ctx, "w_param", None)
    if p is None or p.grad is not None or torch.is_grad_enabled():
        return False
    if getattr(p, "_backward_hooks", None) or getattr(p, "_ew_tied", False):
        return False
    eng = getattr(p, "_ew_engine_hooks", 0)
    post = getattr(p, "_post_accumulate_grad_hooks", None)
    return not post or len(post) <= eng


def _wgrad_side(device):
    """The weight-gradient stream of ``device`` when side-stream weight gradients are on
    (set_wgrad_stream; the trainer's --wgrad-stream), else None."""
    if not _WGRAD_SIDE:
        return None
    s = _SIDE.get(device.index)
    if s is None:
        s = _SIDE[device.index] = torch.cuda.Stream(device)
    return s


def set_wgrad_stream(on: bool):
    """Side-stream weight gradients on / off.  The trainer switches them on around its own
    backward passes only and joins (join_wgrad) right after: every other caller of backward()
    keeps single-stream convs."""
    global _WGRAD_SIDE
    _WGRAD_SIDE = bool(on)


def _issue_side():
    """Issue the collected weight-gradient launches on the side stream, after everything the
    current stream has issued (their inputs)."""
    if not _SIDE_QUEUE:
        return
    jobs = list(_SIDE_QUEUE)
    _SIDE_QUEUE.clear()
    cur = torch.cuda.current_stream()
    for idx in sorted({j[0] for j in jobs}):
        _SIDE[idx].wait_stream(cur)
        _SIDE_PENDING.add(idx)
    global SIDE_LAUNCHES
    SIDE_LAUNCHES += len(jobs)
    for idx, fn, keep in jobs:
        side = _SIDE[idx]
        for t in keep:
            if t is not None:
                t.record_stream(side)
        with torch.cuda.stream(side):
            fn()


def join_wgrad():
    """The current stream waits for the weight gradients issued on the side stream."""
    _issue_side()
    if _SIDE_PENDING:
        cur = torch.cuda.current_stream()
        for idx in list(_SIDE_PENDING):
            cur.wait_stream(_SIDE[idx])
        _SIDE_PENDING.clear()


def flush_pending(final=False, keep_stem_red=False):
    """Run a deferred weight-gradient output transform now (``final`` is accepted for the end-of-
    backward callback; every flush runs the job) and a split-K reduction left for the stem's
    launch (unless ``keep_stem_red``: the stem's own backward, which takes it).  Returns True."""
    global _PENDING
    join_wgrad()  # every caller is about to read (or transform) a weight gradient
    if _STEM_RED[0] and not keep_stem_red:  # left for the stem's reduction launch (C++ side)
        _STEM_RED[0] = False
        require().cf_flush_reduce()
    job = _PENDING
    if job is None:
        return True
    _PENDING = None
    dest, fix = _job_fixup(job)
    src, split, _p, Nc, C, m = job[:6]
    require().wino_f32_wgrad_out(_ptr(src), split, dest, Nc, C, m, _stream())
    if fix is not None:
        fix[0].copy_(fix[1])
    return True


def _flush_final():
    flush_pending(final=True)


def pending() -> bool:
    """True while a deferred transform has not been enqueued yet."""
    return _PENDING is not None


def _take_pending(m):
    """The pending job as riding arguments of an m-tile backward-data call (zeros: none)."""
    global _PENDING
    job = _PENDING
    if job is None or job[5] != m:
        return (0, 1, 0, 0, 0), None
    dest, fix = _job_fixup(job)
    if fix is not None:  # .grad is already a copy: a launch of its own, then the refresh
        flush_pending()
        return (0, 1, 0, 0, 0), None
    _PENDING = None
    src, split, _p, Nc, C = job[:5]
    return (_ptr(src), split, dest, Nc, C), job


_USE_EPOCH = [0]


def new_pass():
    """Start of a forward pass (the exchange engine's ``begin``): resets the tied-weight count."""
    _USE_EPOCH[0] += 1


# the momentum-corrected error-feedback staging of a weight gradient done by the kernel that
# forms it (the small-map backward; ops/csrc/dgc_stage.h): the exchange engine arms a parameter
# with ``_ew_dgc_stage`` (velocity / residual / parameter pointers at its slot, the momentum
# hyper-parameters, its stamp word) and the encode reads e instead of the gradient.
# Opt-in (EWDML_PRODUCER_STAGE=1): measured a wash on VGG-11 -- the encode's first pass gets
# ~10 us shorter and the two small-map backward launches ~4 us longer each
# (profiles/ab/README.md "Round 6"); off, the encode stages every tensor itself
_PRODUCER_STAGE = os.environ.get("EWDML_PRODUCER_STAGE", "0") == "1"
STAGE_RIDES = 0  # weight gradients staged by their producer (tests / diagnostics)
_NO_STAGE = (0, 0, 0, 0.0, 1.0, 0.0, 0, 0, 0)


def _stage_args(ctx):
    """The staging arguments of this conv's weight gradient, or None: armed by the exchange,
    and (as for a deferred transform) dw installed, not accumulated, and read by nothing but
    the engine's encode -- the gradient itself is never written."""
    p = getattr(ctx, "w_param", None)
    st = getattr(p, "_ew_dgc_stage", None) if p is not None else None
    if st is None or not _PRODUCER_STAGE or not _can_defer_any(p):
        return None
    return st


def _can_defer_any(p):
    if not (p.grad is None and p.dtype == torch.float32 and p.requires_grad
            and not torch.is_grad_enabled()):
        return False
    if getattr(p, "_backward_hooks", None) or getattr(p, "_ew_tied", False):
        return False
    eng = getattr(p, "_ew_engine_hooks", 0)
    post = getattr(p, "_post_accumulate_grad_hooks", None)
    return eng > 0 and (not post or len(post) <= eng)


def _can_defer(ctx):
    # opt-in: only parameters whose sole post-accumulate hooks are the exchange engine's (which
    # flushes before it reads); no tensor hooks on the weight (they would see dw unwritten)
    p = getattr(ctx, "w_param", None)
    if not (_DEFER_WOUT and p is not None and p.grad is None and p.dtype == torch.float32
            and p.requires_grad and not torch.is_grad_enabled()):
        return False
    if getattr(p, "_backward_hooks", None) or getattr(p, "_ew_tied", False):
        return False
    eng = getattr(p, "_ew_engine_hooks", 0)
    post = getattr(p, "_post_accumulate_grad_hooks", None)
    return eng > 0 and (not post or len(post) <= eng)


def set_winograd(on: bool, min_c: int = None, tile=None):
    """Winograd on/off, its channel threshold and tile size (2, 4 or "auto")."""
    global _WINO, _WINO_MIN_C, _WINO_TILE
    _WINO = bool(on)
    if min_c is not None:
        _WINO_MIN_C = int(min_c)
    if tile is not None:
        _WINO_TILE = str(tile)


def _pow2(v):
    return v > 0 and v & (v - 1) == 0


def _wino_fits(N, C, Nc, H, W, m):
    t = N * (H // m) * (W // m)
    return (H % m == 0 and W % m == 0 and t % 64 == 0 and _pow2(C) and _pow2(Nc)
            and max(C, Nc) <= (1024 if m == 2 else 512)
            and (m + 2) ** 2 * t * max(C, Nc) < 2 ** 31)


def wino_tile(x, w) -> int:
    """The Winograd output tile m (2 or 4) the fp32 conv of ``x`` by ``w`` takes, 0 for none:
    3x3, power-of-two channel counts in [_WINO_MIN_C, 1024 (m = 2) / 512 (m = 4)], H and W
    multiples of m, N*H*W/m^2 % 64 == 0."""
    return wino_tile_for(tuple(x.shape), x.dtype, w)


def wino_tile_for(shape, dtype, w) -> int:
    """:func:`wino_tile` for an input of this shape and dtype (before it exists)."""
    if not _WINO or dtype != torch.float32 or w.shape[-1] != 3 or w.dtype != dtype:
        return 0
    N, C, H, W = shape
    Nc = w.shape[0]
    if w.shape[1] != C:
        return 0
    if min(C, Nc) <= _WINO_M4_MAX_C:
        return 4 if min(C, Nc) >= 32 and _wino_fits(N, C, Nc, H, W, 4) else 0
    if min(C, Nc) < _WINO_MIN_C:
        return 0
    order = {"2": (2,), "4": (4,)}.get(_WINO_TILE, (4, 2))
    for m in order:
        if _wino_fits(N, C, Nc, H, W, m):
            if (m == 4 and _WINO_TILE == "size"
                    and N * (H // 4) * (W // 4) < _WINO_M4_MIN_TILES):
                continue
            return m
    return 0


def wino_ok(x, w) -> bool:
    return wino_tile(x, w) > 0


def set_smallmap(on: bool):
    """Dense position GEMMs for fp32 3x3 layers over 2x2 maps on / off (off: Winograd)."""
    global _SMALLMAP
    _SMALLMAP = bool(on)


def smallmap_for(shape, dtype, w) -> bool:
    """Whether the fp32 conv of an input of ``shape`` by ``w`` runs as the 2x2-map dense position
    GEMM (``ops/csrc/smallmap_f32.hip``): 3x3 weight, H = W = 2, N, C_in and C_out multiples of
    64."""
    if not _SMALLMAP or dtype != torch.float32 or w.dtype != dtype or tuple(w.shape[-2:]) != (3, 3):
        return False
    N, C, H, W = shape
    Nc = w.shape[0]
    return (H == 2 and W == 2 and w.shape[1] == C and N % 64 == 0 and C % 64 == 0
            and Nc % 64 == 0 and N * 4 * max(C, Nc) < 2 ** 31)


def lazy_1x1_ok(shape, dtype, w) -> bool:
    """Whether the fp32 1x1 conv of an input of ``shape`` forms a lazily applied (unpooled)
    BatchNorm + ReLU input in its GEMM operand staging (forward and weight gradient)."""
    if not _LAZY_1X1 or dtype != torch.float32 or w.dtype != dtype or tuple(w.shape[-2:]) != (1, 1):
        return False
    N, C, H, W = shape
    Nc = w.shape[0]
    return (w.shape[1] == C and C % 64 == 0 and Nc % 64 == 0 and (N * H * W) % 64 == 0
            and N * H * W * max(C, Nc) < 2 ** 31)


def lazy_input_ok(shape, dtype, w) -> bool:
    """Whether the conv of an input of ``shape`` forms a lazily applied BatchNorm(+ReLU) input on
    the fly (Winograd input transform, the 2x2-map GEMM's operand load, or a 1x1 GEMM's operand
    staging)."""
    if tuple(w.shape[-2:]) == (1, 1):
        return lazy_1x1_ok(shape, dtype, w)
    return wino_tile_for(shape, dtype, w) > 0 or smallmap_for(shape, dtype, w)


def _sm_ws(device, N, C, Nc):
    """(slab, tickets) of the 2x2-map GEMMs' in-launch split-K reduction, per (device, stream); the
    tickets are zeroed once and left zero by every launch."""
    C_ = require()
    key = (device.index, _stream())
    need = (C_.sm_f32_ws_floats(N, C, Nc), C_.sm_f32_counters(N, C, Nc))
    ws = _SM_WS.get(key)
    if ws is None or ws[0].numel() < need[0] or ws[1].numel() < need[1]:
        slab = torch.empty(max(need[0], ws[0].numel() if ws else 0), dtype=torch.float32,
                           device=device)
        cnt = torch.zeros(max(need[1], ws[1].numel() if ws else 0), dtype=torch.int32,
                          device=device)
        ws = _SM_WS[key] = (slab, cnt)
    return ws


def epilogue_fusion_ok(x) -> bool:
    """Whether a conv on input ``x`` takes the epilogue fusions (BN backward sums, addend)."""
    return x.numel() <= (_EPI_MAX_F32 if x.dtype == torch.float32 else _EPI_MAX)
_WS = {}


def set_enabled(on: bool):
    global _ENABLED
    _ENABLED = bool(on)


def enabled() -> bool:
    return _ENABLED


def set_bn_bwd_fusion(on: bool):
    global _BN_BWD
    _BN_BWD = bool(on)


def _ws(device):
    """fp32 split-reduction slabs, per (device, stream) (kernels on one stream run in order)."""
    key = (device.index, _stream())
    w = _WS.get(key)
    if w is None:
        # zeros: its last 64 floats are the DMA kernels' zero page (never written)
        w = torch.zeros(require().conv_ws_floats(), dtype=torch.float32, device=device)
        _WS[key] = w
    return w


def _one(v, want):
    return v == want or v == (want, want) or v == [want, want]


def _geometry_ok(x, w, stride, padding, dilation, groups, sizes=(1, 3)):
    if not (_ENABLED and x.is_cuda and x.dim() == 4 and w.dim() == 4):
        return False
    k = w.shape[-1]
    if k not in sizes or w.shape[-2] != k:
        return False
    if padding is None:
        padding = k // 2
    if not (_one(stride, 1) and _one(padding, k // 2) and _one(dilation, 1) and groups == 1):
        return False
    if x.dtype not in _DTYPES or w.dtype != x.dtype or w.shape[1] != x.shape[1]:
        return False
    return (x.is_contiguous(memory_format=torch.channels_last)
            and w.is_contiguous(memory_format=torch.channels_last))


def stem_supported(x, w, stride=1, padding=None, dilation=1, groups=1) -> bool:
    """True for the stem kernels: a 3x3 / pad 1 / stride 1 conv over 3 input channels (VGG's
    first layer, the CIFAR ResNet stem), C_out % 64 == 0, N*H*W % 256 == 0, W <= 256."""
    if not _geometry_ok(x, w, stride, padding, dilation, groups, sizes=(3,)):
        return False
    N, C, H, W = x.shape
    return (C == 3 and w.shape[0] % 64 == 0 and (N * H * W) % 256 == 0 and W <= 256
            and N * H * W * 3 < 2 ** 31 and N * H * W * w.shape[0] < 2 ** 31
            and x.data_ptr() % 16 == 0)


def supported(x, w, stride=1, padding=None, dilation=1, groups=1) -> bool:
    """True if the MFMA kernels take ``conv2d(x, w, stride, padding, dilation, groups)``: a 3x3
    kernel with padding 1 or a 1x1 kernel with padding 0, stride 1 (C_in % 64 == 0), or the
    3-channel stem (:func:`stem_supported`)."""
    if not _geometry_ok(x, w, stride, padding, dilation, groups):
        return False
    if stem_supported(x, w, stride, padding, dilation, groups):
        return True
    N, C, H, W = x.shape
    Nc = w.shape[0]
    if C % 64 or Nc % 64 or (N * H * W) % 64:
        return False
    if x.numel() >= 2 ** 31 or N * H * W * Nc >= 2 ** 31:
        return False
    return x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0


def s2_supported(x, w, stride=2, padding=None, dilation=1, groups=1) -> bool:
    """True for the fp32 stride-2 kernels: 3x3 / pad 1 or 1x1 / pad 0 at stride 2 (the ResNet
    down-sampling convs), channels_last fp32, even H and W, C_in and C_out % 64 == 0,
    N*H*W/4 % 64 == 0."""
    if not (_one(stride, 2) and x.dim() == 4 and w.dim() == 4 and w.dtype == torch.float32):
        return False
    if not _geometry_ok(x, w, 1, padding, dilation, groups):
        return False
    N, C, H, W = x.shape
    Nc = w.shape[0]
    return (H % 2 == 0 and W % 2 == 0 and C % 64 == 0 and Nc % 64 == 0
            and (N * (H // 2) * (W // 2)) % 64 == 0 and x.numel() < 2 ** 31
            and N * H * W * Nc < 2 ** 31 and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def _part_floats(M, C):
    """Capacity of a BN partial-sum buffer [2][rows][C]: the epilogue writes one row per 64 (or
    128) output rows, a split-K reduction up to min(M, 1024) rows (ops/csrc/conv.hip)."""
    return max(1, 2 * max(M // 64, min(M, 1024)) * C)


def _bn_bwd_link(node, x):
    """(h, code, stats, relu) of the fused BN layer ``node`` whose output is ``x`` (see
    ``ops.nn.bn_act``), for its backward statistics in this conv's backward-data epilogue."""
    if node is None:
        return None
    try:
        h, res, code, stats = node.saved_tensors
    except RuntimeError:  # already freed
        return None
    if h.dtype != x.dtype or node.mode not in ("relu", "none", "add_relu"):
        return None
    N, C, H, W = x.shape
    scale = 2 if node.pool else 1
    if tuple(h.shape) != (N, C, H * scale, W * scale):
        return None
    return h, res, code, stats, int(node.mode != "none")


def _arm_fin(job):
    """Arm the BN backward finalisation of ``job`` (see ``_FIN_RIDE``) for the next fp32
    weight-gradient GEMM launch; returns its outputs (coef, dgamma, dbeta, dcbias)."""
    if job is None:
        return None
    from .nn import bn_fin_outputs

    node, part, rows, h, stats = job
    Cb = h.shape[1]
    coef, dg, db, dcb = bn_fin_outputs(node, Cb, h.device)
    cb_dtype = getattr(node, "cb_dtype", None)
    M = h.shape[0] * h.shape[2] * h.shape[3]
    require().cf_arm_bn_fin(_ptr(part), int(rows), Cb, M, _ptr(stats), _ptr(coef), _ptr(dg),
                            _ptr(db), _ptr(dcb), int(cb_dtype == torch.bfloat16))
    return coef, dg, db, dcb


def _fin_done(node, fin):
    """After the weight-gradient launch: the finalisation ran in it (or runs now on its own); the
    BN backward of ``node`` takes its outputs instead of launching it."""
    global FIN_RIDES
    if require().cf_flush_bn_fin(_stream()) == 0:
        FIN_RIDES += 1
    pre = getattr(node, "_ew_pre_bwd", None)
    if pre is not None:
        node._ew_pre_bwd = pre[:4] + (fin,)


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bn_node=None, sink=None):
        C_ = require()
        N, C, H, W = x.shape
        Nc, k = w.shape[0], w.shape[-1]
        ws = _ws(x.device)
        y = torch.empty((N, Nc, H, W), dtype=x.dtype, device=x.device,
                        memory_format=torch.channels_last)
        # BatchNorm partial sums of y from the epilogue (bounded by 2 rows per 64 output rows);
        # the following fused BN (ops/nn.py bn_act) skips its statistics pass when present
        part = torch.empty(_part_floats(N * H * W, Nc), dtype=torch.float32, device=x.device)
        ctx.wino = None
        ctx.sm = None
        ctx.lz = None
        sm = sink is None and smallmap_for(tuple(x.shape), x.dtype, w)
        m = 0 if sm else wino_tile(x, w)
        # x may be the lazily applied output of a fused BN layer (ops/nn.py bn_relu(lazy=True)):
        # the Winograd input transform (or the 2x2-map GEMM's operand load, unpooled, or a 1x1
        # GEMM's operand staging, unpooled) applies that layer on the fly; anything else needs it
        lazy = getattr(x, "_ew_lazy_fwd", None)
        lz1 = (lazy is not None and not (m or sm) and k == 1 and not lazy[4]
               and lazy_1x1_ok(tuple(x.shape), x.dtype, w))
        if lazy is not None and ((not (m or sm) and not lz1) or (sm and lazy[4])):
            from .nn import materialize

            materialize(x)
            lazy = None
        if sm:
            slab, cnt = _sm_ws(x.device, N, C, Nc)
            bh, bstats, _bcode, bnbt, _bpool = lazy if lazy is not None else (None,) * 5
            rows = C_.sm_f32_fwd(_ptr(x) if lazy is None else 0, _ptr(bh), _ptr(bstats),
                                 _ptr(bnbt), _ptr(w), _ptr(y), _ptr(slab), slab.numel(),
                                 _ptr(cnt), cnt.numel(), N, C, Nc, _ptr(part), part.numel(),
                                 _stream())
            if lazy is not None:  # a later materialisation must not count the batch twice
                x._ew_materialize = getattr(x, "_ew_materialize_no_nbt", None)
            # the BN source of x (None: x itself), formed again by the weight gradient
            ctx.sm = ((bh, bstats) if lazy is not None else None,)
        elif m:
            aa = (m + 2) ** 2
            # transformed weight U[a^2][Nc][C] (m = 2: kept for the backward-data GEMMs, read
            # flipped) and input V (kept for the weight-gradient GEMMs)
            U = torch.empty(aa * Nc * C, dtype=torch.float32, device=x.device)
            t = N * (H // m) * (W // m)
            V = torch.empty(aa * t * C, dtype=torch.float32, device=x.device)
            Mo = torch.empty(aa * t * Nc, dtype=torch.float32, device=x.device)
            if lazy is not None:
                bh, bstats, bcode, bnbt, bpool = lazy
                rows = C_.wino_f32_fwd_bn(_ptr(bh), _ptr(bstats), _ptr(bcode), _ptr(bnbt),
                                          int(bpool), _ptr(w), _ptr(U), _ptr(y), _ptr(V),
                                          _ptr(Mo), N, H, W, C, Nc, m, _ptr(part), part.numel(),
                                          _stream())
                # a later materialisation must not count the batch twice
                x._ew_materialize = getattr(x, "_ew_materialize_no_nbt", None)
            else:
                rows = C_.wino_f32_fwd(_ptr(x), _ptr(w), _ptr(U), _ptr(y), _ptr(V), _ptr(Mo), N,
                                       H, W, C, Nc, m, _ptr(part), part.numel(), _stream())
            ctx.wino = (U if m == 2 else None, V, m)
        elif lz1:
            bh, bstats, _bcode, bnbt, _bpool = lazy
            rows = C_.conv_f32_fwd_lz(_ptr(bh), _ptr(bstats), _ptr(bnbt), _ptr(w), _ptr(y),
                                      _ptr(ws), ws.numel(), N, H, W, C, Nc, _ptr(part),
                                      part.numel(), _stream())
            # a later materialisation must not count the batch twice
            x._ew_materialize = getattr(x, "_ew_materialize_no_nbt", None)
            # x itself stays unwritten: the weight gradient forms it from the same source
            ctx.lz = (bh, bstats)
            global LAZY_1X1_USES
            LAZY_1X1_USES += 1
        else:
            fwd = C_.conv_f32_fwd if x.dtype == torch.float32 else C_.conv_fwd
            rows = fwd(_ptr(x), _ptr(w), _ptr(y), _ptr(ws), ws.numel(), N, H, W, C, Nc, k,
                       _ptr(part), part.numel(), _stream())
        ctx.save_for_backward(x, w)
        # the leaf Parameter itself (not a cast / copy): its .grad decides whether the Winograd
        # weight-gradient output transform may be deferred (_can_defer)
        ctx.w_param = w if isinstance(w, torch.nn.Parameter) else None
        ctx.bn_part = (part, rows) if rows > 0 else None
        ctx.bn_node = bn_node
        ctx.sink = sink
        return y

    @staticmethod
    def backward(ctx, dy):
        C_ = require()
        x, w = ctx.saved_tensors
        N, C, H, W = x.shape
        Nc, k = w.shape[0], w.shape[-1]
        if ctx.sm is not None:
            return _Conv._backward_sm(ctx, dy, x, w)
        # dy may be the lazily formed input gradient of the BN layer this conv feeds (ops/nn.py):
        # the Winograd backward-data input transform forms it on the fly, anything else needs it
        lazy = getattr(dy, "_ew_lazy_bwd", None)
        if lazy is not None and not (ctx.wino is not None and ctx.needs_input_grad[0]
                                     and dy.dtype == x.dtype):
            from .nn import materialize

            materialize(dy)
            lazy = None
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        f32 = x.dtype == torch.float32
        wo_job = None  # a deferred Winograd transform riding in this direct conv's bwd-data GEMM
        if ctx.wino is None:  # nothing here carries a deferred transform: run it while warm
            if (_FIN_RIDE and f32 and ctx.needs_input_grad[0] and _PENDING is not None
                    and _PENDING[5] == 2):
                join_wgrad()  # its source may come from the side stream
                wo, wo_job = _take_pending(2)
                if wo_job is not None:
                    require().cf_arm_wgout(*wo)
            else:
                flush_pending()
        ws = _ws(x.device)
        bwd_data = C_.conv_f32_bwd_data if f32 else C_.conv_bwd_data
        dx = dw = None
        fin_job = None  # (BN node, partials, rows, h, stats): its finalisation may ride in the wgrad
        stem_next = False
        D = None  # Winograd: the weight gradient's dy transform, made by the bwd-data pass
        m = ctx.wino[2] if ctx.wino is not None else 0
        aa = (m + 2) ** 2
        t = N * (H // m) * (W // m) if m else 0
        if m and ctx.needs_input_grad[1]:
            D = torch.empty(aa * t * Nc, dtype=torch.float32, device=x.device)
        d_ready = 0
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            node, ctx.bn_node = ctx.bn_node, None
            # a second gradient of x handed over by the BN backward of the block's identity
            # residual (models/resnet.py): added in the epilogue instead of by autograd
            sink, ctx.sink = ctx.sink, None
            add = getattr(sink, "grad", None) if sink is not None else None
            if add is not None and not (add.shape == x.shape and add.dtype == x.dtype
                                        and add.is_contiguous(memory_format=torch.channels_last)
                                        and add.data_ptr() % 16 == 0):
                add = add.contiguous(memory_format=torch.channels_last).to(x.dtype)
            if add is not None:
                global SINK_ADDS
                SINK_ADDS += 1
            link = _bn_bwd_link(node, x)
            if m:
                # m = 2: the forward's U, read flipped; m = 4: the rotated kernel's transform
                # is made here (U2), in the backward input launch
                U = ctx.wino[0]
                if U is None:
                    U = torch.empty(aa * Nc * C, dtype=torch.float32, device=x.device)
                buf = torch.empty(aa * t * (C + Nc), dtype=torch.float32, device=x.device)

                def bwd_data(dy_, w_, dx_, ws_, wsn, *rest):  # same contract, Winograd
                    # a deferred weight-gradient output transform of a later layer rides along
                    wo, job = _take_pending(m)
                    if lazy is not None:  # dy formed from the BN layer's backward on the fly
                        oh, odn, ocode, ostats, ocoef, opool = lazy
                        r = C_.wino_f32_bwd_data_bn(
                            _ptr(oh), _ptr(odn), _ptr(ocode), _ptr(ostats), _ptr(ocoef),
                            int(opool), w_, _ptr(U), dx_, _ptr(buf), _ptr(buf) + 4 * aa * t * Nc,
                            *rest[:5], m, *rest[6:-1], _ptr(D), *wo, rest[-1])
                    else:
                        r = C_.wino_f32_bwd_data(dy_, w_, _ptr(U), dx_, _ptr(buf),
                                                 _ptr(buf) + 4 * aa * t * Nc, *rest[:5], m,
                                                 *rest[6:-1], _ptr(D), *wo, rest[-1])
                    del job  # enqueued: the stream orders any reuse of its buffers after it
                    return r
                d_ready = int(D is not None)
            if link is None:
                bwd_data(_ptr(dy), _ptr(w), _ptr(dx), _ptr(ws), ws.numel(), N, H, W, C, Nc, k, 0,
                         0, 0, 0, 0, 0, 0, _ptr(add), _stream())
            else:
                # the producing BN layer's backward sums (sum dz, sum dz*(h-mean)) per 64 rows
                h, res, code, stats, relu = link
                part = torch.empty(_part_floats(N * H * W, C), dtype=torch.float32,
                                   device=x.device)
                rows = bwd_data(_ptr(dy), _ptr(w), _ptr(dx), _ptr(ws), ws.numel(), N, H, W, C,
                                Nc, k, _ptr(h), _ptr(res), _ptr(code), _ptr(stats), relu,
                                _ptr(part), part.numel(), _ptr(add), _stream())
                if rows > 0:
                    node._ew_pre_bwd = (part, rows, dx, dx._version)
                    if _FIN_RIDE and f32 and ctx.needs_input_grad[1]:
                        fin_job = (node, part, rows, h, stats)
                # the stem's backward runs next: its reduction launch may take this conv's
                stem_next = f32 and getattr(node, "stem_in", False)
            if sink is not None:
                sink.grad, sink.taken = None, True
        if wo_job is not None:
            # taken by the bwd-data GEMM (a 128-row tile) or run now on its own
            if require().cf_flush_wgout(_stream()) == 0:
                global WO_RIDES
                WO_RIDES += 1
            del wo_job  # enqueued: the stream orders any reuse of its buffers after it
        # (formed from the BN source even if x was materialised since: the same values)
        lz, ctx.lz = ctx.lz, None
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w, memory_format=torch.channels_last)
            side = _wgrad_side(x.device) if _dw_may_lag(ctx) else None
            V = ctx.wino[1] if m else None
            fin = _arm_fin(fin_job) if side is None else None

            def launch_wgrad():
                if m:
                    # dw = G^T (sum over tiles of (A dy A^T) V) G: a^2 GEMMs of K = N*H*W/m^2
                    dU = torch.empty(aa * Nc * C, dtype=torch.float32, device=x.device)
                    slabs = torch.empty(_WINO_WG_SPLITS * aa * Nc * C + 64,
                                        dtype=torch.float32, device=x.device)
                    # one pending job at a time: an earlier one is flushed first (if it cannot
                    # be yet, this layer's transform runs now)
                    if _POISON_DW:
                        dw.fill_(float("nan"))
                    defer = side is None and _can_defer(ctx) and flush_pending()
                    split = C_.wino_f32_wgrad(_ptr(dy), _ptr(V), _ptr(dw), _ptr(D), d_ready,
                                              _ptr(dU), _ptr(slabs), slabs.numel(), N, H, W, C,
                                              Nc, m, int(defer), _stream())
                    if defer:
                        global _PENDING
                        _PENDING = (slabs if split > 1 else dU, split, ctx.w_param, Nc, C, m,
                                    (dU, slabs), dw.untyped_storage(), tuple(dw.shape),
                                    dw.stride())
                        torch.autograd.Variable._execution_engine.queue_callback(_flush_final)
                else:
                    wgrad = C_.conv_f32_wgrad if f32 else C_.conv_wgrad
                    wsw = _ws(x.device)  # the current stream's slabs (the side stream's own)
                    # (like the deferred Winograd transforms, dw is then written after this
                    # backward returns: off with _DEFER_WOUT)
                    # only when dw is installed (not accumulated) and nothing but the engine's
                    # hooks reads it before the flush: a flat-view .grad (PS / sharded
                    # topologies), foreign hooks or autograd.grad callers need dw now
                    if stem_next and side is None and _FIN_RIDE and _can_defer(ctx):
                        C_.cf_defer_reduce()  # its split-K reduction: in the stem's launch
                        global STEM_RED_DEFERS
                        STEM_RED_DEFERS += 1
                        if not _STEM_RED[0]:  # run at the latest when the backward pass ends
                            torch.autograd.Variable._execution_engine.queue_callback(_flush_final)
                        _STEM_RED[0] = True
                    if lz is not None:  # x = relu(bn(h)) formed in the GEMM's operand staging
                        C_.conv_f32_wgrad_lz(_ptr(dy), _ptr(lz[0]), _ptr(lz[1]), _ptr(dw),
                                             _ptr(wsw), wsw.numel(), N, H, W, C, Nc, _stream())
                    else:
                        wgrad(_ptr(dy), _ptr(x), _ptr(dw), _ptr(wsw), wsw.numel(), N, H, W, C,
                              Nc, k, _stream())

            if side is None:
                launch_wgrad()
                if fin is not None:
                    _fin_done(fin_job[0], fin)
            else:
                # queued (holding its tensors, so their memory is not reused), issued on the side
                # stream with the next _WGRAD_BATCH - 1 ones or at the first gradient read
                _SIDE_QUEUE.append((x.device.index, launch_wgrad,
                                    (dy, x, dw, V, D) + (lz or ())))
                if len(_SIDE_QUEUE) >= _WGRAD_BATCH:
                    _issue_side()
        ctx.wino = None
        return dx, dw, None, None


    @staticmethod
    def _backward_sm(ctx, dy, x, w):
        """Backward of a 2x2-map conv: input and weight gradient in one launch, dy formed from the
        BN layer this conv feeds when it is lazy, x from the BN layer in front when it was."""
        C_ = require()
        flush_pending()  # a deferred Winograd weight-gradient transform, while its data is warm
        N, C, H, W = x.shape
        Nc = w.shape[0]
        xsrc, = ctx.sm
        ctx.sm = None
        lazy = getattr(dy, "_ew_lazy_bwd", None)
        if lazy is not None and dy.dtype != x.dtype:
            from .nn import materialize

            materialize(dy)
            lazy = None
        if lazy is None:
            dy = dy.contiguous(memory_format=torch.channels_last)
            if dy.dtype != x.dtype:
                dy = dy.to(x.dtype)
            if dy.data_ptr() % 16:
                dy = dy.clone(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w, memory_format=torch.channels_last)
        node, ctx.bn_node = ctx.bn_node, None
        ctx.sink = None
        link = _bn_bwd_link(node, x) if dx is not None else None
        ph, pres, pcode, pstats, prelu = link if link is not None else (None,) * 5
        part = (torch.empty(_part_floats(N * H * W, C), dtype=torch.float32, device=x.device)
                if link is not None else None)
        oh, odn, ocode, ostats, ocoef, opool = lazy if lazy is not None else (None,) * 6
        bh, bstats = xsrc if xsrc is not None else (None, None)
        slab, cnt = _sm_ws(x.device, N, C, Nc)
        # the BN layer's backward finalisation by each channel tile's last row tile of this launch
        # (the weight-gradient tiles run beside it; ops/csrc/smallmap_f32.hip k_sm_bwd)
        fin = None
        if link is not None and _FIN_RIDE:
            from .nn import bn_fin_outputs

            fin = bn_fin_outputs(node, C, x.device)
        coef, fdg, fdb, fdcb = fin if fin is not None else (None,) * 4
        cb_dtype = getattr(node, "cb_dtype", None) if node is not None else None
        # the exchange's momentum-corrected error-feedback staging of this weight's gradient, done
        # by the weight-gradient tiles of this launch (dgc_stage.h): dw is then never stored
        stage = _stage_args(ctx) if dw is not None else None
        if stage is not None:
            global STAGE_RIDES
            STAGE_RIDES += 1
        rows = C_.sm_f32_bwd(_ptr(x) if xsrc is None else 0, _ptr(bh), _ptr(bstats),
                             _ptr(dy) if lazy is None else 0, _ptr(oh), _ptr(odn), _ptr(ocode),
                             _ptr(ostats), _ptr(ocoef), int(bool(opool)), _ptr(w), _ptr(dx),
                             _ptr(dw), _ptr(slab), slab.numel(), _ptr(cnt), cnt.numel(), N, C,
                             Nc, _ptr(ph), _ptr(pres), _ptr(pcode), _ptr(pstats), int(prelu or 0),
                             _ptr(part), part.numel() if part is not None else 0, _ptr(coef),
                             _ptr(fdg), _ptr(fdb), _ptr(fdcb), int(cb_dtype == torch.bfloat16),
                             ph.shape[0] * ph.shape[2] * ph.shape[3] if ph is not None else 0,
                             _stream(), *(stage or _NO_STAGE))
        if rows > 0:
            node._ew_pre_bwd = (part, rows, dx, dx._version)
            if fin is not None:
                global FIN_RIDES
                FIN_RIDES += 1
                node._ew_pre_bwd += (fin,)
        return dx, dw, None, None


class _ConvStem(torch.autograd.Function):
    """3-channel 3x3 stem: MFMA forward (+ BN partials) and weight gradient; the input gradient
    (not needed when x is the network input) goes to MIOpen."""

    @staticmethod
    def forward(ctx, x, w):
        C_ = require()
        N, C, H, W = x.shape
        Nc = w.shape[0]
        y = torch.empty((N, Nc, H, W), dtype=x.dtype, device=x.device,
                        memory_format=torch.channels_last)
        part = torch.empty(max(1, 2 * (N * H * W // 128) * Nc), dtype=torch.float32,
                           device=x.device)
        fwd = C_.conv_f32_stem_fwd if x.dtype == torch.float32 else C_.conv_stem_fwd
        rows = fwd(_ptr(x), _ptr(w), _ptr(y), N, H, W, Nc, _ptr(part), part.numel(), _stream())
        ctx.save_for_backward(x, w)
        ctx.bn_part = (part, rows) if rows > 0 else None
        return y

    @staticmethod
    def backward(ctx, dy):
        C_ = require()
        flush_pending(keep_stem_red=True)  # a deferred Winograd transform, while its data is warm
        x, w = ctx.saved_tensors
        N, C, H, W = x.shape
        Nc = w.shape[0]
        # dy may be the lazily formed input gradient of the BN layer this stem feeds (ops/nn.py):
        # the fp32 weight-gradient kernel forms it on the fly; an input gradient needs it written
        lazy = getattr(dy, "_ew_lazy_bwd", None)
        if lazy is not None and (ctx.needs_input_grad[0] or not ctx.needs_input_grad[1]
                                 or x.dtype != torch.float32):
            from .nn import materialize

            materialize(dy)
            lazy = None
        if lazy is not None:
            oh, odn, ocode, ostats, ocoef, opool = lazy
            ws = _ws(x.device)
            dw = torch.empty_like(w, memory_format=torch.channels_last)
            C_.conv_f32_stem_wgrad_bn(_ptr(oh), _ptr(odn), _ptr(ocode), _ptr(ostats), _ptr(ocoef),
                                      int(opool), _ptr(x), _ptr(dw), _ptr(ws), ws.numel(), N, H,
                                      W, Nc, _stream())
            return None, dw
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        if dy.data_ptr() % 16:  # 16-B loads of dy rows
            dy = dy.clone(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(
                dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            ws = _ws(x.device)
            dw = torch.empty_like(w, memory_format=torch.channels_last)
            wgrad = C_.conv_f32_stem_wgrad if x.dtype == torch.float32 else C_.conv_stem_wgrad
            wgrad(_ptr(dy), _ptr(x), _ptr(dw), _ptr(ws), ws.numel(), N, H, W, Nc, _stream())
        return dx, dw


class _ConvS2(torch.autograd.Function):
    """fp32 stride-2 3x3 / 1x1 convolution (``ops/csrc/conv_f32.hip`` ``k_cf_gemm<..., 2>``): the
    forward and weight gradient gather the strided taps in their im2col loads; the backward data
    runs the four dx phases (pixels (2i + ph, 2j + pw)) as one launch, each phase a GEMM over only
    the taps that reach it (1, 2, 2 and 4 of a 3x3 kernel), so no zero-stuffed work."""

    @staticmethod
    def forward(ctx, x, w):
        C_ = require()
        N, C, H, W = x.shape
        Nc, k = w.shape[0], w.shape[-1]
        ws = _ws(x.device)
        Ho, Wo = H // 2, W // 2
        y = torch.empty((N, Nc, Ho, Wo), dtype=x.dtype, device=x.device,
                        memory_format=torch.channels_last)
        part = torch.empty(_part_floats(N * Ho * Wo, Nc), dtype=torch.float32, device=x.device)
        rows = C_.conv_f32_fwd_s2(_ptr(x), _ptr(w), _ptr(y), _ptr(ws), ws.numel(), N, H, W, C, Nc,
                                  k, _ptr(part), part.numel(), _stream())
        ctx.save_for_backward(x, w)
        ctx.bn_part = (part, rows) if rows > 0 else None
        return y

    @staticmethod
    def backward(ctx, dy):
        from .nn import materialize

        C_ = require()
        flush_pending()  # a deferred Winograd weight-gradient transform, while its data is warm
        x, w = ctx.saved_tensors
        N, C, H, W = x.shape
        Nc, k = w.shape[0], w.shape[-1]
        if getattr(dy, "_ew_lazy_bwd", None) is not None:
            materialize(dy)
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        if dy.data_ptr() % 16:
            dy = dy.clone(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            C_.conv_f32_bwd_data_s2(_ptr(dy), _ptr(w), _ptr(dx), N, H, W, C, Nc, k, 0, _stream())
        if ctx.needs_input_grad[1]:
            ws = _ws(x.device)
            dw = torch.empty_like(w, memory_format=torch.channels_last)
            C_.conv_f32_wgrad_s2(_ptr(dy), _ptr(x), _ptr(dw), _ptr(ws), ws.numel(), N, H, W, C,
                                 Nc, k, _stream())
        return dx, dw


def conv_s2(x, w):
    """``F.conv2d(x, w, stride=2, padding=k // 2)`` (k = 3 or 1) through the fp32 stride-2
    kernels when :func:`s2_supported`, else MIOpen."""
    from .nn import materialize

    x = materialize(x)
    if s2_supported(x, w):
        y = _ConvS2.apply(x, w)
        node = y.grad_fn
        part = getattr(node, "bn_part", None) if node is not None else None
        if part is not None:
            y._ew_bn_part = part
        return y
    return F.conv2d(x, w, stride=2, padding=w.shape[-1] // 2)


SINK_ADDS = 0  # backward-data launches that added a sink's gradient (tests)


class GradSink:
    """Hand-over slot for a second gradient of a conv's input (``grad``: set by the producer's
    backward, consumed and cleared by the conv's backward-data launch; ``taken``: that launch has
    run, so a later producer must hand its gradient to autograd instead)."""

    __slots__ = ("grad", "taken")

    def __init__(self):
        self.grad = None
        self.taken = False


class _SinkTap(torch.autograd.Function):
    """Identity on ``x`` whose backward deposits the incoming gradient in ``sink`` (returning
    none to autograd) while the sink's conv has not run its backward yet.  ResNet projection
    shortcuts read the block input through it: the shortcut branch is recorded after the main
    branch, so autograd runs its backward first and the block's first conv adds its input
    gradient in the backward-data epilogue (models/resnet.py)."""

    @staticmethod
    def forward(ctx, x, sink):
        ctx.sink = sink
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        sink, ctx.sink = ctx.sink, None
        if sink is None or sink.taken:
            return g, None
        sink.grad = g
        return None, None


def sink_tap(x, sink):
    """``x`` for a second consumer whose input gradient goes to ``sink`` (:class:`_SinkTap`)."""
    return _SinkTap.apply(x, sink)


def _apply(x, w, sink=None):
    if x.shape[1] == 3:
        y = _ConvStem.apply(x, w)
        if y.dtype == torch.float32 and y.grad_fn is not None:
            y._ew_stem_out = True  # its BN layer may leave the backward apply to the stem
    else:
        node = getattr(x, "_ew_bn_node", None) if (_BN_BWD and epilogue_fusion_ok(x)) else None
        y = _Conv.apply(x, w, node, sink)
    # hand the epilogue's BatchNorm partials to the consumer (bn_act reads ``_ew_bn_part``)
    node = y.grad_fn  # the autograd ctx of _Conv / _ConvStem (None under no_grad)
    wp = getattr(node, "w_param", None) if node is not None else None
    if wp is not None:
        # a weight used twice in one pass (tied weights) gets its dw summed with the other use's
        # in autograd's input buffer before any hook runs: never deferred (_can_defer).  Only
        # forwards that record autograd history count (node is None under no_grad): an eval or
        # best-worker scoring forward in the same step is no second use.
        if getattr(wp, "_ew_use_epoch", None) == _USE_EPOCH[0]:
            wp._ew_tied = True
        wp._ew_use_epoch = _USE_EPOCH[0]
    part = getattr(node, "bn_part", None) if node is not None else None
    if part is not None:
        y._ew_bn_part = part
    if node is not None and ((_WINO_LAZY_BWD and getattr(node, "wino", None) is not None)
                             or (_SM_LAZY_BWD and getattr(node, "sm", None) is not None)):
        y._ew_wino_out = True  # the BN layer it feeds may leave its backward apply to us
    return y


def conv(x, w):
    """``F.conv2d(x, w, padding=k // 2)`` (k = 3 or 1) through the MFMA kernels when
    :func:`supported`."""
    if supported(x, w):
        return _apply(x, w)
    from .nn import materialize

    return F.conv2d(materialize(x), w, padding=w.shape[-1] // 2)


conv3x3 = conv


def module_supported(m, x) -> bool:
    """True if :func:`conv2d_module` runs ``m`` on the MFMA kernels (not the stem)."""
    return (m.bias is None and m.padding_mode == "zeros" and x.shape[1] != 3
            and supported(x, m.weight, m.stride, m.padding, m.dilation, m.groups))


def conv2d_module(m, x, sink=None):
    """``m(x)`` for an ``nn.Conv2d`` ``m`` without bias, through the MFMA kernels when the layer
    is a stride-1 3x3/pad-1 or 1x1/pad-0 convolution on channels_last bf16/fp32 (else ``m(x)``).
    ``sink`` (:class:`GradSink`, MFMA path only): a second gradient of ``x`` deposited there
    before this conv's backward is added to its input gradient."""
    if (m.bias is None and m.padding_mode == "zeros"
            and supported(x, m.weight, m.stride, m.padding, m.dilation, m.groups)):
        return _apply(x, m.weight, sink)
    if sink is not None:
        raise ValueError("a gradient sink needs the MFMA conv path")
    if (_S2 and m.bias is None and m.padding_mode == "zeros" and x.is_cuda
            and s2_supported(x, m.weight, m.stride, m.padding, m.dilation, m.groups)):
        return conv_s2(x, m.weight)
    from .nn import materialize

    return m(materialize(x))  # a lazily applied BN output is written before a foreign kernel
