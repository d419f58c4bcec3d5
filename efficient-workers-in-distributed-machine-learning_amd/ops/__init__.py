"""Python entry points of the hand-written gfx950 kernels (``ops/csrc/*.hip``).

Every wrapper validates shapes/dtypes/alignment on the host (a kernel launched on a bad operand can
fault the whole GPU node), then launches on torch's *current* HIP stream so calls compose with
``torch.cuda.stream(...)`` and are captured by ``torch.cuda.graph``.

These wrappers only accept device tensors.  CPU execution (Gloo tests) goes through the torch
oracle in ``compress/oracle.py``; there is no silent fallback on the GPU: if the extension is not
built, :func:`require` raises.
"""
import importlib
import os

import torch

_IMPORT_ERROR = None
try:  # torch is imported first so the extension binds to torch's already-loaded HIP runtime
    _ALT = os.environ.get("EWDML_EXT")  # A/B of a compile-time variant: another built _C .so
    if _ALT:
        import importlib.util
        import sys as _sys

        _spec = importlib.util.spec_from_file_location(__name__ + "._C", _ALT)
        _C = importlib.util.module_from_spec(_spec)
        _spec.loader.exec_module(_C)
        _sys.modules[__name__ + "._C"] = _C
    else:
        _C = importlib.import_module(__name__ + "._C")
except ImportError as e:  # pragma: no cover - depends on the build
    _C = None
    _IMPORT_ERROR = e

VK_Q8, VK_Q4, VK_F32 = 0, 1, 2

_SYNC_DEBUG = os.environ.get("EWDML_SYNC_DEBUG") == "1"


class _SyncDebug:
    """``--sync-debug`` / EWDML_SYNC_DEBUG=1: synchronise the device after every custom kernel
    launch so a fault, race or bad operand is reported at the launch that caused it."""

    def __init__(self, mod):
        self._m = mod

    def __getattr__(self, name):
        f = getattr(self._m, name)
        if not callable(f):
            return f

        def call(*a, **k):
            r = f(*a, **k)
            if _SYNC_DEBUG:
                torch.cuda.synchronize()
            return r
        return call


def set_sync_debug(on: bool = True):
    global _SYNC_DEBUG
    _SYNC_DEBUG = bool(on)


def available() -> bool:
    return _C is not None


def require():
    if _C is None:
        raise RuntimeError(
            "ewdml HIP extension is not built or failed to load "
            f"({_IMPORT_ERROR}); run `python -m ewdml.ops.build` (or __graft_entry__.build())")
    return _SyncDebug(_C) if _SYNC_DEBUG else _C


def library_path():
    return getattr(_C, "__file__", None)


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def _check(t, dtype, name, align=16, dense=False):
    """``dense``: any non-overlapping dense layout is fine (the kernel reads the tensor in memory
    order, e.g. a channels_last conv-weight gradient matching its channels_last parameter)."""
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not (t.is_contiguous() or (dense and t.dim() == 4
                                  and t.is_contiguous(memory_format=torch.channels_last))):
        raise ValueError(f"{name} must be contiguous")
    if t.data_ptr() % align:
        raise ValueError(f"{name} must be {align}-byte aligned")


class DevicePlan:
    """Device-resident tables + scratch for one bucket (built once, reused every step)."""

    def __init__(self, plan, device):
        self.plan = plan
        self.tensors = plan.tensor_table(device)
        self.chunks = plan.chunk_table(device)
        self.cblocks = plan.cblock_table(device)  # predictive top-k encode's candidate passes
        C, T = plan.num_chunks, plan.num_tensors
        nbytes = max(require().topk_scratch_bytes(T, C, plan.length, plan.total_cap),
                     require().qsgd_scratch_bytes(T, C))
        self.scratch = torch.zeros(nbytes, dtype=torch.uint8, device=device)


# EWDML_TOPK_PREDICT=0: every top-k encode takes the full passes (A/B of the predictive encode)
_TOPK_PREDICT = os.environ.get("EWDML_TOPK_PREDICT", "1") != "0"
_LB_FAULT = [False]


def set_lookback_fault(on: bool):
    """Test hook: the next top-k encodes' first chunks skip their look-back word, so every later
    chunk of a tensor polls to the bound and reports through the error counter."""
    _LB_FAULT[0] = bool(on)


def topk_stats(dp) -> dict:
    """Counters of a bucket's top-k encodes (synchronises): ``lookback_errors`` (write blocks that
    gave up waiting on a predecessor's look-back word: their payload offsets are wrong -- must be
    0), and the tensor-encodes of the predictive encode on the ``fast`` (candidates only) and the
    ``full`` path (``full_by_tensor``: the first 28 tensors' share of the latter, as [too few
    candidates, too many] pairs)."""
    v = require().topk_stats(_ptr(dp.scratch), dp.plan.num_tensors, dp.plan.num_chunks)
    e, fast, full = v[:3]
    return {"lookback_errors": e, "fast": fast, "full": full,
            "full_by_tensor": [[x & 0xFFFF, x >> 16] for x in v[3:3 + dp.plan.num_tensors]]}


_GRAPH_NODE_TYPES = ["kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event",
                     "event_record", "ext_semas_signal", "ext_semas_wait", "mem_alloc", "mem_free",
                     "memcpy_from_symbol", "memcpy_to_symbol", "batch_mem_op", "t15"]


def graph_info(graph, dot_path: str = "") -> dict:
    """Node / edge counts of a captured graph kept with ``torch.cuda.CUDAGraph(keep_graph=True)``
    (``raw_cuda_graph()``): a straight line has no forks or joins and one root."""
    v = require().graph_info(int(graph), dot_path)
    types = {_GRAPH_NODE_TYPES[i]: int(c) for i, c in enumerate(v[5:]) if c}
    return {"nodes": v[0], "edges": v[1], "forks": v[2], "joins": v[3], "roots": v[4],
            "linear": v[2] == 0 and v[3] == 0 and v[4] <= 1, "types": types}


def topk_lookback_errors(dp) -> int:
    """Times a top-k write block gave up waiting on a predecessor's look-back word (bounded spin;
    0 unless something is badly wrong).  Synchronises."""
    return require().topk_lookback_errors(_ptr(dp.scratch), dp.plan.num_tensors,
                                          dp.plan.num_chunks)


def _check_bucket(dp, grad, name="grad"):
    _check(grad, torch.float32, name)
    if grad.numel() < dp.plan.length:
        raise ValueError(f"{name} has {grad.numel()} elements, bucket needs {dp.plan.length}")


MAX_TENSORS_PER_BUCKET = 128  # EW_MAX_T in csrc/common.h


def grad_pointers(dp, grad):
    """(pointers, bf16 bit mask) of a bucket's per-tensor gradients.  ``grad`` is the bucket's
    flat fp32 view (tensors at the plan offsets) or a list with one fp32/bf16 tensor per plan
    tensor (autograd's own ``p.grad`` tensors, read in place)."""
    plan = dp.plan
    if plan.num_tensors > MAX_TENSORS_PER_BUCKET:
        raise ValueError(f"bucket has {plan.num_tensors} tensors (max {MAX_TENSORS_PER_BUCKET})")
    mask = [0] * (MAX_TENSORS_PER_BUCKET // 32)
    if torch.is_tensor(grad):
        _check_bucket(dp, grad)
        base = grad.data_ptr()
        return [base + 4 * o for o in plan.offsets], mask
    if len(grad) != plan.num_tensors:
        raise ValueError(f"{len(grad)} gradients for a bucket of {plan.num_tensors} tensors")
    ptrs = []
    for i, (t, n) in enumerate(zip(grad, plan.numels)):
        if t.dtype == torch.bfloat16:
            _check(t, torch.bfloat16, "grad tensor", align=8, dense=True)
            mask[i >> 5] |= 1 << (i & 31)
        else:
            _check(t, torch.float32, "grad tensor", dense=True)
        if t.numel() != n:
            raise ValueError(f"gradient has {t.numel()} elements, plan expects {n}")
        ptrs.append(t.data_ptr())
    return ptrs, mask


def _check_shadow(dp, shadow):
    if shadow is not None:
        _check(shadow, torch.bfloat16, "shadow", align=8)
        if shadow.numel() < dp.plan.length:
            raise ValueError("shadow too small for the bucket")


def _keyp(key_tensor):
    if key_tensor is None:
        return 0
    if not key_tensor.is_cuda or key_tensor.dtype != torch.int32 or key_tensor.numel() < 1:
        raise ValueError("key_tensor must be a device int32 tensor")
    return key_tensor.data_ptr()


def topk_encode(dp: DevicePlan, grad, payload, layout, levels: int, norm: str, key: int,
                resid=None, key_tensor=None, dgc=None, apply=None):
    """``dgc``: momentum-corrected error feedback, ``{velocity, momentum, dampening, nesterov,
    weight_decay, param}`` (bucket views; compress/oracle.py dgc_accumulate).

    ``apply`` (a world of one, where the all-gathered payload is this rank's own): the write pass
    also applies the update ``topk_decode_apply`` would with no momentum buffer --
    ``{param, lr, lr_tensor, grad_scale, shadow, key_state, key_seed, key_rank}``: at each sent
    coordinate p -= lr * grad_scale * sent (and the bf16 shadow), then the RNG key state moves to
    the next step; bitwise the decode's result (tests/kernels/test_hip_codecs.py)."""
    C = require()
    ptrs, mask = grad_pointers(dp, grad)
    _check(payload, torch.uint8, "payload")
    if payload.numel() < layout.nbytes:
        raise ValueError("payload too small")
    if resid is not None:
        _check_bucket(dp, resid, "resid")
    if layout.kind == "topk":
        vk = VK_F32
    elif layout.bits == 8:
        vk = VK_Q8
    else:
        vk = VK_Q4
    if vk != VK_F32 and not (1 <= levels <= (127 if layout.bits == 8 else 7)):
        raise ValueError(f"levels={levels} does not fit {layout.bits}-bit codes")
    vel = par = lrt = None
    mom = damp1 = wd = 0.0
    nest, dmask = 0, 1
    if dgc is not None:
        if resid is None:
            raise ValueError("momentum correction needs the residual")
        vel, mom = dgc["velocity"], float(dgc["momentum"])
        _check_bucket(dp, vel, "velocity")
        damp1 = float(1.0 - dgc.get("dampening", 0.0))
        wd = float(dgc.get("weight_decay", 0.0))
        nest = int(bool(dgc.get("nesterov", False)))
        dmask = int(bool(dgc.get("mask", True)))
        if dgc.get("lr") is not None:  # error feedback on the update: the lr inside
            lrt = dgc.get("lr_t")
            if lrt is None:
                raise ValueError("lr-scaled accumulation on the GPU needs the device lr (lr_t)")
        if wd != 0.0:
            par = dgc["param"]
            _check_bucket(dp, par, "param")
    C.topk_encode(ptrs, mask, _ptr(resid), _ptr(dp.chunks), _ptr(dp.tensors), _ptr(dp.scratch),
                  _ptr(payload), layout.nbytes, dp.plan.num_tensors, dp.plan.num_chunks,
                  layout.scales, layout.counts, layout.idx, layout.codes, vk,
                  1 if norm == "l2" else 0, float(levels), float(1.0 / levels), key & 0xFFFFFFFF,
                  dp.plan.bucket_offset & 0xFFFFFFFF, _keyp(key_tensor), _stream(), _ptr(vel),
                  _ptr(par), mom, damp1, wd, nest, layout.bitmap, dmask, _lrp(lrt), dp.plan.length,
                  _ptr(dp.cblocks), dp.plan.num_cblocks, int(_TOPK_PREDICT), int(_LB_FAULT[0]),
                  int(max(dp.plan.ks)) if dp.plan.ks else 0, *_apply_args(dp, apply, norm),
                  _stamps_ptr(dp, dgc))


def _stamps_ptr(dp, dgc):
    """The producer-staging stamp words of a momentum-corrected encode (``dgc["stamps"]``:
    int32 [T] device tensor, 1 = that tensor's producer already staged it this step)."""
    st = None if dgc is None else dgc.get("stamps")
    if st is None:
        return 0
    _check(st, torch.int32, "stamps", align=4)
    if st.numel() < dp.plan.num_tensors:
        raise ValueError("one stamp word per tensor of the bucket")
    return st.data_ptr()


def topk_one_launch(dp) -> bool:
    """Whether this bucket's top-k encode runs as the one-launch kernel (k_pk_one: every chunk
    block resident)."""
    return _TOPK_PREDICT and dp.plan.num_chunks <= require().topk_one_max_blocks()


def _apply_args(dp, apply, norm):
    if apply is None:
        return (0, 0, 0.0, 0, 1.0, 0, 0, 0, 0, 0, 0.0, 0.0, 0.0, 0, 0)
    if not _TOPK_PREDICT or norm != "max":
        raise ValueError("the write-pass apply needs the predictive (max-norm) encode")
    param = apply["param"]
    _check_bucket(dp, param, "param")
    _check_shadow(dp, apply.get("shadow"))
    ks = apply.get("key_state")
    if ks is not None:
        _check(ks, torch.int32, "key_state", align=4)
    dense = "mom" in apply  # receiver-side momentum SGD over every element (one-launch only)
    mom = apply.get("mom")
    if dense:
        if mom is None or not topk_one_launch(dp):
            raise ValueError("the dense write-pass apply needs the momentum buffer and the "
                             "one-launch encode")
        _check_bucket(dp, mom, "mom")
    return (_ptr(param), _ptr(apply.get("shadow")), float(apply["lr"]),
            _lrp(apply.get("lr_tensor")), float(apply.get("grad_scale", 1.0)), _ptr(ks),
            int(apply.get("key_seed", 0)) & 0xFFFFFFFF, int(apply.get("key_rank", 0)) & 0xFFFFFFFF,
            int(dense), _ptr(mom), float(apply.get("momentum", 0.0)),
            float(apply.get("dampening", 0.0)), float(apply.get("weight_decay", 0.0)),
            int(bool(apply.get("nesterov", False))), int(bool(apply.get("first", False))))


def _lrp(lr_tensor):
    """Device fp32 learning rate read by the kernels at run time (None: the ``lr`` argument)."""
    if lr_tensor is None:
        return 0
    if not lr_tensor.is_cuda or lr_tensor.dtype != torch.float32 or lr_tensor.numel() < 1:
        raise ValueError("lr_tensor must be a device fp32 tensor")
    return lr_tensor.data_ptr()


def topk_decode_apply(dp: DevicePlan, recv, layout, levels: int, param=None, mom=None,
                      grad_out=None, lr=0.0, momentum=0.0, dampening=0.0, weight_decay=0.0,
                      grad_scale=1.0, nesterov=False, first=False, shadow=None,
                      key_state=None, key_seed=0, key_rank=0, lr_tensor=None):
    C = require()
    _check(recv, torch.uint8, "recv")
    if recv.dim() != 2 or recv.shape[1] != layout.nbytes:
        raise ValueError(f"recv must be [nranks, {layout.nbytes}]")
    if recv.shape[0] > 64:
        raise ValueError("at most 64 ranks per decode")
    apply = param is not None
    if apply:
        _check_bucket(dp, param, "param")
        if mom is not None:
            _check_bucket(dp, mom, "mom")
        elif momentum != 0.0 or nesterov:
            raise ValueError("a momentum step needs the momentum buffer")
    if grad_out is not None:
        _check_bucket(dp, grad_out, "grad_out")
    if not apply and grad_out is None:
        raise ValueError("nothing to do: pass param/mom and/or grad_out")
    _check_shadow(dp, shadow)
    vk = VK_F32 if layout.kind == "topk" else (VK_Q8 if layout.bits == 8 else VK_Q4)
    C.topk_decode_apply(_ptr(recv), recv.shape[0], layout.nbytes, _ptr(dp.chunks),
                        _ptr(dp.tensors), dp.plan.num_chunks, layout.scales, layout.counts,
                        layout.idx, layout.codes, vk, float(1.0 / levels), _ptr(param), _ptr(mom),
                        _ptr(grad_out), _ptr(shadow), lr, momentum, dampening, weight_decay,
                        grad_scale, int(nesterov), int(first), int(apply), _stream(),
                        _keyp(key_state), key_seed & 0xFFFFFFFF, key_rank & 0xFFFFFFFF,
                        layout.bitmap, _lrp(lr_tensor))


def qsgd_encode(dp: DevicePlan, grad, payload, layout, levels: int, norm: str, key: int,
                resid=None, key_tensor=None):
    C = require()
    ptrs, mask = grad_pointers(dp, grad)
    _check(payload, torch.uint8, "payload")
    if payload.numel() < layout.nbytes:
        raise ValueError("payload too small")
    if resid is not None:
        _check_bucket(dp, resid, "resid")
    if not (1 <= levels <= (127 if layout.bits == 8 else 7)):
        raise ValueError(f"levels={levels} does not fit {layout.bits}-bit codes")
    C.qsgd_encode(ptrs, mask, _ptr(resid), _ptr(dp.chunks), _ptr(dp.tensors), _ptr(dp.scratch),
                  _ptr(payload), layout.nbytes, dp.plan.num_tensors, dp.plan.num_chunks,
                  layout.scales, layout.codes, layout.bits, 1 if norm == "l2" else 0,
                  float(levels), float(1.0 / levels), key & 0xFFFFFFFF,
                  dp.plan.bucket_offset & 0xFFFFFFFF, _keyp(key_tensor), _stream())


def qsgd_decode_apply(dp: DevicePlan, recv, layout, levels: int, param=None, mom=None,
                      grad_out=None, lr=0.0, momentum=0.0, dampening=0.0, weight_decay=0.0,
                      grad_scale=1.0, nesterov=False, first=False, shadow=None,
                      key_state=None, key_seed=0, key_rank=0, lr_tensor=None):
    C = require()
    _check(recv, torch.uint8, "recv")
    if recv.dim() != 2 or recv.shape[1] != layout.nbytes:
        raise ValueError(f"recv must be [nranks, {layout.nbytes}]")
    apply = param is not None
    if apply:
        _check_bucket(dp, param, "param")
        _check_bucket(dp, mom, "mom")
    if grad_out is not None:
        _check_bucket(dp, grad_out, "grad_out")
    if not apply and grad_out is None:
        raise ValueError("nothing to do: pass param/mom and/or grad_out")
    _check_shadow(dp, shadow)
    C.qsgd_decode_apply(_ptr(recv), recv.shape[0], layout.nbytes, _ptr(dp.chunks),
                        _ptr(dp.tensors), dp.plan.num_chunks, layout.scales, layout.codes,
                        layout.bits, float(1.0 / levels), _ptr(param), _ptr(mom), _ptr(grad_out),
                        _ptr(shadow), lr, momentum, dampening, weight_decay, grad_scale,
                        int(nesterov), int(first), int(apply), _stream(), _keyp(key_state),
                        key_seed & 0xFFFFFFFF, key_rank & 0xFFFFFFFF, _lrp(lr_tensor))


_GDT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def sgd_flat(param, mom, grad, lr, momentum=0.0, dampening=0.0, weight_decay=0.0,
             grad_scale=1.0, nesterov=False, first=False, shadow=None, lr_tensor=None):
    C = require()
    _check(param, torch.float32, "param")
    _check(mom, torch.float32, "mom")
    if grad.dtype not in _GDT:
        raise TypeError(f"unsupported grad dtype {grad.dtype}")
    _check(grad, grad.dtype, "grad", align=8)
    n = param.numel()
    if mom.numel() != n or grad.numel() != n or n % 4:
        raise ValueError("param/mom/grad must have equal numel, a multiple of 4")
    if shadow is not None:
        _check(shadow, torch.bfloat16, "shadow", align=8)
        if shadow.numel() != n:
            raise ValueError("shadow must match param")
    C.sgd_flat(_ptr(param), _ptr(mom), _ptr(grad), _ptr(shadow), n, _GDT[grad.dtype], lr,
               momentum, dampening, weight_decay, grad_scale, int(nesterov), int(first),
               _stream(), _lrp(lr_tensor))


def adam_flat(param, exp_avg, exp_avg_sq, max_exp_avg_sq, grad, lr_step, beta1, beta2, eps,
              weight_decay=0.0, grad_scale=1.0, amsgrad=False, shadow=None, step=None, lr=0.0,
              lr_tensor=None):
    """Adam/AMSGrad over flat fp32 buffers.  ``step`` (int32 device tensor, optional): the kernel
    reads t = step + 1 and derives ``lr_step = lr * sqrt(1 - beta2^t) / (1 - beta1^t)`` on the
    device, so a captured graph follows the step count (``lr_step`` is then ignored)."""
    C = require()
    if step is not None:
        _check(step, torch.int32, "step", align=4)
    for t, nm in ((param, "param"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _check(t, torch.float32, nm)
    if amsgrad:
        _check(max_exp_avg_sq, torch.float32, "max_exp_avg_sq")
    _check(grad, grad.dtype, "grad", align=8)
    n = param.numel()
    if n % 4 or grad.numel() != n or exp_avg.numel() != n or exp_avg_sq.numel() != n:
        raise ValueError("flat buffers must have equal numel, a multiple of 4")
    if shadow is not None:
        _check(shadow, torch.bfloat16, "shadow", align=8)
        if shadow.numel() != n:
            raise ValueError("shadow must match param")
    C.adam_flat(_ptr(param), _ptr(exp_avg), _ptr(exp_avg_sq), _ptr(max_exp_avg_sq), _ptr(grad),
                _ptr(shadow), n, _GDT[grad.dtype], lr_step, beta1, beta2, eps, weight_decay,
                grad_scale, int(amsgrad), _stream(), _ptr(step), float(lr), _lrp(lr_tensor))


_DDT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def pack_grads(dp, grads, dst, scale=1.0):
    """Gather the bucket's per-tensor gradients into the flat ``dst`` (fp32/bf16/fp16), * scale."""
    C = require()
    ptrs, mask = grad_pointers(dp, grads)
    if dst.dtype not in _DDT:
        raise TypeError("dst must be fp32, bf16 or fp16")
    _check(dst, dst.dtype, "dst", align=8)
    if dst.numel() < dp.plan.length:
        raise ValueError("dst too small for the bucket")
    C.pack_grads(ptrs, mask, dp.plan.num_tensors, _ptr(dp.chunks), dp.plan.num_chunks, _ptr(dst),
                 _DDT[dst.dtype], float(scale), _stream())


def sgd_ptrs(dp, grads, param, mom, lr, momentum=0.0, dampening=0.0, weight_decay=0.0,
             grad_scale=1.0, nesterov=False, first=False, shadow=None, lr_tensor=None):
    """SGD of one bucket (``param`` / ``mom`` / ``shadow``: its flat views) from autograd's
    per-tensor gradients, read in place through the pointer table (one launch)."""
    C = require()
    ptrs, mask = grad_pointers(dp, grads)
    for t, nm in ((param, "param"), (mom, "mom")):
        _check(t, torch.float32, nm)
        if t.numel() < dp.plan.length:
            raise ValueError(f"{nm} too small for the bucket")
    _check_shadow(dp, shadow)
    C.sgd_ptrs(ptrs, mask, dp.plan.num_tensors, _ptr(dp.chunks), dp.plan.num_chunks, _ptr(param),
               _ptr(mom), _ptr(shadow), lr, momentum, dampening, weight_decay, grad_scale,
               int(nesterov), int(first), _stream(), _lrp(lr_tensor))


def cast_scale(src, dst, scale=1.0):
    C = require()
    _check(src, torch.float32, "src")
    if dst.dtype not in (torch.bfloat16, torch.float16):
        raise TypeError("dst must be bf16 or fp16")
    _check(dst, dst.dtype, "dst", align=8)
    if src.numel() != dst.numel() or src.numel() % 4:
        raise ValueError("src/dst must have equal numel, a multiple of 4")
    C.cast_scale(_ptr(src), _ptr(dst), src.numel(), float(scale),
                 int(dst.dtype == torch.bfloat16), _stream())



# int32 words of a grid arrival ticket (common.h ew_grid_last: 8 sub-counters + 1 top, 128 B
# apart); zero-initialised, left zeroed by every launch
TICKET_INTS = 9 * 32


def make_batch(src, labels, perm, state, done, out, out_y, mean, inv_std, pad=4, augment=True,
               seed=0, rank=0):
    """Fused batch construction (``csrc/data.hip``): ``out[b] = normalise(augment(src[perm[pos*B
    + b]]))``, ``out_y[b] = labels[...]`` with ``pos = state[0]`` (advanced by the kernel)."""
    C_ = require()
    B = out.shape[0]
    N, C, H, W = src.shape
    if src.dtype != torch.uint8 or not src.is_contiguous() or not src.is_cuda:
        raise ValueError("src must be a contiguous uint8 device tensor [N, C, H, W]")
    if C > 4 or len(mean) != C or len(inv_std) != C:
        raise ValueError("make_batch supports C <= 4 channels with per-channel mean/std")
    if tuple(out.shape) != (B, C, H, W) or out.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("out must be fp32/bf16 [B, C, H, W]")
    cl = not out.is_contiguous()
    if cl and not out.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("out must be NCHW- or channels_last-contiguous")
    for t, dt, n in ((labels, torch.int64, "labels"), (perm, torch.int64, "perm"),
                     (state, torch.int64, "state"), (out_y, torch.int64, "out_y"),
                     (done, torch.int32, "done")):
        _check(t, dt, n, align=4)
    if done.numel() < TICKET_INTS:
        raise ValueError(f"done must hold TICKET_INTS ({TICKET_INTS}) zeroed int32")
    if state.numel() != 2 or out_y.numel() != B or labels.numel() != N:
        raise ValueError("state must be int64[2], out_y int64[B], labels int64[N]")
    if perm.numel() < B or B * H * W >= 2 ** 31:
        raise ValueError("perm shorter than one batch / batch too large")
    if augment and 2 * pad + 1 > 256:
        raise ValueError("pad too large")
    C_.make_batch(_ptr(src), _ptr(labels), _ptr(perm), perm.numel(), _ptr(state), _ptr(done), _ptr(out),
                  _ptr(out_y), B, C, H, W, int(pad), int(bool(augment)),
                  int(out.dtype == torch.bfloat16), int(cl), int(seed) & 0xFFFFFFFF,
                  int(rank) & 0xFFFFFFFF, [float(v) for v in mean], [float(v) for v in inv_std],
                  _stream())

def flag_signal(flags, i: int):
    """Stream hand-off (``csrc/stream_flag.hip``): bump counter ``i`` of the int32 ``flags`` (one
    128-B line per counter) on the current stream."""
    _check(flags, torch.int32, "flags", align=128)
    if not 0 <= i < flags.numel() // 32:
        raise ValueError("flag index out of range")
    require().flag_signal(flags.data_ptr() + 128 * i, _stream())


def flag_wait(flags, i: int, seen: int, need: int, err: int):
    """Wait on the current stream until counter ``i`` of ``flags`` has moved ``need`` more times
    than this wait's private ``seen`` counter (also a line of ``flags``) recorded; ``err``: the
    line counting a poll bound reached."""
    _check(flags, torch.int32, "flags", align=128)
    n = flags.numel() // 32
    if not all(0 <= j < n for j in (i, seen, err)) or need < 1:
        raise ValueError("flag index out of range")
    b = flags.data_ptr()
    require().flag_wait(b + 128 * i, b + 128 * seen, int(need), b + 128 * err, _stream())


def build(force: bool = False) -> str:
    from .build import build as _b
    return _b(force=force)


def hip_required() -> bool:
    """True when running on a GPU box where the HIP path must be used (fail loudly otherwise)."""
    return torch.cuda.is_available() and os.environ.get("EWDML_ALLOW_NO_EXT") != "1"
