"""Standalone timing of the 2x2-map conv kernels (ops/csrc/smallmap_f32.hip) on VGG-11's conv7 /
conv8 shape (N 128, 512 -> 512, 2x2) against the Winograd path: forward, and forward + backward
through autograd, us per call (CUDA events over 50 warm iterations)."""
import sys

import torch

sys.path.insert(0, ".")
from ewdml import ops  # noqa: E402
from ewdml.ops import conv  # noqa: E402

C_ = ops.require()
conv.set_enabled(True)
conv.set_winograd(True, 128, 2)
N, C, Nc = 128, 512, 512
x = torch.randn(N, C, 2, 2, device="cuda").contiguous(memory_format=torch.channels_last)
w = (torch.randn(Nc, C, 3, 3, device="cuda") / 48).contiguous(memory_format=torch.channels_last)
dy = torch.randn(N, Nc, 2, 2, device="cuda").contiguous(memory_format=torch.channels_last)


def timed(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / it


y = torch.empty_like(dy)
slab, cnt = conv._sm_ws(x.device, N, C, Nc)
part = torch.empty(2 * 8 * Nc, device="cuda")
dx = torch.empty_like(x)
dw = torch.empty_like(w)


def fwd():
    C_.sm_f32_fwd(x.data_ptr(), 0, 0, 0, w.data_ptr(), y.data_ptr(), slab.data_ptr(), slab.numel(),
                  cnt.data_ptr(), cnt.numel(), N, C, Nc, part.data_ptr(), part.numel(),
                  torch.cuda.current_stream().cuda_stream)


def bwd(want_dx=True, want_dw=True):
    C_.sm_f32_bwd(x.data_ptr(), 0, 0, dy.data_ptr(), 0, 0, 0, 0, 0, 0, w.data_ptr(),
                  dx.data_ptr() if want_dx else 0, dw.data_ptr() if want_dw else 0,
                  slab.data_ptr(), slab.numel(), cnt.data_ptr(), cnt.numel(), N, C, Nc,
                  0, 0, 0, 0, 0, 0, 0, torch.cuda.current_stream().cuda_stream)


print(f"sm fwd            {timed(fwd):7.1f} us  ({2 * N * 4 * Nc * 4 * C / timed(fwd) / 1e6:.1f} TF/s)")
print(f"sm bwd data       {timed(lambda: bwd(True, False)):7.1f} us")
print(f"sm bwd wgrad      {timed(lambda: bwd(False, True)):7.1f} us")
print(f"sm bwd both       {timed(bwd):7.1f} us")
for sm in (True, False):
    conv.set_smallmap(sm)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)

    def fb():
        conv.conv(xa, wa).backward(dy)

    with torch.no_grad():
        tf = timed(lambda: conv.conv(x, w))
    print(f"{'sm  ' if sm else 'wino'} autograd fwd {tf:7.1f} us   fwd+bwd {timed(fb):7.1f} us")
