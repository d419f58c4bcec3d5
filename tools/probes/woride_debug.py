"""Debug: does the deferred Winograd transform reach the direct conv's backward-data launch?"""
import torch

from ewdml import ops
from ewdml.ops import conv

ops.require()
conv.set_enabled(True)
conv.set_winograd(True, 128, "2")
N, H = 128, 16
w0 = torch.nn.Parameter(torch.randn(128, 64, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last) / 24)
w1 = torch.nn.Parameter(torch.randn(128, 128, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last) / 34)
for w in (w0, w1):
    w._ew_engine_hooks = 1
    w.register_post_accumulate_grad_hook(lambda p: None)
x = torch.randn(N, 64, H, H, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(True)
dy = torch.randn(N, 128, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
orig_take = conv._take_pending


def take(m):
    print("take_pending m", m, "pending", None if conv._PENDING is None else conv._PENDING[5], flush=True)
    r = orig_take(m)
    print(" ->", r[0], r[1] is not None, flush=True)
    return r


conv._take_pending = take
orig_can = conv._can_defer


def can(ctx):
    r = orig_can(ctx)
    print("can_defer", r, flush=True)
    return r


conv._can_defer = can
h = conv.conv(x, w0)
conv.conv(h, w1).backward(dy)
torch.cuda.synchronize()
print("rides", conv.WO_RIDES, flush=True)
