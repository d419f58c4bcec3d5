"""Which gradients of conv -> BN -> 2x2 conv -> BN(-pool) differ between lazy and materialised BN,
and which side is closer to float64."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from ewdml import ops  # noqa: E402
from ewdml.ops import conv, nn as fnn  # noqa: E402

ops.require()
conv.set_enabled(True)
conv.set_winograd(True, 64, 2)
conv.set_smallmap(True)
pool = len(sys.argv) < 2 or sys.argv[1] == "pool"
N, C = 64, 128
g0 = torch.Generator(device="cuda").manual_seed(61)
x0 = torch.randn(N, C, 2, 2, device="cuda", generator=g0).contiguous(memory_format=torch.channels_last)
w0 = (torch.randn(C, C, 3, 3, device="cuda", generator=g0) / 34).contiguous(memory_format=torch.channels_last)
w1 = (torch.randn(C, C, 3, 3, device="cuda", generator=g0) / 34).contiguous(memory_format=torch.channels_last)
bns = [torch.nn.BatchNorm2d(C).cuda() for _ in range(2)]
with torch.no_grad():
    for bn in bns:
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
gshape = (N, C, 1, 1) if pool else (N, C, 2, 2)
g = torch.randn(gshape, device="cuda").contiguous(memory_format=torch.channels_last)
names = ["out", "x.grad", "w0.grad", "w1.grad", "bnA.w", "bnA.b", "bnB.w", "bnB.b"]
runs = []
for lazy in (True, False, True, True):
    fnn._LAZY_BWD = lazy
    b0, b1 = copy.deepcopy(bns[0]), copy.deepcopy(bns[1])
    xa, wa, wb = (t.clone().requires_grad_(True) for t in (x0, w0, w1))
    h = conv.conv(xa, wa)
    y = fnn.bn_relu(h, None, b0, pool=False, lazy=lazy)
    z = conv.conv(y, wb)
    out = fnn.bn_act(z, b1, "relu", pool=pool)
    out.backward(g)
    torch.cuda.synchronize()
    runs.append([out, xa.grad, wa.grad, wb.grad, b0.weight.grad, b0.bias.grad, b1.weight.grad,
                 b1.bias.grad])
# float64 reference on the CPU
xr, w0r, w1r = (t.detach().double().cpu().requires_grad_(True) for t in (x0, w0, w1))
b0r, b1r = copy.deepcopy(bns[0]).double().cpu(), copy.deepcopy(bns[1]).double().cpu()
hr = F.conv2d(xr, w0r, padding=1)
yr = F.relu(b0r(hr))
zr = F.conv2d(yr, w1r, padding=1)
outr = F.relu(b1r(zr))
if pool:
    outr = F.max_pool2d(outr, 2, 2)
outr.backward(g.double().cpu())
ref = [outr, xr.grad, w0r.grad, w1r.grad, b0r.weight.grad, b0r.bias.grad, b1r.weight.grad, b1r.bias.grad]


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


print("lazy runs agree:", [all(torch.equal(runs[0][i], runs[k][i]) for i in range(8)) for k in (2, 3)])
for i, n in enumerate(names):
    print(f"{n:8s} equal={torch.equal(runs[0][i], runs[1][i])!s:5s} lazy-vs-fp64 {rel(runs[0][i], ref[i]):.2e}"
          f"  mat-vs-fp64 {rel(runs[1][i], ref[i]):.2e}")
