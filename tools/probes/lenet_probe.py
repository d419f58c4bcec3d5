"""Standalone timing of the fused LeNet kernels (ops/csrc/lenet_f32.hip): the forward pair and the
backward pair of launches at several batches, captured in a HIP graph (20 launches per replay) so
the host does not bound the measurement; us per call.  EWDML_LN_PART=1 / 2 restricts the
conv-backward launch to one of its two block sets."""
import os
import sys

import torch

sys.path.insert(0, ".")
from ewdml import ops  # noqa: E402
from ewdml.models.lenet import LeNet  # noqa: E402
from ewdml.ops import _ptr, lenet  # noqa: E402

C_ = ops.require()


def graphed(fn, reps=20, it=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (it * reps)


for B in (16, 32, 64, 128):
    torch.manual_seed(0)
    m = LeNet().cuda()
    x = torch.randn(B, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    K = 10
    f = dict(dtype=torch.float32, device="cuda")
    a1, a2 = torch.empty(B, 2880, **f), torch.empty(B, 800, **f)
    c1 = torch.empty(B, 2880, dtype=torch.uint8, device="cuda")
    c2 = torch.empty(B, 800, dtype=torch.uint8, device="cuda")
    h1, dh1, dp2 = torch.empty(B, 500, **f), torch.empty(B, 500, **f), torch.empty(B, 800, **f)
    lg, dlg, lr, loss = torch.empty(B, K, **f), torch.empty(B, K, **f), torch.empty(B, **f), torch.empty((), **f)
    g1 = torch.ones((), **f)
    ps = lenet._params(m)
    grads = [torch.empty_like(p) for p in ps]
    ws, cnt = lenet._ws(x.device, B)
    P = [_ptr(p) for p in ps]

    def fwd():
        C_.lenet_fwd(_ptr(x), *P, _ptr(y), B, K, _ptr(a1), _ptr(c1), _ptr(a2), _ptr(c2), _ptr(h1),
                     _ptr(lg), _ptr(dlg), _ptr(dh1), _ptr(lr), _ptr(loss), _ptr(ws), ws.numel(),
                     _ptr(cnt), cnt.numel(), torch.cuda.current_stream().cuda_stream)

    def bwd():
        C_.lenet_bwd(_ptr(x), P[2], P[4], _ptr(a1), _ptr(c1), _ptr(a2), _ptr(c2), _ptr(h1),
                     _ptr(dlg), _ptr(dh1), _ptr(g1), B, K, _ptr(dp2), *[_ptr(t) for t in grads],
                     _ptr(ws), ws.numel(), _ptr(cnt), cnt.numel(),
                     torch.cuda.current_stream().cuda_stream)

    fwd()
    tf, tb = graphed(fwd), graphed(bwd)
    print(f"B {B:4d}  part {os.environ.get('EWDML_LN_PART', '0')}  fwd pair {tf:7.1f} us  "
          f"bwd pair {tb:7.1f} us", flush=True)

# phase stamps of one conv-backward launch (B = 64): wall_clock64 ticks (100 MHz) per block
if os.environ.get("EWDML_LN_PART", "0") == "0":
    B = 64
    torch.manual_seed(0)
    m = LeNet().cuda()
    x = torch.randn(B, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    for _ in range(3):
        loss, _ = m.fused_loss(x, y)
        loss.backward()
    torch.cuda.synchronize()
    nblk = 4 * B + 10 * ((B + 1) // 2)
    buf = torch.zeros(nblk, 8, dtype=torch.int64, device="cuda")
    C_.lenet_set_prof(_ptr(buf))
    loss, _ = m.fused_loss(x, y)
    loss.backward()
    torch.cuda.synchronize()
    C_.lenet_set_prof(0)
    st = buf.cpu()
    t0 = int(st[:, 0][st[:, 0] > 0].min())
    na = 4 * B

    def show(name, rows, names):
        import statistics as S
        print(f"{name}: {rows.shape[0]} blocks; start spread {(int(rows[:, 0].max()) - int(rows[:, 0].min())) / 100:.2f} us")
        for i in range(1, len(names)):
            d = [(int(r[i]) - int(r[i - 1])) / 100 for r in rows if r[i] > 0 and r[i - 1] > 0]
            if d:
                print(f"  {names[i - 1]:>10} -> {names[i]:<10} n {len(d):4d}  median {S.median(d):7.2f} us  max {max(d):7.2f} us")
        end = max(int(v) for v in rows.flatten() if v > 0)
        print(f"  last stamp at {(end - t0) / 100:.2f} us after the first block start")

    show("part A", st[:na], ["start", "staged", "gathered", "partial", "ticket1", "level1", "ticket2", "end"])
    show("part B", st[na:], ["start", "staged", "computed", "ticket", "end"])
