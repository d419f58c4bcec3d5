"""sm_f32_bwd with dy formed in-kernel (KIND 2, pooled / not) against dy formed by torch."""
import sys

import torch

sys.path.insert(0, ".")
from ewdml import ops  # noqa: E402
from ewdml.ops import conv  # noqa: E402

C_ = ops.require()
torch.manual_seed(0)
N, C, Nc = 64, 128, 128
cl = torch.channels_last
x = torch.randn(N, C, 2, 2, device="cuda").contiguous(memory_format=cl)
w = (torch.randn(Nc, C, 3, 3, device="cuda") / 34).contiguous(memory_format=cl)
h = torch.randn(N, Nc, 2, 2, device="cuda").contiguous(memory_format=cl)
mean = torch.randn(Nc, device="cuda") * 0.1
sc = torch.rand(Nc, device="cuda") + 0.5
sh = torch.randn(Nc, device="cuda") * 0.1
stats = torch.cat([mean, torch.ones(Nc, device="cuda"), sc, sh]).contiguous()
coef = (torch.randn(2 * Nc, device="cuda") * 0.01).contiguous()
s = torch.cuda.current_stream().cuda_stream
slab, cnt = conv._sm_ws(x.device, N, C, Nc)
for pool, cfill in ((True, None), (True, 0), (True, 1), (True, 2), (True, 3), (False, None)):
    if pool:
        dn = torch.randn(N, Nc, 1, 1, device="cuda").contiguous(memory_format=cl)
        code = torch.randint(0, 4, (N, 1, 1, Nc), device="cuda", dtype=torch.uint8)
        if cfill is not None:
            code.fill_(cfill)
        # dz at 2x2 position p = (code == p) * dn
        hh = h.permute(0, 2, 3, 1).reshape(N, 4, Nc)
        routed = torch.stack([(code.reshape(N, Nc) == p).float() * dn.reshape(N, Nc)
                              for p in range(4)], 1)
    else:
        dn = torch.randn(N, Nc, 2, 2, device="cuda").contiguous(memory_format=cl)
        code = None
        hh = h.permute(0, 2, 3, 1).reshape(N, 4, Nc)
        routed = dn.permute(0, 2, 3, 1).reshape(N, 4, Nc)
    z = hh * sc + sh
    dz = torch.where(z <= 0, torch.zeros_like(routed), routed)
    dyv = sc * dz + coef[:Nc] * (hh - mean) + coef[Nc:]
    dy = dyv.reshape(N, 2, 2, Nc).permute(0, 3, 1, 2).contiguous(memory_format=cl)
    outs = []
    for kind in (2, 0):
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        C_.sm_f32_bwd(x.data_ptr(), 0, 0, dy.data_ptr() if kind == 0 else 0,
                      h.data_ptr() if kind == 2 else 0, dn.data_ptr() if kind == 2 else 0,
                      code.data_ptr() if (kind == 2 and pool) else 0,
                      stats.data_ptr() if kind == 2 else 0, coef.data_ptr() if kind == 2 else 0,
                      int(pool), w.data_ptr(), dx.data_ptr(), dw.data_ptr(), slab.data_ptr(),
                      slab.numel(), cnt.data_ptr(), cnt.numel(), N, C, Nc, 0, 0, 0, 0, 0, 0, 0, s)
        torch.cuda.synchronize()
        outs.append((dx, dw))
    (dx2, dw2), (dx0, dw0) = outs
    rel = lambda a, b: float((a - b).norm() / b.norm())  # noqa: E731
    print(f"pool={pool} code={cfill}: dx rel {rel(dx2, dx0):.3e} equal {torch.equal(dx2, dx0)}; "
          f"dw rel {rel(dw2, dw0):.3e} equal {torch.equal(dw2, dw0)}")
