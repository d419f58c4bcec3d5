"""Diagnose fp32 step accuracy of the fused path per configuration against a float64 CPU step.

    python tools/debug_f32_step.py [net]
"""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch
import torch.nn.functional as F

import ewdml  # noqa: F401
from ewdml.models import build_model, resnet
from ewdml.ops import conv


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def main():
    net = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
    torch.manual_seed(0)
    m0 = build_model(net, 10).to(memory_format=torch.channels_last)
    for mod in m0.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    x = torch.randn(32, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,))
    m64 = copy.deepcopy(m0).double()
    out64 = m64(x.double())
    F.cross_entropy(out64, y).backward()
    names = [n for n, _ in m64.named_parameters()]
    g64 = [p.grad for p in m64.parameters()]
    for label, on, sink, fuse in (("hip sink+fuse", True, True, True),
                                  ("hip nosink fuse", True, False, True),
                                  ("hip sink nofuse", True, True, False),
                                  ("hip nosink nofuse", True, False, False),
                                  ("miopen", False, False, False)):
        m = copy.deepcopy(m0).cuda()
        conv.set_enabled(on)
        conv.set_bn_bwd_fusion(fuse)
        resnet.set_residual_sink(sink)
        out = m(x.cuda())
        F.cross_entropy(out, y.cuda()).backward()
        errs = [(rel(p.grad, r), n) for p, r, n in zip(m.parameters(), g64, names)
                if float(r.norm()) > 1e-6]
        errs.sort(reverse=True)
        mean = sum(e for e, _ in errs) / len(errs)
        print(f"{label:20s} out {rel(out, out64):.3g} grad mean {mean:.3g} worst "
              + ", ".join(f"{n}={e:.2g}" for e, n in errs[:4]), flush=True)
        if os.environ.get("ALL"):
            for p, r, n in list(zip(m.parameters(), g64, names))[::-1]:
                print(f"    {n:32s} {rel(p.grad, r):.3g}  |g| {float(r.norm()):.3g}")
    conv.set_enabled(True)
    conv.set_bn_bwd_fusion(True)
    resnet.set_residual_sink(True)




def per_conv(net="resnet18"):
    """Check every HIP conv backward of one fused fp32 step against float64 on its own inputs."""
    from ewdml.ops import conv as cmod

    recs = []
    orig = cmod._Conv.backward

    def bwd(ctx, dy):
        x, w = ctx.saved_tensors
        dx, dw, a, b = orig(ctx, dy)
        recs.append((x.detach().clone(), w.detach().clone(), dy.detach().clone(),
                     None if dx is None else dx.detach().clone(), dw.detach().clone()))
        return dx, dw, a, b

    cmod._Conv.backward = staticmethod(bwd)
    torch.manual_seed(0)
    m = build_model(net, 10).to(memory_format=torch.channels_last).cuda()
    x = torch.randn(32, 3, 32, 32).contiguous(memory_format=torch.channels_last).cuda()
    y = torch.randint(0, 10, (32,)).cuda()
    F.cross_entropy(m(x), y).backward()
    cmod._Conv.backward = orig
    for x, w, dy, dx, dw in recs:
        k = w.shape[-1]
        xr = x.double().cpu().requires_grad_(True)
        wr = w.double().cpu().requires_grad_(True)
        F.conv2d(xr, wr, padding=k // 2).backward(dy.double().cpu())
        print(tuple(x.shape), tuple(w.shape), "dy cl", dy.is_contiguous(memory_format=torch.channels_last),
              "dx", None if dx is None else f"{rel(dx, xr.grad):.3g}", "dw", f"{rel(dw, wr.grad):.3g}",
              flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "per_conv":
        per_conv(sys.argv[1])
    else:
        main()
