"""Per-parameter gradient differences of one fp32 VGG-11 step with the lazy BN forward / backward
(ops/nn.py, winograd_f32.hip WgSrc) switched on and off separately."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch
import torch.nn.functional as F

import ewdml  # noqa: F401
from ewdml.models import build_model, fused
from ewdml.ops import conv
from ewdml.ops import nn as fnn


CODES = []
BWD = []


def _patch_bwd():
    cls = fnn._BNAct
    orig = cls.backward

    def bwd(ctx, dy):
        pre = getattr(ctx, "_ew_pre_bwd", None)
        h, res, code, stats = ctx.saved_tensors
        C = dy.shape[1]
        ref = None
        if not ctx.pool:  # fp64 sums from the recorded operands (unpooled layers)
            hd = h.double().permute(0, 2, 3, 1).reshape(-1, C)
            dd = dy.double().permute(0, 2, 3, 1).reshape(-1, C)
            st = stats.double().view(4, C)
            z = hd * st[2] + st[3]
            dz = torch.where(z > 0, dd, torch.zeros_like(dd))
            ref = torch.stack([dz.sum(0), (dz * (hd - st[0])).sum(0)])
        got = None
        if pre is not None:
            got = pre[0][:2 * pre[1] * C].view(2, pre[1], C).double().sum(1)
        BWD.append((dy.detach().clone(),
                    None if pre is None else pre[0][:2 * pre[1] * C].clone(),
                    None if pre is None else pre[1], ref, got, h.detach().clone(),
                    stats.detach().clone()))
        out = orig(ctx, dy)
        BWD.append(("dx", out[0].detach().clone() if out[0] is not None else None))
        return out

    cls.backward = staticmethod(bwd)


def grads(model, x, y):
    m = copy.deepcopy(model)
    CODES.clear()
    orig = fnn.bn_relu

    def rec(h, cb, bn, pool=False, lazy=False):
        out = orig(h, cb, bn, pool, lazy=lazy)
        CODES.append((out, pool, lazy))
        return out

    fnn.bn_relu = rec
    try:
        out = m(x)
    finally:
        fnn.bn_relu = orig
    torch.cuda.synchronize()
    codes = [(o.grad_fn.saved_tensors[2].clone() if p else None, lz) for o, p, lz in CODES]
    BWD.clear()
    F.cross_entropy(out, y).backward()
    return (out.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}, codes,
            list(BWD))


def main():
    conv.set_winograd(True, 128, 2)
    torch.manual_seed(0)
    m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last).cuda()
    for mod in m0.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    torch.manual_seed(0)  # the data of tests/kernels/test_conv_f32.py::test_fp32_vgg11_step_vs_fp64
    m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last)
    for mod in m0.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    x = torch.randn(32, 3, 32, 32).contiguous(memory_format=torch.channels_last).cuda()
    y = torch.randint(0, 10, (32,)).cuda()
    m0 = m0.cuda()
    _patch_bwd()
    res = {}
    for name, lf, lb in [("none", False, False), ("fwd", True, False), ("bwd", False, True),
                         ("both", True, True)]:
        fused._LAZY, fnn._LAZY_BWD = lf, lb
        res[name] = grads(m0, x, y)
    fused._LAZY, fnn._LAZY_BWD = True, True
    m64 = copy.deepcopy(m0).cpu().double()
    F.cross_entropy(m64(x.cpu().double()), y.cpu()).backward()
    g64 = {k: p.grad for k, p in m64.named_parameters()}
    conv.set_enabled(False)
    res["miopen"] = grads(m0, x, y)
    conv.set_enabled(True)
    for name in ("none", "fwd", "bwd", "both", "miopen"):
        worst = sorted(((float((res[name][1][k].double().cpu() - g64[k]).norm() / g64[k].norm()),
                         k, float(g64[k].norm())) for k in g64 if float(g64[k].norm()) > 1e-6),
                       reverse=True)[:4]
        print("vs fp64", name, worst, flush=True)
    b0, b1 = res["none"][3], res["fwd"][3]
    for i, (a, b) in enumerate(zip(b0, b1)):
        if a[0] == "dx":
            if a[1] is not None:
                print(f"bn-bwd[{i}] dx rel {float((a[1] - b[1]).norm() / a[1].norm()):.3e}",
                      flush=True)
            continue
        msg = f"bn-bwd[{i}] dy rel {float((a[0] - b[0]).norm() / a[0].norm()):.3e}"
        if a[1] is not None and b[1] is not None and a[2] == b[2]:
            msg += f" pre rel {float((a[1] - b[1]).norm() / a[1].norm()):.3e} rows {a[2]}"
        else:
            msg += f" pre {a[2]} vs {b[2]}"
        print(msg, flush=True)
        print(f"     h rel {float((a[5] - b[5]).norm() / a[5].norm()):.3e} stats rel "
              + " ".join(f"{float((a[6].view(4, -1)[q] - b[6].view(4, -1)[q]).norm() / a[6].view(4, -1)[q].norm()):.2e}"
                         for q in range(4)), flush=True)
        for nm, e in (("none", a), ("fwd", b)):
            if e[3] is not None and e[4] is not None:
                r = e[3]
                print(f"     {nm}: s1 rel {float((e[4][0] - r[0]).norm() / r[0].norm()):.3e} "
                      f"s2 rel {float((e[4][1] - r[1]).norm() / r[1].norm()):.3e} "
                      f"|s1|/sum|dz| {float(r[0].norm()):.3e}", flush=True)
    c0 = res["none"][2]
    for (a, la), (b, lb) in zip(res["fwd"][2], c0):
        if a is not None:
            print("codes lazy", la, "differ", int((a != b).sum()), "of", a.numel(), flush=True)
    o0, g0 = res["none"][0], res["none"][1]
    for name in ("fwd", "bwd", "both"):
        o, g = res[name][0], res[name][1]
        print(name, "out rel", float((o - o0).norm() / o0.norm()), flush=True)
        for k in g0:
            r = float((g[k] - g0[k]).norm() / (g0[k].norm() + 1e-30))
            if r > 1e-6:
                print(f"   {k:40s} {r:.3e}", flush=True)


if __name__ == "__main__":
    main()
