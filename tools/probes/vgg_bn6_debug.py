"""VGG-11 fp32 at batch 32 / 64 / 128: BN6 bias gradient (features.19.bias) of the HIP path and
MIOpen path against float64, worst channels."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from ewdml import ops  # noqa: E402
from ewdml.models import build_model  # noqa: E402
from ewdml.ops import conv  # noqa: E402

ops.require()
conv.set_winograd(True, 128, 2)
conv.set_smallmap(True)
for B in (32, 64, 128):
    torch.manual_seed(0)
    m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last)
    for mod in m0.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    x = torch.randn(B, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (B,))
    m64 = copy.deepcopy(m0).double()
    F.cross_entropy(m64(x.double()), y).backward()
    r = dict(m64.named_parameters())["features.19.bias"].grad
    out = {}
    for on in (True, False):
        conv.set_enabled(on)
        m = copy.deepcopy(m0).cuda()
        F.cross_entropy(m(x.cuda()), y.cuda()).backward()
        out[on] = dict(m.named_parameters())["features.19.bias"].grad.double().cpu()
    conv.set_enabled(True)
    for on in (True, False):
        d = (out[on] - r).abs()
        top = torch.topk(d, 4)
        print(f"B={B} {'hip   ' if on else 'miopen'} rel {float(d.norm() / r.norm()):.2e} |ref| "
              f"{float(r.abs().mean()):.2e} worst ch {top.indices.tolist()} diff "
              f"{[f'{v:.2e}' for v in top.values.tolist()]} ref {[f'{float(r[i]):.2e}' for i in top.indices]}")
