"""VGG-11 fp32 step at batch 64: per-parameter gradient error against float64 for the small-map
path on / off and the BN-backward-sum fusion on / off (which layer's BN gradients drift)."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from ewdml import ops  # noqa: E402
from ewdml.models import build_model  # noqa: E402
from ewdml.ops import conv  # noqa: E402

ops.require()
conv.set_enabled(True)
conv.set_winograd(True, 128, 2)
torch.manual_seed(0)
m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last)
for mod in m0.modules():
    if isinstance(mod, torch.nn.Dropout):
        mod.p = 0.0
x = torch.randn(64, 3, 32, 32).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (64,))
m64 = copy.deepcopy(m0).double()
F.cross_entropy(m64(x.double()), y).backward()
g64 = {n: p.grad for n, p in m64.named_parameters()}


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


res = {}
for sm in (True, False):
    for fused in (True, False):
        conv.set_smallmap(sm)
        conv.set_bn_bwd_fusion(fused)
        m = copy.deepcopy(m0).cuda()
        F.cross_entropy(m(x.cuda()), y.cuda()).backward()
        res[(sm, fused)] = {n: rel(p.grad, g64[n]) for n, p in m.named_parameters()}
names = [n for n in g64 if "features.1" in n or "features.2" in n or n.endswith("bias")]
print("param".ljust(22), " ".join(f"sm={a!s:5} fu={b!s:5}" for a, b in res))
for n in g64:
    if g64[n].norm() < 1e-6:
        continue
    print(n.ljust(22), " ".join(f"{res[k][n]:17.2e}" for k in res))
