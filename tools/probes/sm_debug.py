"""Which gradients differ between two VGG-11 fp32 steps (lazy / materialised BN, small-map convs)."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import ewdml  # noqa: E402,F401
from ewdml.models import build_model, fused  # noqa: E402
from ewdml.ops import conv, nn as onn  # noqa: E402

conv.set_enabled(True)
conv.set_winograd(True, 128, 2)
conv.set_smallmap(True)
torch.manual_seed(0)
m0 = build_model("vgg11", 10).to(memory_format=torch.channels_last).cuda()
for mod in m0.modules():
    if isinstance(mod, torch.nn.Dropout):
        mod.p = 0.0
x = torch.randn(64, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (64,), device="cuda")


def run(lazy, sm=True):
    fused._LAZY = lazy
    onn._LAZY_BWD = lazy
    conv.set_smallmap(sm)
    m = copy.deepcopy(m0)
    loss = F.cross_entropy(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    fused._LAZY = True
    onn._LAZY_BWD = True
    return {n: p.grad.clone() for n, p in m.named_parameters()}, float(loss)


runs = {k: run(*k) for k in [(True, True), (True, True), (False, True), (False, True),
                             (True, False), (False, False)]}
keys = list(runs)
ref = runs[keys[0]][0]
for k in keys[1:]:
    g, l = runs[k]
    diff = [n for n in ref if not torch.equal(ref[n], g[n])]
    print(k, "loss", l, "differing grads vs lazy/sm:", diff[:12], len(diff))
a, b = runs[(True, True)][0], runs[(True, True)][0]
