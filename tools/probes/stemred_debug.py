"""Debug: which conv backward sees the stem's BN layer as its link (deferred reduction)?"""
import torch
import torch.nn.functional as F

from ewdml import ops
from ewdml.models import build_model
from ewdml.ops import conv as cmod

ops.require()
orig_link = cmod._bn_bwd_link


def link(node, x):
    r = orig_link(node, x)
    print("link", tuple(x.shape), "node", type(node).__name__ if node is not None else None,
          "stem_in", getattr(node, "stem_in", None), "link", r is not None, flush=True)
    return r


cmod._bn_bwd_link = link
orig_defer = ops.require().cf_defer_reduce
m = build_model("vgg11", 10).to(memory_format=torch.channels_last).cuda()
x = torch.randn(128, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (128,), device="cuda")
F.cross_entropy(m(x), y).backward()
torch.cuda.synchronize()
print("stem_red flag after", cmod._STEM_RED, flush=True)
