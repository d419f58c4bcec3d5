"""Which ResNet blocks hand their shortcut gradient to the first conv's epilogue (GradSink) and
which leave the sum to autograd: one fp32 training step of ResNet-50 CIFAR on the GPU, logging the
order of the _SinkTap backwards (deposited / returned) and the sink-adding backward-data launches.

    python tools/probes/sink_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import ewdml  # noqa: E402
from ewdml.models import build_model  # noqa: E402
from ewdml.ops import conv as cv  # noqa: E402

events = []
orig = cv._SinkTap.backward


def tap_backward(ctx, g):
    sink = ctx.sink
    r = orig(ctx, g)
    events.append(("tap", tuple(g.shape), "returned" if r[0] is not None else "deposited",
                   None if sink is None else sink.taken))
    return r


cv._SinkTap.backward = staticmethod(tap_backward)
ewdml.ops.require()
torch.manual_seed(0)
m = build_model("ResNet50", 10).cuda().to(memory_format=torch.channels_last)
x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (32,), device="cuda")
before = cv.SINK_ADDS
loss = torch.nn.functional.cross_entropy(m(x), y)
loss.backward()
torch.cuda.synchronize()
for e in events:
    print(e)
print("sink adds", cv.SINK_ADDS - before)
