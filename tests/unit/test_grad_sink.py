"""GradSink hand-over (ops/conv.py ``sink_tap``): the shortcut branch's input gradient reaches the
consuming conv's backward when autograd runs the shortcut first (it was recorded last), and goes
back to autograd's own sum when the consumer has already run -- either way x.grad is the sum."""
import torch

import ewdml  # noqa: F401
from ewdml.ops.conv import GradSink, sink_tap


class _Consumer(torch.autograd.Function):
    """Stands in for the block's first conv: y = 2x, dx = 2 dy + the sink's gradient."""

    @staticmethod
    def forward(ctx, x, sink):
        ctx.sink = sink
        return 2 * x

    @staticmethod
    def backward(ctx, dy):
        sink, ctx.sink = ctx.sink, None
        dx = 2 * dy
        if sink.grad is not None:
            dx = dx + sink.grad
        sink.grad, sink.taken = None, True
        return dx, None


def test_sink_tap_deposits_when_the_shortcut_runs_first():
    torch.manual_seed(0)
    x = torch.randn(16, requires_grad=True)
    w1, w2 = torch.randn(16), torch.randn(16)
    sink = GradSink()
    y1 = _Consumer.apply(x, sink)
    y2 = sink_tap(x, sink) * w2          # recorded last: autograd runs it first
    (y1 * w1 + y2).sum().backward()
    assert sink.taken and sink.grad is None
    torch.testing.assert_close(x.grad, 2 * w1 + w2, rtol=0, atol=0)


def test_sink_tap_falls_back_to_autograd_when_the_consumer_ran_first():
    torch.manual_seed(0)
    x = torch.randn(16, requires_grad=True)
    w1, w2 = torch.randn(16), torch.randn(16)
    sink = GradSink()
    y2 = sink_tap(x, sink) * w2          # recorded first: runs after the consumer
    y1 = _Consumer.apply(x, sink)
    (y1 * w1 + y2).sum().backward()
    assert sink.taken and sink.grad is None
    torch.testing.assert_close(x.grad, 2 * w1 + w2, rtol=0, atol=0)
