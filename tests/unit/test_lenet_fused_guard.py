"""The fused LeNet step's guard (ops/lenet.py): off the GPU, under a fc ReLU or for other input
shapes it declines (returns None) and the trainer runs the module composition."""
import torch

from ewdml.models.lenet import LeNet
from ewdml.ops import lenet


def test_fused_loss_declines_on_cpu():
    m = LeNet()
    x = torch.randn(4, 1, 28, 28)
    y = torch.randint(0, 10, (4,))
    assert not lenet.supported(m, x, y)
    assert m.fused_loss(x, y) is None


def test_fused_loss_declines_fc_relu_and_other_shapes():
    m = LeNet(fc_relu=True)
    assert not lenet.supported(m, torch.randn(2, 1, 28, 28), torch.zeros(2, dtype=torch.int64))
    m = LeNet()
    assert not lenet.supported(m, torch.randn(2, 1, 32, 32), torch.zeros(2, dtype=torch.int64))
