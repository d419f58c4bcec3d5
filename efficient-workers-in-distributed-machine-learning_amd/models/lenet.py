"""LeNet for 1x28x28 inputs.

Parity: ``PyTorch-parameter-server/src/model_ops/lenet.py:15-36`` (conv 1->20 k5, pool, relu,
conv 20->50 k5, pool, relu, fc 800->500, fc 500->10 -- note the reference has *no* nonlinearity
between the two fully connected layers).  431,080 parameters in 8 tensors.

``fc_relu=True`` inserts the missing ReLU (off by default so the parameter/compute graph matches
the reference exactly).
"""
import torch.nn as nn
import torch.nn.functional as F

from .fused import pool2


class LeNet(nn.Module):
    def __init__(self, num_classes: int = 10, fc_relu: bool = False):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5, 1)
        self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(4 * 4 * 50, 500)
        self.fc2 = nn.Linear(500, num_classes)
        self.fc_relu = fc_relu

    def forward(self, x):
        x = F.relu(pool2(self.conv1(x)))
        x = F.relu(pool2(self.conv2(x)))
        x = self.fc1(x.flatten(1))
        if self.fc_relu:
            x = F.relu(x)
        return self.fc2(x)

    # its fused fp32 step (four launches, latency-bound at batch 64) beats the bf16 autocast path
    # (cuBLAS-class GEMMs and MIOpen convs per layer): the trainer keeps it under --amp bf16
    fused_fp32_beats_amp = True

    def fused_loss(self, x, y):
        """(mean cross-entropy, logits) through the fused HIP step (``ops/lenet.py``: four
        launches), or None where it does not apply (the caller then runs ``forward``)."""
        from ..ops.lenet import lenet_loss

        return lenet_loss(self, x, y)

    def name(self):
        return "lenet"


class MnistNet(nn.Module):
    """The Horovod example network (``horvod_pytorch.py:43-59``): conv10-conv20-dropout2d-fc50-fc10
    with log-softmax output."""

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 10, kernel_size=5)
        self.conv2 = nn.Conv2d(10, 20, kernel_size=5)
        self.conv2_drop = nn.Dropout2d()
        self.fc1 = nn.Linear(320, 50)
        self.fc2 = nn.Linear(50, num_classes)

    def forward(self, x):
        x = F.relu(pool2(self.conv1(x)))
        x = F.relu(pool2(self.conv2_drop(self.conv2(x))))
        x = F.relu(self.fc1(x.flatten(1)))
        x = F.dropout(x, training=self.training)
        return F.log_softmax(self.fc2(x), dim=1)


class KerasMnistCNN(nn.Module):
    """The Horovod TF/Keras example network (``tensorflow_mnist.py:27-36``): Conv2D(32, 3x3, relu)
    -> Conv2D(64, 3x3, relu) -> MaxPool 2x2 -> Dropout 0.25 -> Flatten -> Dense(128, relu) ->
    Dropout 0.5 -> Dense(10).  Keras 'valid' padding; logits out (the loss applies the softmax,
    as SparseCategoricalCrossentropy on the softmax output does)."""

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, kernel_size=3)
        self.conv2 = nn.Conv2d(32, 64, kernel_size=3)
        self.drop1 = nn.Dropout(0.25)
        self.fc1 = nn.Linear(64 * 12 * 12, 128)
        self.drop2 = nn.Dropout(0.5)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x):
        x = F.relu(self.conv2(F.relu(self.conv1(x))))
        x = self.drop1(pool2(x))
        x = self.drop2(F.relu(self.fc1(x.flatten(1))))
        return self.fc2(x)
