"""LeNet (the reference ``Net``) and its two pipeline halves.

Reference: ``Net`` task1/pytorch/model.py:12-35 (copies in task2/model.py:13-37,
task2/model-mp.py:13-37, task3/model.py:12-36); ``SubNetConv`` task4/model.py:18-32;
``SubNetFC`` task4/model.py:34-47.

Native schedule (3 fused stages instead of ~10 ATen ops):
  conv1+bias+ReLU+pool2 → conv2+bias+ReLU+pool2 → flatten(view) → fc1+bias+ReLU → fc2+bias
"""
from __future__ import annotations

from dmlab.nn.layers import Conv2d, Flatten, Linear
from dmlab.nn.program import Program


class Net(Program):
    def __init__(self, in_channels: int = 1, num_classes: int = 10):
        super().__init__()
        self.conv1 = Conv2d(in_channels, 6, 5, 1, 2, bias=True, relu=True, pool=2)
        self.conv2 = Conv2d(6, 16, 5, 1, 0, bias=True, relu=True, pool=2)
        self.flatten = Flatten()
        self.fc1 = Linear(16 * 5 * 5, 120, relu=True)
        self.fc2 = Linear(120, num_classes)
        self.build([self.conv1, self.conv2, self.flatten, self.fc1, self.fc2])


LeNet = Net


class SubNetConv(Program):
    """Pipeline stage 0: conv trunk → (B, 400)."""

    def __init__(self, in_channels: int = 1):
        super().__init__()
        self.conv1 = Conv2d(in_channels, 6, 5, 1, 2, bias=True, relu=True, pool=2)
        self.conv2 = Conv2d(6, 16, 5, 1, 0, bias=True, relu=True, pool=2)
        self.flatten = Flatten()
        self.build([self.conv1, self.conv2, self.flatten])


class SubNetFC(Program):
    """Pipeline stage 1: fc head → logits (B, num_classes)."""

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.fc1 = Linear(16 * 5 * 5, 120, relu=True)
        self.fc2 = Linear(120, num_classes)
        self.build([self.fc1, self.fc2])
