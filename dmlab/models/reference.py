"""Plain-PyTorch definitions of every model family, used as the numerical
reference for the native HIP programs and as the CPU execution path.

* ``TorchLeNet``  — the reference ``Net`` (task1/pytorch/model.py:12-35; identical
  copies in task2/model.py:13-37, task3/model.py:12-36): conv(1→6,k5,p2)→ReLU→pool2
  → conv(6→16,k5)→ReLU→pool2 → fc 400→120 → ReLU → fc 120→10 (51,902 params).
* ``TorchMLP``    — the MindSpore ``ForwardNN`` (codes/task1/mindspore/model.ipynb,
  cells defining Dense 784→512→256→128→64→32→10).  ``reference_compat=True``
  reproduces the notebook's softmax-before-SoftmaxCrossEntropy.
* ``TorchResNet18`` — the BASELINE.json headline "ResNet-18-shaped CNN" (extension,
  not in the reference): 7×7/2 stem, BN, ReLU, 3×3/2 maxpool, 4 stages of 2
  BasicBlocks (64/128/256/512), global avgpool, fc.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class TorchLeNet(nn.Module):
    def __init__(self, in_channels: int = 1, num_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, 6, kernel_size=5, stride=1, padding=2)
        self.conv2 = nn.Conv2d(6, 16, kernel_size=5, stride=1, padding=0)
        self.fc1 = nn.Linear(16 * 5 * 5, 120)
        self.fc2 = nn.Linear(120, num_classes)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv1(x)), 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = x.flatten(1)
        return self.fc2(F.relu(self.fc1(x)))


class TorchMLP(nn.Module):
    DIMS = (784, 512, 256, 128, 64, 32, 10)

    def __init__(self, dims=DIMS, reference_compat: bool = False):
        super().__init__()
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(dims[:-1], dims[1:]))
        self.reference_compat = reference_compat

    def forward(self, x):
        x = x.flatten(1)
        for i, l in enumerate(self.layers):
            x = l(x)
            if i < len(self.layers) - 1:
                x = F.relu(x)
        if self.reference_compat:
            x = F.softmax(x, dim=1)
        return x


class TorchBasicBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, 0, bias=False),
                                      nn.BatchNorm2d(cout))

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + idt)


class TorchResNet18(nn.Module):
    def __init__(self, num_classes: int = 1000, in_channels: int = 3, widths=(64, 128, 256, 512)):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, widths[0], 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(widths[0])
        blocks = []
        cin = widths[0]
        for i, w in enumerate(widths):
            stride = 1 if i == 0 else 2
            blocks.append(TorchBasicBlock(cin, w, stride))
            blocks.append(TorchBasicBlock(w, w, 1))
            cin = w
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(widths[-1], num_classes)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.blocks(x)
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.fc(x)
