"""ResNet-50 for synthetic ImageNet-shaped data (BASELINE.json config 3: "ResNet-50 on
synthetic ImageNet shapes, top-k sparsified gradients + error feedback, 8 peers").

Channels-last bf16 so MIOpen picks its NHWC implicit-GEMM (MFMA) convolution kernels;
BatchNorm statistics are buffers that the trainers average at every synchronisation.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        nn.init.zeros_(self.bn3.weight)  # zero-init residual branch (Goyal et al.)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(y + idt)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), n_classes: int = 1000, width: int = 64):
        super().__init__()
        self.stem = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn = nn.BatchNorm2d(width)
        blocks = []
        cin = width
        for i, n in enumerate(layers):
            w = width * (2**i)
            for j in range(n):
                blocks.append(Bottleneck(cin, w, stride=2 if (j == 0 and i > 0) else 1))
                cin = w * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, n_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x, y=None):
        x = F.relu(self.bn(self.stem(x)))
        x = F.max_pool2d(x, 3, 2, 1)
        x = self.blocks(x)
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        logits = self.fc(x)
        if y is None:
            return logits
        return F.cross_entropy(logits.float(), y)


def resnet50(n_classes=1000):
    return ResNet((3, 4, 6, 3), n_classes)


def resnet_tiny(n_classes=10):
    return ResNet((1, 1, 1, 1), n_classes, width=8)
