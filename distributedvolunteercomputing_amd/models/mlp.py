"""2-layer MLP on MNIST shapes (BASELINE.json config 1: "2 local volunteer procs on CPU/gloo,
2-layer MLP on synthetic MNIST shapes, local-SGD + periodic all-reduce")."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class MLP(nn.Module):
    def __init__(self, d_in: int = 784, hidden: int = 256, n_classes: int = 10, seed: int = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w1 = nn.Parameter(torch.randn(hidden, d_in, generator=g) * (2.0 / d_in) ** 0.5)
        self.b1 = nn.Parameter(torch.zeros(hidden))
        self.w2 = nn.Parameter(torch.randn(n_classes, hidden, generator=g) * (1.0 / hidden) ** 0.5)
        self.b2 = nn.Parameter(torch.zeros(n_classes))
        self.n_classes = n_classes

    def forward(self, x, y=None):
        h = F.relu(F.linear(x.flatten(1).to(self.w1.dtype), self.w1, self.b1))
        logits = F.linear(h, self.w2, self.b2)
        if y is None:
            return logits
        return F.cross_entropy(logits.float(), y)


def synthetic_mnist(n: int, seed: int = 0, device="cpu", n_classes: int = 10):
    """Linearly separable synthetic 'MNIST': 28x28 images whose class is encoded by a
    fixed random template plus noise (so training loss must go down)."""
    g = torch.Generator().manual_seed(1234)
    templates = torch.randn(n_classes, 784, generator=g)
    g2 = torch.Generator().manual_seed(seed)
    y = torch.randint(0, n_classes, (n,), generator=g2)
    x = templates[y] + 0.5 * torch.randn(n, 784, generator=g2)
    return x.view(n, 1, 28, 28).to(device), y.to(device)


_ = ops  # the MLP uses plain torch ops; kept importable alongside the other models
