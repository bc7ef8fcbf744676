"""2-layer MLP on MNIST-shaped input (BASELINE.json config 1: gloo/host backend, world_size=2, CPU)."""
from __future__ import annotations

import torch.nn.functional as F
from torch import nn as tnn

from .. import ops
from ..nn.modules import Linear


class MLP(tnn.Module):
    def __init__(self, in_features: int = 784, hidden: int = 512, classes: int = 10):
        super().__init__()
        self.fc1 = Linear(in_features, hidden)
        self.fc2 = Linear(hidden, classes)
        self.aten = False          # torch.nn.functional path (autocast-able; ``--dtype bf16``)

    def forward(self, x):
        x = x.reshape(x.shape[0], -1)
        if self.aten:
            x = F.relu(F.linear(x, self.fc1.weight, self.fc1.bias))
            return F.log_softmax(F.linear(x, self.fc2.weight, self.fc2.bias), dim=1)
        x = ops.relu(self.fc1(x))
        return ops.log_softmax(self.fc2(x), dim=1)
