"""2-layer MLP on MNIST-shaped input (BASELINE.json config 1: gloo/host backend, world_size=2, CPU)."""
from __future__ import annotations

from torch import nn as tnn

from .. import ops
from ..nn.modules import Linear


class MLP(tnn.Module):
    def __init__(self, in_features: int = 784, hidden: int = 512, classes: int = 10):
        super().__init__()
        self.fc1 = Linear(in_features, hidden)
        self.fc2 = Linear(hidden, classes)

    def forward(self, x):
        x = x.reshape(x.shape[0], -1)
        x = ops.relu(self.fc1(x))
        return ops.log_softmax(self.fc2(x), dim=1)
