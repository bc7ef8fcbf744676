"""The reference toy CNN (``Net``, /root/reference/mnist/main.py:130-147).

Parameter names, shapes, registration order and initialisation are identical to the reference
(``conv1.weight [20,1,5,5] … fc2.bias [10]``), so ``state_dict`` files are interchangeable.

Execution:
* GPU input  -> one fused HIP autograd Function (``ops.LeNetFunction``: 4 forward launches, 3 backward)
* CPU input  -> the layer-by-layer ATen CPU path (the reference's ``--no-cuda`` mode)
* ``net.aten = True`` -> the same layer-by-layer path through ``torch.nn.functional`` on any device,
  which ``torch.autocast`` can lower to bf16 (``scripts/mnist.py --dtype bf16``: the framework's
  toy-CNN kernels are fp32, the reference's dtype)
The high-throughput trainer (``engine.LeNetTrainStep``) runs the same kernels without autograd
and fuses the loss and the optimizer into the step.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn as tnn

from .. import ops
from ..nn.modules import Conv2d, Linear

PARAM_SPECS = (
    ("conv1.weight", (20, 1, 5, 5)),
    ("conv1.bias", (20,)),
    ("conv2.weight", (50, 20, 5, 5)),
    ("conv2.bias", (50,)),
    ("fc1.weight", (500, 800)),
    ("fc1.bias", (500,)),
    ("fc2.weight", (10, 500)),
    ("fc2.bias", (10,)),
)
NUM_PARAMS = 431080


class Net(tnn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = Conv2d(1, 20, 5, 1)
        self.conv2 = Conv2d(20, 50, 5, 1)
        self.fc1 = Linear(4 * 4 * 50, 500)
        self.fc2 = Linear(500, 10)
        self.aten = False

    def forward(self, x):
        if self.aten:
            x = F.max_pool2d(F.relu(F.conv2d(x, self.conv1.weight, self.conv1.bias)), 2, 2)
            x = F.max_pool2d(F.relu(F.conv2d(x, self.conv2.weight, self.conv2.bias)), 2, 2)
            x = F.relu(F.linear(x.reshape(-1, 4 * 4 * 50), self.fc1.weight, self.fc1.bias))
            return F.log_softmax(F.linear(x, self.fc2.weight, self.fc2.bias), dim=1)
        if x.is_cuda:
            return ops.lenet_forward(x, self)
        x = ops.relu(self.conv1(x))
        x = ops.max_pool2d(x, 2, 2)
        x = ops.relu(self.conv2(x))
        x = ops.max_pool2d(x, 2, 2)
        x = x.view(-1, 4 * 4 * 50)
        x = ops.relu(self.fc1(x))
        x = self.fc2(x)
        return ops.log_softmax(x, dim=1)


def build_net(seed: int | None = None, device=None) -> Net:
    """Construct ``Net`` with a deterministic init (``seed``) -- the reference seeds nothing (Q2)."""
    if seed is not None:
        g = torch.random.get_rng_state()
        torch.manual_seed(seed)
        net = Net()
        torch.random.set_rng_state(g)
    else:
        net = Net()
    return net.to(device) if device is not None else net
