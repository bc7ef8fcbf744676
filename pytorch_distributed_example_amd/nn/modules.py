"""Layer modules with PyTorch-identical parameters, state_dict keys and initialisation.

``Conv2d`` / ``Linear`` reproduce ``torch.nn.Conv2d`` / ``torch.nn.Linear`` parameter shapes and
``reset_parameters`` (kaiming_uniform_(a=sqrt(5)) weight, U(+-1/sqrt(fan_in)) bias, weight first)
so that under the same seed a model built from them draws exactly the reference's initial weights
(reference: ``nn.Conv2d``/``nn.Linear`` at /root/reference/mnist/main.py:134-137).

Forward on a GPU tensor runs the framework's HIP kernels (``ops``); CPU tensors run ATen CPU ops
(the reference's ``--no-cuda`` path).  There is no GPU->ATen fallback.
"""
from __future__ import annotations

import math

import torch
from torch import nn as tnn
from torch.nn import init

from .. import ops


class Linear(tnn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, device=None, dtype=None):
        super().__init__()
        fk = {"device": device, "dtype": dtype or torch.float32}
        self.in_features = in_features
        self.out_features = out_features
        self.weight = tnn.Parameter(torch.empty(out_features, in_features, **fk))
        self.bias = tnn.Parameter(torch.empty(out_features, **fk)) if bias else None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1.0 / math.sqrt(self.in_features) if self.in_features > 0 else 0.0
            init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"


class Conv2d(tnn.Module):
    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1, padding: int = 0,
                 bias: bool = True, device=None, dtype=None):
        super().__init__()
        fk = {"device": device, "dtype": dtype or torch.float32}
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        self.stride = stride
        self.padding = padding
        self.weight = tnn.Parameter(torch.empty(out_channels, in_channels, *self.kernel_size, **fk))
        self.bias = tnn.Parameter(torch.empty(out_channels, **fk)) if bias else None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.in_channels * self.kernel_size[0] * self.kernel_size[1]
            bound = 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0.0
            init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return ops.conv2d(x, self.weight, self.bias, self.stride, self.padding)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}")


class ReLU(tnn.Module):
    def forward(self, x):
        return ops.relu(x)
