"""Functional ops.  GPU tensors run the framework's CDNA4 HIP kernels; CPU tensors run ATen CPU.

There is no GPU fallback to ATen: a GPU op without a HIP kernel raises (see ``_ext.kernels``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .lenet_fused import LeNetFunction, lenet_forward, pack_conv2_weight  # noqa: F401
from . import generic  # noqa: F401
from . import transformer  # noqa: F401


def linear(x, weight, bias=None):
    if x.is_cuda:
        return generic.linear(x, weight, bias)
    return F.linear(x, weight, bias)


def relu(x):
    if x.is_cuda:
        return generic.relu(x)
    return F.relu(x)


def conv2d(x, weight, bias=None, stride=1, padding=0):
    if x.is_cuda:
        return generic.conv2d(x, weight, bias, stride, padding)
    return F.conv2d(x, weight, bias, stride, padding)


def max_pool2d(x, kernel_size=2, stride=2):
    if x.is_cuda:
        return generic.max_pool2d(x, kernel_size, stride)
    return F.max_pool2d(x, kernel_size, stride)


def log_softmax(x, dim=1):
    if x.is_cuda:
        return generic.log_softmax(x, dim)
    return F.log_softmax(x, dim=dim)


def cross_entropy(logits, target, reduction="mean"):
    """``F.cross_entropy`` (log_softmax + nll) — one fused HIP kernel forward and backward on GPU."""
    if logits.is_cuda:
        return generic.cross_entropy(logits, target, reduction)
    return F.cross_entropy(logits, target, reduction=reduction)
