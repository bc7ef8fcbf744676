"""Modules with PyTorch-compatible parameters whose GPU forward runs HIP kernels."""
from .modules import Conv2d, Linear, ReLU  # noqa: F401
