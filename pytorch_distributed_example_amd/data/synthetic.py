"""Synthetic, device-resident MNIST-shaped datasets (no torchvision, no network on the GPU box).

The reference trains on FashionMNIST and evaluates on MNIST (/root/reference/mnist/main.py:156,173,
survey quirk Q4), both ``ToTensor`` + ``Normalize((0.1307,), (0.3081,))``.  We generate two
independent synthetic sets of the same shapes/dtypes (``[N,1,28,28]`` fp32, ``[N]`` int64 labels):
each class has a fixed random low-frequency prototype in [0,1]; a sample is its class prototype
plus pixel noise, clamped to [0,1] and normalised with the reference constants.  Being class
conditional, the data is learnable, so loss / accuracy curves are meaningful.

If real IDX files are present under ``root`` (``train-images-idx3-ubyte`` …) they are used instead.
"""
from __future__ import annotations

import gzip
import os

import numpy as np
import torch

MEAN, STD = 0.1307, 0.3081


class TensorDataset:
    """Images + labels already materialised (on any device)."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, name: str = "synthetic"):
        assert images.shape[0] == labels.shape[0]
        self.images = images
        self.labels = labels
        self.name = name

    def __len__(self):
        return self.images.shape[0]

    def __getitem__(self, i):
        return self.images[i], self.labels[i]

    def to(self, device):
        return TensorDataset(self.images.to(device), self.labels.to(device), self.name)


def _prototypes(seed: int, classes: int = 10) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    low = torch.rand(classes, 1, 7, 7, generator=g)
    proto = torch.nn.functional.interpolate(low, size=(28, 28), mode="bilinear", align_corners=False)
    return proto.clamp(0, 1)


def synthetic_mnist(n: int, seed: int = 0, device="cpu", kind: str = "fashion", noise: float = 0.35,
                    chunk: int = 16384) -> TensorDataset:
    """``n`` samples of a class-conditional synthetic MNIST-like set, generated on ``device``."""
    device = torch.device(device)
    base_seed = {"fashion": 1000, "digits": 2000}.get(kind, 3000) + seed
    proto = _prototypes(base_seed).to(device)
    g = torch.Generator(device=device).manual_seed(base_seed + 1)
    labels = torch.randint(0, 10, (n,), generator=g, device=device, dtype=torch.int64)
    images = torch.empty(n, 1, 28, 28, device=device, dtype=torch.float32)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        x = proto[labels[s:e]] + noise * torch.randn(e - s, 1, 28, 28, generator=g, device=device)
        images[s:e] = (x.clamp_(0, 1) - MEAN) / STD
    return TensorDataset(images, labels, name=f"synthetic-{kind}")


def _read_idx(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    nd = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i: 8 + 4 * i], "big") for i in range(nd)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd).reshape(dims)


def idx_dataset(root: str, train: bool, device="cpu"):
    """Real (Fashion)MNIST from IDX files if present, else None."""
    pre = "train" if train else "t10k"
    for suffix in ("", ".gz"):
        ip = os.path.join(root, f"{pre}-images-idx3-ubyte{suffix}")
        lp = os.path.join(root, f"{pre}-labels-idx1-ubyte{suffix}")
        if os.path.exists(ip) and os.path.exists(lp):
            x = torch.from_numpy(_read_idx(ip).copy()).float().div_(255.0).sub_(MEAN).div_(STD)
            y = torch.from_numpy(_read_idx(lp).copy()).long()
            return TensorDataset(x.view(-1, 1, 28, 28).to(device), y.to(device), name=f"idx:{root}")
    return None
