"""Samplers with ``torch.utils.data.distributed.DistributedSampler``-identical index semantics.

The reference shards the training set with ``DistributedSampler(train_set)`` (rank / world size
taken from the default process group, /root/reference/mnist/main.py:164) and never calls
``set_epoch`` (so every epoch reuses the epoch-0 permutation, survey quirk Q5).  This sampler
reproduces torch's algorithm exactly (torch/utils/data/distributed.py:66-146):

* ``num_samples = ceil(N / W)`` (or ``ceil((N - W) / W)`` with ``drop_last`` and a remainder),
  ``total_size = num_samples * W``
* ``randperm(N)`` from a CPU generator seeded ``seed + epoch`` when shuffling
* pad by wrapping the permutation (or truncate with ``drop_last``)
* rank r takes ``indices[r : total_size : W]``

It additionally exposes the indices as one int32 tensor (``indices_tensor``) so the training engine
can upload an epoch's permutation to the device once and gather batches inside its first kernel.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch


class DistributedSampler:
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            from .. import dist

            if not dist.is_initialized():
                raise RuntimeError("DistributedSampler needs num_replicas/rank or an initialised process group")
            num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
            rank = dist.get_rank() if rank is None else rank
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = int(num_replicas)
        self.rank = int(rank)
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if self.drop_last and n % self.num_replicas != 0:
            self.num_samples = math.ceil((n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def indices_tensor(self) -> torch.Tensor:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        if not self.drop_last:
            pad = self.total_size - n
            if pad > 0:
                reps = math.ceil(pad / n)
                idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[: self.total_size]
        assert idx.numel() == self.total_size
        out = idx[self.rank: self.total_size: self.num_replicas]
        assert out.numel() == self.num_samples
        return out.to(torch.int32)

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices_tensor().tolist())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch


class RandomSampler:
    """Shuffling sampler for the single-process path (reference: ``DataLoader(shuffle=True)``,
    /root/reference/mnist/main.py:158-162): a fresh permutation every epoch from a seeded generator."""

    def __init__(self, dataset, seed: int = 0):
        self.dataset = dataset
        self.seed = seed
        self.epoch = 0

    def indices_tensor(self) -> torch.Tensor:
        g = torch.Generator()
        g.manual_seed(self.seed * 1000003 + self.epoch)
        idx = torch.randperm(len(self.dataset), generator=g).to(torch.int32)
        self.epoch += 1
        return idx

    def __iter__(self):
        return iter(self.indices_tensor().tolist())

    def __len__(self):
        return len(self.dataset)

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch


class SequentialSampler:
    def __init__(self, dataset):
        self.dataset = dataset

    def indices_tensor(self) -> torch.Tensor:
        return torch.arange(len(self.dataset), dtype=torch.int32)

    def __iter__(self):
        return iter(range(len(self.dataset)))

    def __len__(self):
        return len(self.dataset)

    def set_epoch(self, epoch: int) -> None:
        pass
