"""Batch iterator over an in-memory (device-resident) dataset.

Replaces ``torch.utils.data.DataLoader`` + ``default_collate`` for the reference's usage
(/root/reference/mnist/main.py:150-177): instead of per-sample Python fetch + transform + collate
and an H2D copy per step, the whole dataset lives on the device and a batch is one index gather.
Batch boundaries (including the ragged final batch) are identical to DataLoader(drop_last=False).
"""
from __future__ import annotations

import math

import torch

from .sampler import DistributedSampler, RandomSampler, SequentialSampler  # noqa: F401


class DeviceDataLoader:
    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, sampler=None, drop_last: bool = False,
                 seed: int = 0):
        if sampler is not None and shuffle:
            raise ValueError("sampler option is mutually exclusive with shuffle")
        self.dataset = dataset
        self.batch_size = batch_size
        self.drop_last = drop_last
        if sampler is None:
            sampler = RandomSampler(dataset, seed=seed) if shuffle else SequentialSampler(dataset)
        self.sampler = sampler

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def epoch_indices(self) -> torch.Tensor:
        """This epoch's sample order as int32 (advances RandomSampler's epoch, like DataLoader)."""
        return self.sampler.indices_tensor()

    def __iter__(self):
        idx = self.epoch_indices().to(self.dataset.images.device, torch.long)
        n = idx.numel()
        stop = (n // self.batch_size) * self.batch_size if self.drop_last else n
        for s in range(0, stop, self.batch_size):
            sel = idx[s: min(s + self.batch_size, stop)]
            yield self.dataset.images.index_select(0, sel), self.dataset.labels.index_select(0, sel)
