"""Samplers.

* :class:`DistributedSampler` -- the reference's rank-sharded sampler
  (``/root/reference/mingpt/trainer.py:73-81``) with the reshuffle-per-epoch contract honoured:
  the trainer calls :meth:`set_epoch` every epoch (fixes D20, identical permutation every epoch).
* :class:`InfiniteRandomSampler` -- upstream minGPT's
  ``RandomSampler(replacement=True, num_samples=int(1e10))``, sharded by rank so every rank draws
  an independent stream (iteration-based ``Trainer``).
"""
from __future__ import annotations

import math
from typing import Iterator

import torch
from torch.utils.data import Sampler


class DistributedSampler(Sampler):
    def __init__(self, dataset, num_replicas: int = 1, rank: int = 0, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        self.n = len(dataset)
        self.num_replicas, self.rank = num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        self.start = 0
        if drop_last:
            self.num_samples = self.n // num_replicas
        else:
            self.num_samples = math.ceil(self.n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int, start: int = 0) -> None:
        """Select the epoch's permutation; ``start`` skips this rank's first ``start`` samples
        (mid-epoch resume from a step-granular snapshot)."""
        self.epoch = epoch
        self.start = start

    def __iter__(self) -> Iterator[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            idx += (idx * math.ceil(pad / max(1, len(idx))))[:pad]
        else:
            idx = idx[: self.total_size]
        return iter(idx[self.rank: self.total_size: self.num_replicas][self.start:])

    def __len__(self) -> int:
        return self.num_samples - self.start


class InfiniteRandomSampler(Sampler):
    def __init__(self, dataset, rank: int = 0, seed: int = 0, num_samples: int = int(1e10)):
        self.n = len(dataset)
        self.rank, self.seed, self.num_samples = rank, seed, num_samples

    def __iter__(self):
        g = torch.Generator()
        g.manual_seed(self.seed * 1000003 + self.rank)
        remaining = self.num_samples
        while remaining > 0:
            k = min(remaining, 1 << 16)
            for i in torch.randint(self.n, (k,), generator=g).tolist():
                yield i
            remaining -= k

    def __len__(self):
        return self.num_samples
