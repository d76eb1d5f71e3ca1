"""Data-partitioning samplers for data-parallel training (lab 3).

The reference ships ``MySampler`` as a skeleton whose ``__iter__`` raises
NotImplementedError (codes/task3/sampler.py:5-25) and asks the
student for two strategies (sections/task3.tex:21-23):

* **random partition** (:class:`PartitionSampler`): one global permutation per
  epoch (seed + epoch, identical on every rank), padded to a multiple of the world
  size, then sharded so that ranks see *disjoint* subsets that together cover the
  dataset — the ``DistributedSampler`` semantics used by task2/model.py:124.
* **random sampling** (:class:`RandomSampleSampler`): every rank draws its own
  indices i.i.d. (with or without replacement inside the rank) from the *whole*
  dataset with a rank-dependent seed (task3/model.py:111 passes ``seed=rank``);
  shards may overlap.

Both implement ``set_epoch`` (task3.tex:52) — the reference never calls it (B3);
our training loops do.  ``MySampler`` is kept as the reference-named entry point.
"""
from __future__ import annotations

import math

import torch
from torch.utils.data import Sampler


class _RankSampler(Sampler):
    def __init__(self, dataset, num_replicas: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if num_replicas < 1 or not (0 <= rank < num_replicas):
            raise ValueError(f"invalid rank {rank} for num_replicas {num_replicas}")
        self.dataset = dataset
        self.n = len(dataset)
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.epoch = 0
        self.drop_last = drop_last
        if drop_last and self.n % num_replicas:
            self.num_samples = self.n // num_replicas
        else:
            self.num_samples = math.ceil(self.n / num_replicas)  # task3/sampler.py:14
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __len__(self) -> int:
        return self.num_samples

    def indices(self) -> torch.Tensor:
        raise NotImplementedError

    def __iter__(self):
        return iter(self.indices().tolist())


class PartitionSampler(_RankSampler):
    """Random partition: disjoint per-rank shards of one shared permutation."""

    def indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n)
        if self.total_size > self.n:  # pad by wrapping (every sample seen >= once)
            reps = math.ceil((self.total_size - self.n) / self.n)
            idx = torch.cat([idx] + [idx] * reps)[: self.total_size]
        else:
            idx = idx[: self.total_size]
        return idx[self.rank: self.total_size: self.num_replicas]


class RandomSampleSampler(_RankSampler):
    """Random sampling: independent per-rank draws from the whole dataset.

    ``replacement=False`` draws a per-rank random subset (no duplicates inside a
    rank, overlaps across ranks allowed); ``replacement=True`` draws i.i.d.
    indices (bootstrap).  The seed is ``seed * 1_000_003 + rank`` mixed with the
    epoch so ranks differ even when the caller passes the same seed."""

    def __init__(self, *a, replacement: bool = False, **kw):
        super().__init__(*a, **kw)
        self.replacement = replacement

    def indices(self) -> torch.Tensor:
        g = torch.Generator().manual_seed(
            (self.seed * 1_000_003 + self.rank * 7919 + self.epoch * 104_729) & 0x7FFFFFFF)
        if self.replacement:
            return torch.randint(0, self.n, (self.num_samples,), generator=g)
        if not self.shuffle:
            start = (self.rank * self.num_samples) % self.n
            return (torch.arange(self.num_samples) + start) % self.n
        return torch.randperm(self.n, generator=g)[: self.num_samples]


class MySampler(_RankSampler):
    """Reference-named sampler (codes/task3/sampler.py:5) with both strategies.

    ``mode='partition'`` (default) or ``mode='random'``; the reference CLI flag
    ``--mode`` (task4/model.py:149, default 'division') maps 'division' to
    partition."""

    def __init__(self, dataset, num_replicas, rank, shuffle=True, seed=0, mode="partition",
                 drop_last=False):
        super().__init__(dataset, num_replicas, rank, shuffle, seed, drop_last)
        mode = {"division": "partition"}.get(mode, mode)
        if mode not in ("partition", "random"):
            raise ValueError(f"unknown sampling mode {mode!r}")
        self.mode = mode
        cls = PartitionSampler if mode == "partition" else RandomSampleSampler
        self._impl = cls(dataset, num_replicas, rank, shuffle, seed, drop_last)

    def set_epoch(self, epoch):
        super().set_epoch(epoch)
        self._impl.set_epoch(epoch)

    def indices(self):
        return self._impl.indices()


def make_sampler(kind: str, dataset, num_replicas, rank, shuffle=True, seed=0):
    kind = {"division": "partition"}.get(kind, kind)
    if kind == "partition":
        return PartitionSampler(dataset, num_replicas, rank, shuffle, seed)
    if kind in ("random", "sampling"):
        return RandomSampleSampler(dataset, num_replicas, rank, shuffle, seed)
    if kind == "bootstrap":
        return RandomSampleSampler(dataset, num_replicas, rank, shuffle, seed, replacement=True)
    raise ValueError(f"unknown sampler {kind!r}")
