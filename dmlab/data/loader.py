"""Device-resident batch loader.

The reference iterates ``torch.utils.data.DataLoader`` on the host (PIL →
tensor per sample, ``num_workers=0``) and copies every batch with ``.cuda()``
(task1/pytorch/model.py:47, task2/model.py:52).  Here the whole
dataset lives on the device (MNIST is 188 MB fp32 — nothing against 288 GB of
HBM3E) and a batch is one ``index_select`` gather driven by the sampler's index
list, which is itself uploaded once per epoch.
"""
from __future__ import annotations

import torch


class DeviceLoader:
    def __init__(self, dataset, batch_size: int, sampler=None, shuffle: bool = False,
                 drop_last: bool = False, seed: int = 0, device=None):
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.sampler = sampler
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.seed = seed
        self.epoch = 0
        self.device = device if device is not None else dataset.images.device

    def set_epoch(self, epoch: int):
        self.epoch = epoch
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def _indices(self) -> torch.Tensor:
        if self.sampler is not None:
            if hasattr(self.sampler, "indices"):
                return self.sampler.indices()
            return torch.tensor(list(iter(self.sampler)), dtype=torch.long)
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            return torch.randperm(n, generator=g)
        return torch.arange(n)

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        idx = self._indices().to(self.device)
        n = idx.numel()
        bs = self.batch_size
        stop = (n // bs) * bs if self.drop_last else n
        for s in range(0, stop, bs):
            yield self.dataset.batch(idx[s: s + bs])
