"""Device-resident batch loader.

The reference iterates ``torch.utils.data.DataLoader`` on the host (PIL →
tensor per sample, ``num_workers=0``) and copies every batch with ``.cuda()``
(task1/pytorch/model.py:47, task2/model.py:52).  Here the whole
dataset lives on the device (MNIST is 188 MB fp32 — nothing against 288 GB of
HBM3E) and a batch is one ``index_select`` gather driven by the sampler's index
list, which is itself uploaded once per epoch.
"""
from __future__ import annotations

from typing import NamedTuple

import torch


class Gathered(NamedTuple):
    """A batch named by row indices into a device-resident dataset, not yet gathered.

    A consumer that can fuse the gather into its first pass takes it as is (the ResNet stem's
    space-to-depth packing reads ``images[idx[n]]`` directly: the batch is never copied);
    every other consumer calls :meth:`materialize` (one ``index_select``)."""

    images: torch.Tensor
    idx: torch.Tensor

    @property
    def shape(self):
        return (self.idx.numel(),) + tuple(self.images.shape[1:])

    @property
    def device(self):
        return self.images.device

    @property
    def is_cuda(self):
        return self.images.is_cuda

    def materialize(self) -> torch.Tensor:
        return self.images.index_select(0, self.idx)


class DeviceCursor:
    """The epoch's sampler order resident on the device plus a device-side batch cursor.

    For steps captured into a hipGraph: the graph reads batch ``cursor`` of ``order`` and
    advances the cursor itself (no per-step host work, not even an index copy).  ``refill``
    uploads the next epoch's order into the SAME buffer (captured pointers stay valid) and
    rewinds the cursor.  ``tail`` holds the shard's partial last batch (the indices past the
    whole batches; empty when the shard size is a multiple of the batch), refreshed with the
    order, for a loop that runs it as one uncaptured step (reference drop_last=False)."""

    def __init__(self, loader: "DeviceLoader"):
        self.loader = loader
        bs = loader.batch_size
        self.nbatch = len(loader.sampler if loader.sampler is not None else loader.dataset) // bs  # whole batches only (drop_last): a fixed batch shape
        if self.nbatch < 1:
            raise ValueError("the sampler's shard holds fewer than one batch")
        idx = loader._device_indices()
        self.order = idx[: self.nbatch * bs].contiguous()
        self.tail = idx[self.nbatch * bs:].contiguous()
        self.cursor = torch.zeros(1, dtype=torch.int32, device=loader.device)

    def refill(self, epoch: int):
        self.loader.set_epoch(epoch)
        idx = self.loader._device_indices()
        self.order.copy_(idx[: self.order.numel()])
        if self.tail.numel():
            self.tail.copy_(idx[self.order.numel(): self.order.numel() + self.tail.numel()])
        self.cursor.zero_()


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

    def _device_indices(self) -> torch.Tensor:
        """The epoch's index list on the loader's device.  Uploaded from pinned memory without
        blocking: a pageable copy would synchronise the stream once per epoch and drain the
        host's run-ahead of the GPU."""
        idx = self._indices()
        if self.device.type == "cuda":
            return idx.pin_memory().to(self.device, non_blocking=True)
        return idx.to(self.device)

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        idx = self._device_indices()
        n = idx.numel()
        bs = self.batch_size
        stop = (n // bs) * bs if self.drop_last else n
        for s in range(0, stop, bs):
            yield self.dataset.batch(idx[s: s + bs])

    def iter_gathered(self):
        """Like iteration, but yields ``(Gathered(images, idx), labels)``: the image gather is
        left to the consumer (fused into the ResNet stem's input packing); labels are
        gathered (B int64)."""
        idx = self._device_indices()
        n = idx.numel()
        bs = self.batch_size
        stop = (n // bs) * bs if self.drop_last else n
        im, lb = self.dataset.images, self.dataset.labels
        for s in range(0, stop, bs):
            sl = idx[s: s + bs]
            yield Gathered(im, sl), lb.index_select(0, sl)

    def cursor(self) -> DeviceCursor:
        """Device-resident epoch order + cursor, for hipGraph-captured steps."""
        return DeviceCursor(self)
