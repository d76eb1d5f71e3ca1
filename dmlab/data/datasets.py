"""Datasets: synthetic MNIST/ImageNet-shaped data and an optional real-MNIST reader.

The reference downloads torchvision MNIST with ``ToTensor()`` only
(task1/pytorch/model.py:87-94, task2/model.py:107,118-122).  Neither torchvision
nor the network exist here, so the default is :class:`SyntheticMNIST`: a
deterministic, *learnable* (class-prototype + noise) dataset of the same shape
(1×28×28 in [0,1], labels 0-9, 60k train / 10k test).  :class:`MNIST` reads the
standard idx files if they are present under ``root`` (no download).

All datasets can be materialised directly on a device (``.to(device)``) so the
training loop gathers batches with one index-select per step instead of a
per-sample host DataLoader.
"""
from __future__ import annotations

import gzip
import struct
from pathlib import Path

import torch


class TensorDataset(torch.utils.data.Dataset):
    """(images, labels) held as two tensors; indexable like torchvision datasets."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor):
        assert images.shape[0] == labels.shape[0]
        self.images = images
        self.labels = labels

    def __len__(self):
        return self.images.shape[0]

    def __getitem__(self, i):
        return self.images[i], int(self.labels[i])

    def to(self, device, dtype=None, memory_format=None):
        im = self.images.to(device)
        if dtype is not None:
            im = im.to(dtype)
        if memory_format is not None:
            im = im.contiguous(memory_format=memory_format)
        return TensorDataset(im, self.labels.to(device))

    def batch(self, idx: torch.Tensor):
        """Gather a batch by index tensor (device-side when the data is on device)."""
        idx = idx.to(self.images.device, non_blocking=True)
        return self.images.index_select(0, idx), self.labels.index_select(0, idx)


def _prototypes(num_classes, shape, gen):
    # smooth class prototypes: low-frequency random fields, upsampled
    c, h, w = shape
    base = torch.rand(num_classes, c, max(h // 4, 1), max(w // 4, 1), generator=gen)
    proto = torch.nn.functional.interpolate(base, size=(h, w), mode="bilinear",
                                            align_corners=False)
    return proto


def synthetic_classification(n, shape, num_classes, seed, noise=0.35, sparse=True):
    """Learnable synthetic data: each class is a smooth random prototype; a sample
    is its prototype with per-pixel noise.  ``sparse=True`` thresholds the field
    into MNIST-like strokes on a zero background (mean intensity ~0.1)."""
    gen = torch.Generator().manual_seed(seed)
    proto_gen = torch.Generator().manual_seed(1234)  # prototypes shared by train/test
    proto = _prototypes(num_classes, shape, proto_gen)
    labels = torch.randint(0, num_classes, (n,), generator=gen)
    out = torch.empty((n,) + tuple(shape))
    chunk = 8192
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        nz = torch.rand((e - s,) + tuple(shape), generator=gen)
        f = (1 - noise) * proto[labels[s:e]] + noise * nz
        if sparse:
            f = ((f - 0.55) * 4.0).clamp_(0, 1)
        out[s:e] = f
    return TensorDataset(out.clamp_(0, 1), labels)


class SyntheticMNIST(TensorDataset):
    """MNIST-shaped synthetic data: (1,28,28) float in [0,1], labels 0..9."""

    def __init__(self, train: bool = True, n: int | None = None, seed: int = 0,
                 noise: float | None = None, label_noise: float | None = None):
        import os

        # difficulty (the lab report raises it so the comparisons do not all saturate at
        # 100 %): pixel noise mixed into the class prototype, and a fraction of labels
        # replaced by uniformly random ones (caps the reachable accuracy)
        if noise is None:
            noise = float(os.environ.get("DMLAB_SYNTH_NOISE", "0.35"))
        if label_noise is None:
            label_noise = float(os.environ.get("DMLAB_SYNTH_LABEL_NOISE", "0"))
        n = n if n is not None else (60000 if train else 10000)
        ds = synthetic_classification(n, (1, 28, 28), 10, seed + (0 if train else 99991), noise=noise)
        labels = ds.labels
        if label_noise > 0:
            g = torch.Generator().manual_seed(seed + 7 + (0 if train else 99991))
            flip = torch.rand(n, generator=g) < label_noise
            labels = torch.where(flip, torch.randint(0, 10, (n,), generator=g), labels)
        super().__init__(ds.images, labels)


# uint8 images (what a decoded JPEG pipeline delivers) are normalised as ImageNet RGB:
# x = (u / 255 - mean) / std per channel, by the first layer (the fused ResNet stem reads the
# bytes and normalises on the fly: dmlab.ops.convbn); fp32 / bf16 images are used as stored
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def input_affine(dtype):
    """(scale[3], bias[3]) with x = raw * scale + bias for an image tensor of ``dtype``."""
    if dtype == torch.uint8:
        return ([1.0 / (255.0 * s) for s in IMAGENET_STD],
                [-m / s for m, s in zip(IMAGENET_MEAN, IMAGENET_STD)])
    return [1.0, 1.0, 1.0], [0.0, 0.0, 0.0]


def normalize_input(x: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """The reference-path equivalent of the stem's on-the-fly normalisation ((N,3,H,W))."""
    if x.dtype != torch.uint8:
        return x
    sc, bi = input_affine(torch.uint8)
    sc = torch.tensor(sc, device=x.device, dtype=torch.float32).view(1, 3, 1, 1)
    bi = torch.tensor(bi, device=x.device, dtype=torch.float32).view(1, 3, 1, 1)
    return (x.float() * sc + bi).to(dtype)


class SyntheticImageNet(TensorDataset):
    """ImageNet-shaped synthetic data for the ResNet-18 benchmark.

    Generated directly on ``device`` (no host copy) with uniform pixels; the
    benchmark measures throughput, not accuracy (BASELINE.json: synthetic data,
    random-init weights).  ``dtype=torch.uint8`` stores decoded-image bytes (uniform in
    0..255), normalised by the model's first layer (:func:`input_affine`)."""

    def __init__(self, n: int, res: int = 224, num_classes: int = 1000, device="cpu",
                 dtype=torch.float32, channels_last=True, seed: int = 0):
        g = torch.Generator(device=device).manual_seed(seed)
        fmt = torch.channels_last if channels_last else torch.contiguous_format
        im = torch.rand((n, 3, res, res), generator=g, device=device, dtype=torch.float32)
        if dtype == torch.uint8:
            im = (im * 256.0).floor_().clamp_(0, 255)
        im = im.to(dtype).contiguous(memory_format=fmt)
        lb = torch.randint(0, num_classes, (n,), generator=g, device=device)
        super().__init__(im, lb)


def _read_idx(path: Path) -> torch.Tensor:
    op = gzip.open if path.suffix == ".gz" else open
    with op(path, "rb") as f:
        data = f.read()
    magic, = struct.unpack(">I", data[:4])
    ndim = magic & 0xFF
    dims = struct.unpack(">" + "I" * ndim, data[4:4 + 4 * ndim])
    t = torch.frombuffer(bytearray(data[4 + 4 * ndim:]), dtype=torch.uint8)
    return t.reshape(dims)


class MNIST(TensorDataset):
    """Real MNIST from idx files under ``root/MNIST/raw`` (torchvision layout) or
    ``root``.  No download (there is no network); raises FileNotFoundError."""

    FILES = {True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
             False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}

    def __init__(self, root="./data", train=True):
        root = Path(root)
        cands = [root / "MNIST" / "raw", root]
        imf, lbf = self.FILES[train]
        for d in cands:
            for suf in ("", ".gz"):
                a, b = d / (imf + suf), d / (lbf + suf)
                if a.exists() and b.exists():
                    im = _read_idx(a).float().div_(255.0).unsqueeze(1)  # ToTensor()
                    lb = _read_idx(b).long()
                    super().__init__(im, lb)
                    return
        raise FileNotFoundError(f"MNIST idx files not found under {root}")


def load_mnist(root="./data", train=True, synthetic: bool | None = None, n=None, seed=0):
    """Real MNIST if available (and synthetic is not forced), else synthetic."""
    if synthetic is not True:
        try:
            ds = MNIST(root, train)
            if n is not None:
                ds = TensorDataset(ds.images[:n], ds.labels[:n])
            return ds
        except FileNotFoundError:
            if synthetic is False:
                raise
    return SyntheticMNIST(train=train, n=n, seed=seed)
