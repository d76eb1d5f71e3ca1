"""Native path of :class:`dmlab.nn.layers.Conv2d` for thin convolutions (LeNet).

Kernels: ``csrc/conv_small.hip`` (fused conv+bias+ReLU+pool2 forward; unpool /
backward-data / split-batch backward-weight).  Layout NCHW, activations fp32 or
bf16, weights read straight from the fp32 master (they are tiny)."""
from __future__ import annotations

import math

import torch

from ._native import lib


def _check(layer, x):
    if layer.stride != 1:
        raise NotImplementedError("native thin conv supports stride 1 (LeNet); use ConvBN for strided")
    if layer.k not in (3, 5):
        raise NotImplementedError(f"native thin conv supports k in (3,5), got {layer.k}")


def conv_fwd(layer, x, ctx, train):
    _check(layer, x)
    x = x.contiguous()
    B, C, H, W = x.shape
    k, p, pool = layer.k, layer.padding, layer.pool
    OH, OW = H + 2 * p - k + 1, W + 2 * p - k + 1
    y = torch.empty((B, layer.cout, OH // pool, OW // pool), device=x.device, dtype=x.dtype)
    mask = torch.empty(y.shape, device=x.device, dtype=torch.uint8) if pool > 1 else None
    lib().conv_small_fwd(x, layer.weight.detach(),
                         layer.bias.detach() if layer.bias is not None else None,
                         y, mask, p, pool, layer.relu)
    if train:
        ctx["x"], ctx["y"], ctx["mask"] = x, y, mask
    return y


def _batch_slice(B, cout, cin):
    target_blocks = 1024
    S = max(1, min(B, math.ceil(target_blocks / max(cout * cin, 1))))
    return max(1, math.ceil(B / S))


def conv_bwd(layer, dy, ctx, need_dx):
    x, y, mask = ctx["x"], ctx["y"], ctx["mask"]
    dy = dy.reshape(y.shape).to(y.dtype).contiguous()
    B, C, H, W = x.shape
    k, p = layer.k, layer.padding
    bs = _batch_slice(B, layer.cout, C)
    L = lib()
    work = torch.empty(L.conv_small_workspace(B, C, H, W, layer.cout, k, p, bs),
                       device=x.device, dtype=torch.float32)
    dx = torch.empty_like(x) if need_dx else None
    dw = layer.grad_slot("weight")
    db = layer.grad_slot("bias") if layer.bias is not None else None
    L.conv_small_bwd(x, layer.weight.detach(), dy, y, mask, dx, dw, db, work, p, layer.pool,
                     layer.relu, 1.0 if layer.accumulate else 0.0, bs)
    return dx
