"""Native NHWC bf16 pooling (ResNet stem max-pool, global average pool)."""
from __future__ import annotations

import torch

from ._native import lib
from .convbn import empty_nhwc


def maxpool_fwd(layer, x, ctx, train):
    N, H, W, C = x.shape
    k, s, p = layer.k, layer.stride, layer.padding
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    y = empty_nhwc(N, OH, OW, C, x)
    idx = torch.empty((N, OH, OW, C), device=x.device, dtype=torch.uint8)
    lib().maxpool_fwd(x, y, idx, k, s, p)
    if train:
        ctx.update(idx=idx, xshape=x.shape)
    return y


def maxpool_bwd(layer, dy, ctx, need_dx):
    if not need_dx:
        return None
    N, H, W, C = ctx["xshape"]
    dx = empty_nhwc(N, H, W, C, dy)
    lib().maxpool_bwd(dy.contiguous(), ctx["idx"], dx, layer.k, layer.stride, layer.padding)
    return dx


def avgpool_fwd(layer, x, ctx, train):
    N, H, W, C = x.shape
    y = torch.empty((N, C), device=x.device, dtype=torch.bfloat16)
    lib().avgpool_fwd(x, y)
    if train:
        ctx["xshape"] = x.shape
    return y


def avgpool_bwd(layer, dy, ctx, need_dx):
    if not need_dx:
        return None
    N, H, W, C = ctx["xshape"]
    dx = empty_nhwc(N, H, W, C, dy)
    lib().avgpool_bwd(dy.to(torch.bfloat16).contiguous(), dx)
    return dx
