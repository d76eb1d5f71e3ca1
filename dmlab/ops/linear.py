"""Native path of :class:`dmlab.nn.layers.Linear` on the strided fp32-MFMA GEMM
(``csrc/gemm.hip``): bias + ReLU fused into the forward epilogue, the ReLU
backward fused into the operand loads of both backward GEMMs, bias gradient by a
column-sum kernel.  Weight gradients are written (or accumulated, beta=1)
directly into the flat gradient buffer.

bf16 activations (the ResNet classifier head) run the same strided GEMM on bf16 MFMA
(``lowp``: ``v_mfma_f32_16x16x32_bf16``, the fp32 master weight rounded to bf16 while it
is staged, fp32 accumulation and fp32 weight gradient): the exact fp32-MFMA path is
4x slower per FLOP and only LeNet's fp32 numerics need it."""
from __future__ import annotations

import torch

from ._native import lib


def linear_fwd(layer, x, ctx, train):
    B = x.shape[0]
    x2 = x.reshape(B, -1).contiguous()
    assert x2.shape[1] == layer.fin, (x2.shape, layer.fin)
    y = torch.empty((B, layer.fout), device=x.device, dtype=x.dtype)
    w = layer.weight.detach()
    lib().gemm(x2, None, w, y, None, layer.bias.detach() if layer.bias is not None else None,
               B, layer.fout, layer.fin, layer.fin, 1, 1, layer.fin, layer.fout, 1.0, 0.0,
               layer.relu, lowp=x2.dtype == torch.bfloat16)
    if train:
        ctx["x"], ctx["y"], ctx["xshape"] = x2, y, x.shape
    return y


def linear_bwd(layer, dy, ctx, need_dx):
    x, y = ctx["x"], ctx["y"]
    dy = dy.to(y.dtype).contiguous()
    B, fin, fout = x.shape[0], layer.fin, layer.fout
    mask = y if layer.relu else None
    beta = 1.0 if layer.accumulate else 0.0
    L = lib()
    lowp = x.dtype == torch.bfloat16
    # dW[fout, fin] = dYᵀ · X
    L.gemm(dy, mask, x, None, layer.grad_slot("weight"), None, fout, fin, B, 1, fout, fin, 1, fin,
           1.0, beta, False, lowp=lowp)
    if layer.bias is not None:
        L.colsum(dy, mask, layer.grad_slot("bias"), beta)
    if not need_dx:
        return None
    dx = torch.empty((B, fin), device=x.device, dtype=x.dtype)
    L.gemm(dy, mask, layer.weight.detach(), dx, None, None, B, fin, fout, fout, 1, fin, 1, fin,
           1.0, 0.0, False, lowp=lowp)
    return dx.reshape(ctx["xshape"])
