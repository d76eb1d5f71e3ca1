"""Native path of :class:`dmlab.nn.layers.Linear` on the strided fp32-MFMA GEMM
(``csrc/gemm.hip``): bias + ReLU fused into the forward epilogue, the ReLU
backward fused into the operand loads of both backward GEMMs, bias gradient by a
column-sum kernel.  Weight gradients are written (or accumulated, beta=1)
directly into the flat gradient buffer.

bf16 activations (the ResNet classifier head, a plain 256x512x1000 GEMM) go to the
vendor library instead (hipBLASLt through ``torch.mm``, bf16 operands, fp32 weight
gradient via ``out_dtype``): the strided fp32-MFMA kernel is sized for LeNet's
tiny layers and reached only ~4 TFLOP/s on that shape."""
from __future__ import annotations

import torch

from ._native import lib


def _lib_path(layer, x):
    return x.dtype == torch.bfloat16 and not layer.relu


def linear_fwd(layer, x, ctx, train):
    B = x.shape[0]
    x2 = x.reshape(B, -1).contiguous()
    assert x2.shape[1] == layer.fin, (x2.shape, layer.fin)
    if _lib_path(layer, x2):
        w16 = layer.weight.detach().to(torch.bfloat16)
        if layer.bias is not None:
            y = torch.addmm(layer.bias.detach().to(torch.bfloat16), x2, w16.t())
        else:
            y = torch.mm(x2, w16.t())
        if train:
            ctx["x"], ctx["y"], ctx["xshape"], ctx["w16"] = x2, y, x.shape, w16
        return y
    y = torch.empty((B, layer.fout), device=x.device, dtype=x.dtype)
    w = layer.weight.detach()
    lib().gemm(x2, None, w, y, None, layer.bias.detach() if layer.bias is not None else None,
               B, layer.fout, layer.fin, layer.fin, 1, 1, layer.fin, layer.fout, 1.0, 0.0,
               layer.relu)
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
    if "w16" in ctx:
        gw = torch.mm(dy.t(), x, out_dtype=torch.float32)
        slot = layer.grad_slot("weight")
        if beta:
            slot.add_(gw)
        else:
            slot.copy_(gw)
        if layer.bias is not None:
            L.colsum(dy, None, layer.grad_slot("bias"), beta)
        if not need_dx:
            return None
        return torch.mm(dy, ctx["w16"]).reshape(ctx["xshape"])
    # dW[fout, fin] = dYᵀ · X
    L.gemm(dy, mask, x, None, layer.grad_slot("weight"), None, fout, fin, B, 1, fout, fin, 1, fin,
           1.0, beta, False)
    if layer.bias is not None:
        L.colsum(dy, mask, layer.grad_slot("bias"), beta)
    if not need_dx:
        return None
    dx = torch.empty((B, fin), device=x.device, dtype=x.dtype)
    L.gemm(dy, mask, layer.weight.detach(), dx, None, None, B, fin, fout, fout, 1, fin, 1, fin,
           1.0, 0.0, False)
    return dx.reshape(ctx["xshape"])
