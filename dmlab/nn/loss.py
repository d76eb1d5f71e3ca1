"""Cross-entropy loss (``nn.CrossEntropyLoss`` mean semantics).

On a HIP device one fused kernel computes the mean loss AND the logits gradient
(softmax − onehot)/B during the forward; backward only scales it
by the incoming gradient.  CPU tensors use ``F.cross_entropy``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        from dmlab.ops._native import lib

        logits = logits.contiguous()
        B = logits.shape[0]
        rowloss = torch.empty(B, device=logits.device, dtype=torch.float32)
        loss = torch.empty((), device=logits.device, dtype=torch.float32)
        need = ctx.needs_input_grad[0]
        dlogits = torch.empty_like(logits) if need else None
        lib().cross_entropy(logits, labels.contiguous(), rowloss, loss, dlogits, 1.0 / B)
        ctx.save_for_backward(dlogits if need else None)
        return loss

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        if d is None:
            return None, None
        return d * g.to(d.dtype), None


def cross_entropy(logits, labels):
    if logits.is_cuda:
        return _CEFn.apply(logits, labels)
    return F.cross_entropy(logits.float() if logits.dtype != torch.float32 else logits, labels)


class CrossEntropyLoss(nn.Module):
    def forward(self, logits, labels):
        return cross_entropy(logits, labels)


@torch.no_grad()
def count_correct(logits, labels, counter=None):
    """Add the number of correct argmax predictions to a device counter (int64)."""
    if counter is None:
        counter = torch.zeros((), device=logits.device, dtype=torch.long)
    if logits.is_cuda:
        from dmlab.ops._native import lib

        lib().argmax_count(logits.contiguous(), labels.contiguous(), counter)
    else:
        counter += (logits.argmax(1) == labels).sum()
    return counter
