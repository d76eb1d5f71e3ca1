"""Optimisers: the reference's hand-written GD/Adam plus torch-compatible SGD.

Reference: ``BaseOptimizer``/``GdOptimizer``/``AdamOptimizer``
(codes/task1/pytorch/MyOptimizer.py:3-43) and ``torch.optim.SGD(lr, momentum=.9)``
(task2/model.py:131, task3/model.py:118).

When the parameters are exactly the parameters of one :class:`~dmlab.nn.program.Program`
(one flat buffer), a step is ONE fused kernel launch over the flat buffer
(``csrc/optim.hip``) on a HIP device, or a handful of vectorised torch ops on the
CPU.  Any other parameter set (e.g. a plain ``nn.Module``) takes the
per-tensor path with the same formulas.

``grad_scale`` multiplies the gradient inside the step — the data-parallel
1/world_size average is folded in there instead of a separate divide kernel
(SURVEY K24).  It is runtime configuration owned by DDP, so it is not part of
``state_dict``.
"""
from __future__ import annotations

import torch


def _flat_of(params):
    """Return the FlatParams owning exactly `params`, or None."""
    from dmlab.nn.flat import FlatParams  # noqa: F401

    owners = set()
    for p in params:
        f = getattr(p, "_dm_flat", None)
        if f is None:
            return None
        owners.add(id(f))
    if len(owners) != 1:
        return None
    flat = params[0]._dm_flat
    if len(flat.params) != len(params) or {id(p) for p in flat.params} != {id(p) for p in params}:
        return None
    return flat


class BaseOptimizer:
    """Reference API: holds ``list(params)`` and ``lr``; ``zero_grad`` detaches
    and zeros each grad (MyOptimizer.py:11-15)."""

    def __init__(self, params, lr=0.001):
        self.params = [p for p in params]
        if self.params and isinstance(self.params[0], dict):
            raise TypeError("parameter groups are not supported; pass a parameter iterable")
        # one persistent group dict: `for g in opt.param_groups: g["lr"] = x` (the usual LR
        # schedule idiom) writes straight into the value step() reads
        self._groups = [{"params": self.params, "lr": lr}]
        # runtime data-parallel config (DDP.fold_average_into sets 1/ws), NOT optimiser
        # state: it is neither saved nor restored, so a resume on another world size
        # (or without DDP) does not inherit a stale 1/N factor
        self.grad_scale = 1.0
        self.flat = _flat_of(self.params)
        self.step_count = 0

    @property
    def lr(self):
        return self._groups[0]["lr"]

    @lr.setter
    def lr(self, v):
        self._groups[0]["lr"] = v

    @property
    def param_groups(self):  # one group: enough for manual LR schedules and logging
        return self._groups

    def step(self):
        raise NotImplementedError

    def zero_grad(self, set_to_none: bool = False):
        if self.flat is not None and self.flat.attached():
            # gradients are views of the flat buffer; the next Program backward
            # overwrites them instead of accumulating -> no memset needed
            self.flat.mark_grads_consumed()
            if self.flat.device.type == "cpu":
                self.flat.grad.zero_()
            return
        for p in self.params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.detach_()
                    p.grad.zero_()

    def _native(self):
        return self.flat is not None and self.flat.device.type == "cuda"

    def _state_tensors(self):
        return {}

    def state_dict(self):
        sd = {"lr": self.lr, "step_count": self.step_count}
        sd.update({k: v.detach().clone() for k, v in self._state_tensors().items()
                   if v is not None})
        return sd

    def load_state_dict(self, sd):
        self.lr = sd["lr"]
        self.step_count = sd.get("step_count", 0)
        # a "grad_scale" key written by older checkpoints is ignored on purpose (see __init__)
        for k, t in self._state_tensors().items():
            if t is not None and k in sd:
                with torch.no_grad():
                    t.copy_(sd[k])


class GdOptimizer(BaseOptimizer):
    """p ← p − lr·g (MyOptimizer.py:18-24). SGD when fed mini-batches."""

    def step(self):
        self.step_count += 1
        if self._native():
            from dmlab.ops._native import lib

            f = self.flat
            lib().sgd_step(f.data, f.grad, None, None, self.lr, 0.0, 0.0, 0.0,
                           self.grad_scale, False, False)
            f.mark_updated()
            return
        with torch.no_grad():
            if self.flat is not None:
                self.flat.data.sub_(self.flat.grad, alpha=self.lr * self.grad_scale)
                return
            for p in self.params:
                if p.grad is not None:
                    p.data = p.data - self.lr * self.grad_scale * p.grad


class AdamOptimizer(BaseOptimizer):
    """Adam exactly as the reference writes it (MyOptimizer.py:26-43):
    m ← b1·m + (1−b1)·g ; v ← b2·v + (1−b2)·g² ; p ← p − lr/(√v+ε)·m.
    No bias correction by default; ``bias_correction=True`` gives
    textbook Adam."""

    def __init__(self, params, lr=0.001, b1=0.9, b2=0.999, epsilon=1e-8,
                 bias_correction=False, weight_decay=0.0):
        super().__init__(params, lr)
        self.beta1, self.beta2, self.epsilon = b1, b2, epsilon
        self.bias_correction = bias_correction
        self.weight_decay = weight_decay
        if self.flat is not None:
            self.m = torch.zeros_like(self.flat.data)
            self.v = torch.zeros_like(self.flat.data)
        else:
            self.momentums = [torch.zeros_like(p) for p in self.params]
            self.velocities = [torch.zeros_like(p) for p in self.params]

    def _state_tensors(self):
        if self.flat is not None:
            return {"m": self.m, "v": self.v}
        d = {f"m{i}": t for i, t in enumerate(self.momentums)}
        d.update({f"v{i}": t for i, t in enumerate(self.velocities)})
        return d

    def _bc(self):
        t = self.step_count
        if not self.bias_correction:
            return 1.0, 1.0
        return 1.0 / (1 - self.beta1 ** t), 1.0 / (1 - self.beta2 ** t)

    def step(self):
        self.step_count += 1
        bc1, bc2 = self._bc()
        b1, b2, eps, lr = self.beta1, self.beta2, self.epsilon, self.lr
        if self._native():
            from dmlab.ops._native import lib

            f = self.flat
            lib().adam_step(f.data, f.grad, self.m, self.v, None, lr, b1, b2, eps,
                            self.weight_decay, self.grad_scale, bc1, bc2)
            f.mark_updated()
            return
        with torch.no_grad():
            if self.flat is not None:
                pairs = [(self.flat.data, self.flat.grad, self.m, self.v)]
            else:
                pairs = [(p, p.grad, m, v) for p, m, v in
                         zip(self.params, self.momentums, self.velocities) if p.grad is not None]
            for p, g, m, v in pairs:
                g = g * self.grad_scale
                if self.weight_decay:
                    g = g + self.weight_decay * p
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                p.sub_(lr * (m * bc1) / ((v * bc2).sqrt() + eps))


class SGD(BaseOptimizer):
    """torch.optim.SGD semantics (momentum, dampening, nesterov, weight decay)."""

    def __init__(self, params, lr=0.01, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False):
        super().__init__(params, lr)
        self.momentum, self.dampening = momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        if self.flat is not None:
            self.buf = torch.zeros_like(self.flat.data) if momentum else None
        else:
            self.bufs = [None] * len(self.params)

    def _state_tensors(self):
        if self.flat is not None:
            return {"buf": self.buf}
        return {f"buf{i}": b for i, b in enumerate(self.bufs)}

    def load_state_dict(self, sd):
        if self.flat is None:  # per-tensor buffers are created lazily: materialise them
            for i, p in enumerate(self.params):
                if f"buf{i}" in sd and self.bufs[i] is None:
                    self.bufs[i] = torch.zeros_like(p)
        super().load_state_dict(sd)

    def step(self):
        self.step_count += 1
        first = self.step_count == 1
        if self._native():
            from dmlab.ops._native import lib

            f = self.flat
            lib().sgd_step(f.data, f.grad, self.buf, None, self.lr, self.momentum,
                           self.dampening, self.weight_decay, self.grad_scale,
                           self.nesterov, first)
            f.mark_updated()
            return
        with torch.no_grad():
            if self.flat is not None:
                items = [(self.flat.data, self.flat.grad, 0)]
            else:
                items = [(p, p.grad, i) for i, p in enumerate(self.params) if p.grad is not None]
            for p, g, i in items:
                d = g * self.grad_scale
                if self.weight_decay:
                    d = d + self.weight_decay * p
                if self.momentum:
                    if self.flat is not None:
                        if first:
                            self.buf.copy_(d)
                        else:
                            self.buf.mul_(self.momentum).add_(d, alpha=1 - self.dampening)
                        b = self.buf
                    else:
                        b = self.bufs[i]
                        if b is None:
                            b = self.bufs[i] = d.clone()
                        else:
                            b.mul_(self.momentum).add_(d, alpha=1 - self.dampening)
                    d = d + self.momentum * b if self.nesterov else b
                p.sub_(d, alpha=self.lr)
