"""One flat fp32 buffer for all parameters, one for all gradients.

Every parameter of a :class:`~dmlab.nn.program.Program` is re-pointed
(``param.data = view``) into a single contiguous fp32 buffer laid out in
*reverse execution order* (the order backward produces gradients), and
``param.grad`` is a view into a matching flat gradient buffer.  Consequences:

* the fused optimisers (``csrc/optim.hip``) update every parameter in ONE launch;
* data-parallel gradient buckets are contiguous slices of the grad buffer, so
  the RCCL all-reduce runs in place on them with no pack/unpack copies, and they
  become ready in order as backward proceeds (overlap);
* the bf16 compute copy of the weights is refreshed by one cast launch (or
  written directly by the fused optimiser).

Each slot is padded to 64 elements (256 B) so every view is 16-B aligned for
vector loads.
"""
from __future__ import annotations

import torch

ALIGN = 64


def _round(n, a=ALIGN):
    return (n + a - 1) // a * a


class FlatParams:
    def __init__(self, named_params, device, dtype=torch.float32):
        """named_params: ordered list of (qualified_name, nn.Parameter)."""
        self.names = [n for n, _ in named_params]
        self.params = [p for _, p in named_params]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _round(p.numel())
        self.numel = max(off, ALIGN)
        self.device = torch.device(device)
        self.data = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self.grad = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self._bf16 = None
        self._bf16_version = None
        self._ext_version = 0  # bumped by native optimisers that write via raw pointers
        self.grad_valid = False  # grads hold a complete, un-consumed gradient
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                v = self.data[o:o + p.numel()].view_as(p)
                v.copy_(p.data)
                p.data = v
                p._dm_flat = self
        self.attach_grads()

    # ------------------------------------------------------------ views
    def grad_view(self, i):
        p, o = self.params[i], self.offsets[i]
        return self.grad[o:o + p.numel()].view_as(p)

    def data_view(self, i):
        p, o = self.params[i], self.offsets[i]
        return self.data[o:o + p.numel()].view_as(p)

    def index_of(self, p):
        for i, q in enumerate(self.params):
            if q is p:
                return i
        raise KeyError("parameter not in flat buffer")

    def attached(self) -> bool:
        """True if every param.grad is still our view (no set_to_none happened)."""
        for i, p in enumerate(self.params):
            g = p.grad
            if g is None or g.data_ptr() != self.grad.data_ptr() + 4 * self.offsets[i]:
                return False
        return True

    def attach_grads(self):
        for i, p in enumerate(self.params):
            p.grad = self.grad_view(i)

    def prepare_backward(self) -> bool:
        """Called at the start of backward.  Returns True if gradients must be
        accumulated into the existing values (torch semantics when the caller did
        not zero / set_to_none the grads), False if they may be overwritten."""
        if not self.attached():
            self.attach_grads()
            self.grad_valid = False
        return self.grad_valid

    def mark_grads_consumed(self):
        """Our optimisers call this instead of zeroing: next backward overwrites."""
        self.grad_valid = False

    # ------------------------------------------------------------ bf16 shadow
    def version(self):
        """Changes whenever the fp32 master weights change (torch in-place ops bump
        ``_version``; native optimiser launches call :meth:`mark_updated`)."""
        # ``param.data = view`` keeps each Parameter's own version counter, so sum
        # them (a torch optimiser's in-place update bumps exactly one of these).
        return (sum(p._version for p in self.params), self.data._version, self._ext_version)

    def mark_updated(self):
        self._ext_version += 1

    def bf16(self) -> torch.Tensor:
        """bf16 copy of all weights, refreshed only when the fp32 master changed."""
        ver = self.version()
        if self._bf16 is None:
            self._bf16 = torch.empty(self.numel, device=self.device, dtype=torch.bfloat16)
        if ver != self._bf16_version:
            if self.device.type == "cuda":
                from dmlab.ops._native import lib

                lib().cast_f32_bf16(self.data, self._bf16)
            else:
                self._bf16.copy_(self.data)
            self._bf16_version = ver
        return self._bf16

    def bf16_view(self, i):
        p, o = self.params[i], self.offsets[i]
        return self.bf16()[o:o + p.numel()].view(p.shape)

    def shadow_written(self):
        """The fused optimiser wrote the bf16 shadow together with the fp32 update."""
        self._bf16_version = self.version()
