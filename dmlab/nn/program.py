"""Explicit forward/backward programs (the dmlab execution engine).

A :class:`Program` is an ``nn.Module`` whose layers each implement an explicit
``fwd``/``bwd`` pair.  The whole program runs as ONE autograd node
(:class:`_ProgramFn`): its backward walks the layers in reverse, writes weight
gradients *directly* into the flat gradient buffer (no AccumulateGrad copies),
and notifies a gradient hook after every layer so a data-parallel reducer can
launch bucket all-reduces while the remaining layers are still computing.

Each layer has two interchangeable implementations selected per call:

* ``native`` — hand-written HIP kernels (``dmlab._C``), used for every HIP
  device tensor.  If the extension is missing this raises; there is no silent
  fallback.
* ``torch``  — plain PyTorch ops through local autograd; the numerical
  reference and the CPU execution path (BASELINE config 1 is CPU-only).

Reference mapping: the reference models are plain ``nn.Module``s trained by
autograd (task1/pytorch/model.py:12-35, task4/model.py:18-47); a Program keeps
that user-facing contract (``out = model(x); loss.backward(); opt.step()``)
while replacing the per-op autograd graph with an explicit schedule.
"""
from __future__ import annotations

import collections
import contextlib
import os

from typing import Callable, Optional

import torch
import torch.nn as nn

from .flat import FlatParams


class Ctx(dict):
    """Per-call saved state of one layer (activations, masks, stats)."""


class Layer(nn.Module):
    """Base class: subclasses define parameters in ``__init__`` and implement
    ``torch_forward`` (reference) and optionally ``native_fwd``/``native_bwd``."""

    native_ok = True  # False: layer has no native kernels yet (torch path on GPU is an error)

    def __init__(self):
        super().__init__()
        self._prog: Optional["Program"] = None
        self._pidx: dict[str, int] = {}

    # ---------------------------------------------------------------- helpers
    def grad_slot(self, name: str) -> torch.Tensor:
        return self._prog.flat.grad_view(self._pidx[name])

    def write_grad(self, name: str, g: torch.Tensor):
        slot = self.grad_slot(name)
        if self._prog._accumulate:
            slot.add_(g.reshape(slot.shape).to(slot.dtype))
        else:
            slot.copy_(g.reshape(slot.shape))

    @property
    def accumulate(self) -> bool:
        return self._prog._accumulate

    # ---------------------------------------------------------------- torch reference path
    def torch_forward(self, x: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def t_fwd(self, x, ctx: Ctx, train: bool):
        if not train:
            with torch.no_grad():
                return self.torch_forward(x)
        xi = x.detach().requires_grad_(x.is_floating_point())
        with torch.enable_grad():
            y = self.torch_forward(xi)
        ctx["x"], ctx["y"] = xi, y
        return y.detach()

    def t_bwd(self, dy, ctx: Ctx, need_dx: bool):
        xi, y = ctx["x"], ctx["y"]
        names = [n for n, p in self.named_parameters(recurse=True) if p.requires_grad]
        params = [self.get_parameter(n) for n in names]
        inputs = ([xi] if need_dx and xi.requires_grad else []) + params
        if not inputs:
            return None
        grads = torch.autograd.grad(y, inputs, dy, allow_unused=True)
        dx = grads[0] if (need_dx and xi.requires_grad) else None
        pg = grads[1:] if dx is not None else grads
        for n, g in zip(names, pg):
            if g is not None:
                self._prog._write_grad_by_param(self.get_parameter(n), g)
        return dx

    # ---------------------------------------------------------------- dispatch
    def fwd(self, x, ctx: Ctx, train: bool):
        if self._prog._use_native(x):
            return self.native_fwd(x, ctx, train)
        return self.t_fwd(x, ctx, train)

    def bwd(self, dy, ctx: Ctx, need_dx: bool):
        if self._prog._use_native(dy):
            return self.native_bwd(dy, ctx, need_dx)
        return self.t_bwd(dy, ctx, need_dx)

    def native_fwd(self, x, ctx, train):  # pragma: no cover - overridden
        raise NotImplementedError(f"{type(self).__name__} has no native forward")

    def native_bwd(self, dy, ctx, need_dx):  # pragma: no cover - overridden
        raise NotImplementedError(f"{type(self).__name__} has no native backward")

    def forward(self, x):  # standalone use (e.g. inside a plain nn.Module)
        return self.torch_forward(x)


_ROCTX = os.environ.get("DMLAB_ROCTX", "0") == "1"


@contextlib.contextmanager
def _range(name):
    """roctx range (``DMLAB_ROCTX=1``) around a layer's forward/backward, visible in
    ``rocprofv3 --marker-trace``; a no-op otherwise."""
    if not _ROCTX:
        yield
        return
    torch.cuda.nvtx.range_push(name)  # ROCm builds of torch route nvtx to roctx
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


class _ProgramFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, prog):
        ctxs = []
        h = x
        for li, layer in enumerate(prog.layers):
            c = Ctx()
            with _range(f"fwd:{li}:{type(layer).__name__}"):
                h = layer.fwd(h, c, True)
            ctxs.append(c)
        ctx.prog = prog
        ctx.ctxs = ctxs
        ctx.need_dx = isinstance(x, torch.Tensor) and x.requires_grad
        return h

    @staticmethod
    def backward(ctx, dy):
        prog = ctx.prog
        prog._accumulate = prog.flat.prepare_backward()
        dy = dy.contiguous() if not prog._native_active else dy
        n = len(prog.layers)
        # Weight gradients off the critical path: layers that support it (ConvBN) queue
        # their wgrad on a second stream, which overlaps the data-gradient / BN-backward
        # chain of the following layers (the chain is a sequence of short and latency-
        # bound kernels that leave CUs idle).  A layer's grad hooks (DDP bucket launches)
        # run one layer later, after the main stream has waited for that layer's wgrads.
        side = prog._side_stream() if prog._native_active else None
        main = torch.cuda.current_stream() if side is not None else None
        if side is not None:
            side.wait_stream(main)  # fork (under hipGraph capture: joins the capture)
        prog._wgrad_stream = side
        pending = []  # (layer index, event after its wgrads) whose hooks have not run
        pending_main = []  # layers whose hooks run on the main stream after the join

        # Hooks registered stream_ok (DDP without a communication-dtype copy) are issued on
        # the side stream once it has caught up with the main stream: the collective they
        # launch is then ordered after the layer's weight gradients (side) and its other
        # parameter gradients (main) without the main stream ever waiting on the side
        # stream.  Other hooks keep the one-layer-lag scheme (main waits on the wgrad event),
        # which left 400-460 us of main-stream gaps per ResNet-18 step.
        side_hooks = side is not None and bool(prog._grad_hooks) and all(
            prog._hook_stream_ok.get(h, False) for h in prog._grad_hooks)

        def run_side_hooks(js):
            # a layer whose hooks enqueue nothing (no bucket completes there) runs them as
            # host bookkeeping: no event on the main stream, no side-stream wait (each costs
            # a few us of command-processor time between the main stream's kernels)
            if not any(prog._hook_enqueues(h, j) for j in js for h in prog._grad_hooks):
                for j in js:
                    for hook in prog._grad_hooks:
                        hook(prog, j)
                return
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for j in js:
                    for hook in prog._grad_hooks:
                        hook(prog, j)

        try:
            for i in range(n - 1, -1, -1):
                layer = prog.layers[i]
                need_dx = i > 0 or ctx.need_dx
                # the layer whose output gradient this one produces (its backward runs next):
                # layers may fold that layer's BN-backward reduction into their last kernel
                layer._bwd_next = (prog.layers[i - 1], ctx.ctxs[i - 1]) if i > 0 else None
                try:
                    with _range(f"bwd:{i}:{type(layer).__name__}"):
                        dy = layer.bwd(dy, ctx.ctxs[i], need_dx)
                finally:
                    layer._bwd_next = None
                ctx.ctxs[i] = None  # free saved activations as soon as possible
                if side is None:
                    for hook in prog._grad_hooks:
                        hook(prog, i)
                    continue
                if side_hooks:
                    if i == 0:
                        # the step's last layer: its hooks run on the main stream after the
                        # side stream's join below, so the final bucket's collective is
                        # ordered by that one join instead of main -> side -> comm -> main
                        # (each cross-queue hop ~25 us on MI355X: profiles/forcecomm_tail_r6.txt)
                        pending_main.append(i)
                        continue
                    run_side_hooks([i])
                    continue
                for j, ev in pending:
                    main.wait_event(ev)
                    for hook in prog._grad_hooks:
                        hook(prog, j)
                pending = []
                if prog._grad_hooks:
                    ev = torch.cuda.Event()
                    ev.record(side)
                    pending.append((i, ev))
        finally:
            prog._wgrad_stream = None
        if side is not None:
            main.wait_stream(side)
            if prog.max_inflight > 0 and not torch.cuda.is_current_stream_capturing():
                ev = torch.cuda.Event()
                ev.record(main)
                prog._inflight.append(ev)
            for j, _ in pending:
                for hook in prog._grad_hooks:
                    hook(prog, j)
            # hooks called here run with every gradient already ordered before the current
            # (main) stream: ``tail_hook`` tells a reducer it may issue its collective on
            # this stream directly (no communication-stream hop)
            prog.tail_hook = True
            try:
                for j in pending_main:
                    for hook in prog._grad_hooks:
                        hook(prog, j)
            finally:
                prog.tail_hook = False
        prog.flat.grad_valid = True
        for hook in prog._post_backward_hooks:
            hook(prog)
        return (dy if ctx.need_dx else None), None, None


class Program(nn.Module):
    """A sequence of :class:`Layer` objects with flat parameters.

    Subclasses build their layers and call :meth:`build` with the execution
    order.  ``backend``: ``"auto"`` (native on HIP tensors, torch on CPU),
    ``"torch"`` (reference ops everywhere, used for parity tests and for the
    stock-PyTorch comparison) or ``"native"`` (error on CPU).
    """

    def __init__(self):
        super().__init__()
        self.layers: list[Layer] = []
        self.flat: Optional[FlatParams] = None
        self.backend = "auto"
        self.compute_dtype = torch.float32
        self._accumulate = False
        self._native_active = False
        self._grad_hooks: list[Callable] = []
        # hook -> may run on the side stream (keyed by the hook object itself, not its id: a
        # removed hook's id could be reused by an unrelated function)
        self._hook_stream_ok: dict[Callable, bool] = {}
        # hook -> predicate(layer index): does the hook enqueue device work for that layer
        # (absent: always assumed to)
        self._hook_enqueues_pred: dict[Callable, Callable] = {}
        self._post_backward_hooks: list[Callable] = []
        self._anchor = torch.zeros(1, requires_grad=True)
        self._wver = None
        self._uses_side_stream = False  # set by subclasses whose layers queue wgrads aside
        self._side_streams = {}
        self._wgrad_stream = None
        self.tail_hook = False  # True while grad hooks run on the main stream after the join
        # Events at the end of the last backward passes (two-stream programs).  Tensors one
        # stream hands to the other are freed with the caching allocator's cross-stream
        # events, which only complete when the GPU reaches them: with the host free to run
        # many steps ahead, those blocks pile up (ResNet-18 b1024: 9 GB allocated, 95-110 GB
        # reserved, and a box with less free memory hit allocator retries at 195 ms/step).
        # forward() waits for the backward `max_inflight` steps back, which keeps the host
        # ahead of the GPU (a step enqueues in a fraction of its GPU time) but bounds that.
        self._inflight = collections.deque()
        self.max_inflight = int(os.environ.get("DMLAB_MAX_INFLIGHT", "2"))

    # ---------------------------------------------------------------- construction
    def build(self, layers):
        object.__setattr__(self, "layers", list(layers))  # order list (modules are attrs)
        for layer in self.layers:
            for m in layer.modules():
                if isinstance(m, Layer):
                    object.__setattr__(m, "_prog", self)
        self._flatten()
        return self

    def _flatten(self):
        # reverse execution order: the first bucket to become ready in backward
        # (last layer's grads) is at offset 0.
        named = []
        seen = set()
        for layer in reversed(self.layers):
            for n, p in layer.named_parameters():
                if id(p) not in seen:
                    seen.add(id(p))
                    named.append((n, p))
        device = named[0][1].device if named else torch.device("cpu")
        self.flat = FlatParams(named, device)
        index = {id(p): i for i, (_, p) in enumerate(named)}
        for layer in self.layers:
            for m in layer.modules():
                if isinstance(m, Layer):
                    m._pidx = {n: index[id(p)] for n, p in m.named_parameters(recurse=False)}
        self._param_index = index

    def _write_grad_by_param(self, p, g):
        slot = self.flat.grad_view(self._param_index[id(p)])
        if self._accumulate:
            slot.add_(g.reshape(slot.shape))
        else:
            slot.copy_(g.reshape(slot.shape))

    def _apply(self, fn, *args, **kwargs):
        super()._apply(fn, *args, **kwargs)
        if self.flat is not None:
            self._flatten()  # re-flatten after .to()/.cuda()
        self._anchor = self._anchor.detach().to(self.flat.device if self.flat else "cpu")
        self._anchor.requires_grad_(True)
        return self

    def set_backend(self, backend: str):
        assert backend in ("auto", "torch", "native")
        self.backend = backend
        return self

    def set_dtype(self, dtype):
        """Compute dtype of the native path (fp32 master weights are kept)."""
        self.compute_dtype = dtype
        return self

    def _use_native(self, t: torch.Tensor) -> bool:
        if self.backend == "torch":
            return False
        if t.is_cuda:  # a tensor, or a not-yet-gathered loader batch (dmlab.data.Gathered)
            return True
        if self.backend == "native":
            raise RuntimeError("native backend requested for a CPU tensor")
        return False

    # ---------------------------------------------------------------- hooks
    def _hook_enqueues(self, fn, layer_idx) -> bool:
        pred = self._hook_enqueues_pred.get(fn)
        return True if pred is None else bool(pred(layer_idx))

    def register_grad_hook(self, fn, stream_ok: bool = False, enqueues=None):
        """fn(program, layer_index) after layer i wrote its weight gradients.

        stream_ok: fn only enqueues stream-ordered device work on the current stream (e.g.
        collectives over the layer's gradient buckets) and keeps no tensor it allocates past
        the call; with a two-stream backward it is then called with the weight-gradient
        stream current, once that stream has caught up with the main stream, so the main
        stream never waits for it.  ``enqueues(layer_index) -> bool``: whether fn enqueues
        device work for that layer (False: it runs as host bookkeeping, no stream join)."""
        self._grad_hooks.append(fn)
        self._hook_stream_ok[fn] = bool(stream_ok)
        if enqueues is not None:
            self._hook_enqueues_pred[fn] = enqueues

    def remove_grad_hook(self, fn):
        self._grad_hooks.remove(fn)
        if fn not in self._grad_hooks:
            self._hook_stream_ok.pop(fn, None)
            self._hook_enqueues_pred.pop(fn, None)

    def register_post_backward_hook(self, fn):
        self._post_backward_hooks.append(fn)

    def layer_params(self, i):
        return [self._param_index[id(p)] for p in self.layers[i].parameters()]

    # ---------------------------------------------------------------- execution
    # the first layer's native forward reads a dmlab.data.Gathered batch straight from the
    # dataset (subclasses whose stem fuses the loader gather set this)
    accepts_gathered = False

    def forward(self, x):
        if not isinstance(x, torch.Tensor) and hasattr(x, "materialize"):
            if not (self.accepts_gathered and self._use_native(x)):
                x = x.materialize()
        self._native_active = self._use_native(x)
        if self._inflight and not torch.cuda.is_current_stream_capturing():
            while len(self._inflight) >= max(1, self.max_inflight):
                self._inflight.popleft().synchronize()
        if self._native_active:
            self._wver = self.flat.version()  # packed-weight caches key on this
            self.prepare_native(x)
        if self.training and torch.is_grad_enabled():
            return _ProgramFn.apply(x, self._anchor, self)
        h = x
        for layer in self.layers:
            h = layer.fwd(h, Ctx(), False)
        return h

    def _side_stream(self):
        """Second HIP stream for off-critical-path backward work (weight gradients), or
        None when disabled (``DMLAB_WGRAD_STREAM=0``) or no layer uses it."""
        if not self._uses_side_stream or os.environ.get("DMLAB_WGRAD_STREAM", "1") == "0":
            return None
        dev = torch.cuda.current_device()
        st = self._side_streams.get(dev)
        if st is None:
            # default priority (a higher-priority side stream measured -1.2 %:
            # profiles/bench_ab_side_stream_knobs_r3.jsonl)
            # (a CU-masked side stream measured slower at 50-75 % of the CUs:
            # profiles/wgrad_blocks_sidemask_ab_r4m.txt)
            st = self._side_streams[dev] = torch.cuda.Stream(device=dev)
        return st

    def _aux_stream(self):
        """Third HIP stream, at the step stream's high priority, for critical-path work that
        can run beside the main chain (a projection shortcut's BN backward); None when
        disabled (``DMLAB_AUX_STREAM=0``) or without a side stream."""
        if self._side_stream() is None or os.environ.get("DMLAB_AUX_STREAM", "1") == "0":
            return None
        dev = torch.cuda.current_device()
        key = ("aux", dev)
        st = self._side_streams.get(key)
        if st is None:
            lo, hi = torch.cuda.Stream.priority_range()
            st = self._side_streams[key] = torch.cuda.Stream(device=dev, priority=min(lo, hi))
        return st

    def prepare_native(self, x):
        """Hook for subclasses: convert input layout / refresh packed weights."""
