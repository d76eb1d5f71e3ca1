"""Gradient aggregation primitives (lab 2) — the reference ``dist_utils`` API.

Reference (codes/task2/dist_utils.py:33-49, task3/dist_utils.py:33-46):

* ``init_parameters``            8 × ``broadcast(param, 0)``             (X1)
* ``allreduce_average_gradients`` 8 × ``all_reduce(SUM)`` + 8 × ``/= ws``  (X2, X3)
* ``allgather_average_gradients`` 8 × ``all_gather`` into a list that aliases
  ONE tensor twice → every rank gets the last rank's gradient, ws hard-coded to 2
                                                           (X4)

Here every primitive is *coalesced*: a :class:`~dmlab.nn.program.Program` keeps
all grads in one flat buffer, so an aggregation is ONE collective over it (RCCL
over xGMI on MI355X; gloo on CPU).  The average uses ``ReduceOp.AVG`` on RCCL
(no separate divide kernel) and SUM×(1/ws) on gloo.  All-gather aggregation is
correct for any world size: ``all_gather_into_tensor`` into ``[ws, N]`` then one
HIP row-mean kernel (K25).  ``granularity="per_param"`` reproduces the
reference's one-collective-per-tensor call pattern for the comm-cost comparison.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from . import env


def _flat_of_model(model):
    return getattr(model, "flat", None)


def _grads(model):
    return [p.grad for p in model.parameters() if p.grad is not None]


def _flatten(ts):
    return torch._utils._flatten_dense_tensors(ts)


def _unflatten_into(flat, ts):
    for t, s in zip(ts, torch._utils._unflatten_dense_tensors(flat, ts)):
        t.copy_(s)


def _is_nccl():
    return env.is_initialized() and dist.get_backend() == "nccl"


_AVG_OK = None


def avg_supported() -> bool:
    """Whether the backend implements ReduceOp.AVG (RCCL: ncclAvg).  Probed once
    with a 1-element collective; gloo never does."""
    global _AVG_OK
    if _AVG_OK is None:
        _AVG_OK = False
        if _is_nccl():
            try:
                t = torch.ones(1, device=env.device())
                dist.all_reduce(t, op=dist.ReduceOp.AVG)
                _AVG_OK = abs(t.item() - 1.0) < 1e-6
            except Exception:
                _AVG_OK = False
    return _AVG_OK


def all_reduce_mean_(t: torch.Tensor, async_op=False):
    ws = env.get_world_size()
    if ws == 1:
        return None
    if avg_supported():
        return dist.all_reduce(t, op=dist.ReduceOp.AVG, async_op=async_op)
    w = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=async_op)
    if async_op:
        return _ScaleAfter(w, t, 1.0 / ws)
    t.mul_(1.0 / ws)
    return None


class _ScaleAfter:
    """Async handle whose wait() also applies the 1/ws scale (gloo has no AVG)."""

    def __init__(self, work, t, s):
        self.work, self.t, self.s = work, t, s

    def wait(self):
        self.work.wait()
        self.t.mul_(self.s)
        return True


# ------------------------------------------------------------------ reference API
def dist_init(world_size, rank, master_addr="localhost", master_port="12355", backend=None):
    """Reference signature (task2/dist_utils.py:6); torchrun env wins if present."""
    if master_addr == "localhost":
        master_addr = "127.0.0.1"
    env.init(world_size, rank, master_addr, master_port, backend=backend)
    return True


def get_local_rank():
    return env.get_local_rank()


def get_rank():
    return env.get_rank()


def get_world_size():
    return env.get_world_size()


@torch.no_grad()
def init_parameters(model, src: int = 0, buffers: bool = True, force: bool = False):
    """Broadcast rank-``src`` parameters (and BN buffers) to every rank in ONE
    collective over the flat buffer (reference: one broadcast per tensor).  ``force``:
    broadcast through an initialised 1-rank group too (exercises the collective path)."""
    if env.get_world_size() <= 1 and not (force and env.is_initialized()):
        return
    flat = _flat_of_model(model)
    if flat is not None:
        dist.broadcast(flat.data, src)
        if hasattr(flat, "mark_updated"):
            flat.mark_updated()
    else:
        ps = [p.data for p in model.parameters()]
        if ps:
            f = _flatten(ps)
            dist.broadcast(f, src)
            _unflatten_into(f, ps)
    if buffers:
        bs = [b for b in model.buffers() if b.is_floating_point()]
        if bs:
            f = _flatten(bs)
            dist.broadcast(f, src)
            _unflatten_into(f, bs)


@torch.no_grad()
def allreduce_average_gradients(model, granularity: str = "flat", average: bool = True,
                                force: bool = False):
    ws = env.get_world_size()
    if ws <= 1 and not (force and env.is_initialized()):
        return
    flat = _flat_of_model(model)
    if granularity == "per_param":
        for g in _grads(model):  # reference call pattern (X2/X3)
            dist.all_reduce(g, op=dist.ReduceOp.SUM)
            if average:
                g.div_(ws)
        return
    if flat is not None and flat.attached():
        buf = flat.grad
        if average:
            all_reduce_mean_(buf)
        else:
            dist.all_reduce(buf)
        return
    gs = _grads(model)
    if not gs:
        return
    f = _flatten(gs)
    if average:
        all_reduce_mean_(f)
    else:
        dist.all_reduce(f)
    _unflatten_into(f, gs)


average_gradients = allreduce_average_gradients


@torch.no_grad()
def allgather_average_gradients(model, granularity: str = "flat", force: bool = False):
    """Correct all-gather mean for any world size (fixes SURVEY B1)."""
    ws = env.get_world_size()
    if ws <= 1 and not (force and env.is_initialized()):
        return
    flat = _flat_of_model(model)
    if granularity == "per_param":
        for g in _grads(model):
            parts = [torch.empty_like(g) for _ in range(ws)]  # distinct buffers
            dist.all_gather(parts, g)
            g.copy_(torch.stack(parts).mean(0))
        return
    if flat is not None and flat.attached():
        src = flat.grad
        gathered = torch.empty((ws, src.numel()), device=src.device, dtype=src.dtype)
        _all_gather_rows(gathered, src)
        _rows_mean(gathered, src)
        return
    gs = _grads(model)
    f = _flatten(gs)
    gathered = torch.empty((ws, f.numel()), device=f.device, dtype=f.dtype)
    _all_gather_rows(gathered, f)
    _rows_mean(gathered, f)
    _unflatten_into(f, gs)


def _all_gather_rows(gathered, src):
    """[ws, N] <- every rank's src; one RCCL all_gather_into_tensor (gloo: list form
    into row views, still one collective)."""
    if _is_nccl():
        dist.all_gather_into_tensor(gathered, src)
    else:
        dist.all_gather(list(gathered.unbind(0)), src)


def _rows_mean(gathered, out):
    if gathered.is_cuda and gathered.dtype == torch.float32:
        from dmlab.ops._native import lib

        lib().rows_mean(gathered, out, 1.0 / gathered.shape[0])
    else:
        out.copy_(gathered.mean(0))


@torch.no_grad()
def allgather_average_gradients_reference_compat(model):
    """Bit-for-bit reproduction of the reference bug (task2/dist_utils.py:44-49):
    ``[zeros_like(g)] * 2`` aliases one buffer, so the "mean" is the last rank's
    gradient and world sizes other than 2 fail.  Only for the lab comparison."""
    for p in model.parameters():
        params = [torch.zeros_like(p.grad.data)] * 2
        dist.all_gather(params, p.grad.data)
        p.grad.data.copy_(torch.mean(torch.stack(params), dim=0))


# ------------------------------------------------------------------ aggregator object
class GradAggregator:
    """Callable gradient aggregation with communication timing (lab 2).

    ``method``: ``allreduce`` | ``allgather`` | ``allgather_ref`` (B1 compat) |
    ``allreduce_xgmi`` (the one-shot peer-memory kernel of :mod:`dmlab.parallel.xgmi` over
    the flat gradient buffer, averaging folded into its epilogue: GPU ranks of one node);
    ``granularity``: ``flat`` (one coalesced collective) | ``per_param``.

    ``timing``:
      * ``"events"`` (default on a HIP device): a pair of HIP events on the current stream
        brackets each aggregation (the manual's ``torch.cuda.Event`` recipe,
        ``task2.tex:69-80``).  RCCL orders the current stream after the collective, so the
        interval is the device-side communication time, including the wait for a slow
        peer; nothing synchronises the host, so the measurement does not drain backward
        the way a ``synchronize()`` pair would.  ``comm_time`` reads the events back once.
      * ``"sync"``: the old wall-clock bracket with a stream synchronise on both sides.
      * ``"host"``: host wall time only (the reference's ``time.time()`` pair,
        model-mp.py:61-66; with an asynchronous backend it measures only the enqueue).
    On the CPU (gloo) the collectives are synchronous and wall time is exact."""

    def __init__(self, model, method="allreduce", granularity="flat", timing=None,
                 sync_timing=None, force=False):
        self.model, self.method, self.granularity = model, method, granularity
        if timing is None:
            # the legacy flag keeps its meaning: True = synchronised wall clock, False = host
            # wall time only; neither given = device-side event timing
            timing = "events" if sync_timing is None else ("sync" if sync_timing else "host")
        self.timing = timing
        self.force = force
        self._host_time = 0.0
        self._events = []
        self.calls = 0

    def _on_gpu(self):
        return torch.cuda.is_available() and next(self.model.parameters()).is_cuda

    def _aggregate(self):
        if self.method == "allreduce":
            allreduce_average_gradients(self.model, self.granularity, force=self.force)
        elif self.method == "allgather":
            allgather_average_gradients(self.model, self.granularity, force=self.force)
        elif self.method == "allgather_ref":
            allgather_average_gradients_reference_compat(self.model)
        elif self.method == "allreduce_xgmi":
            ws = env.get_world_size()
            if ws <= 1 and not (self.force and env.is_initialized()):
                return
            flat = _flat_of_model(self.model)
            if flat is None or not flat.grad.is_cuda:
                raise ValueError("allreduce_xgmi: a Program model on a GPU")
            if getattr(self, "_xgmi", None) is None:
                from .xgmi import XGMIAllReduce

                self._xgmi = XGMIAllReduce(cap=flat.grad.numel())
            self._xgmi(flat.grad, scale=1.0 / ws)
        else:
            raise ValueError(self.method)

    def __call__(self):
        """Aggregate; returns the host-measured seconds, or None with event timing."""
        gpu = self._on_gpu()
        self.calls += 1
        if gpu and self.timing == "events":
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            self._aggregate()
            e.record()
            self._events.append((s, e))
            return None
        if gpu and self.timing == "sync":
            torch.cuda.current_stream().synchronize()
        t0 = time.perf_counter()
        self._aggregate()
        if gpu and self.timing == "sync":
            torch.cuda.current_stream().synchronize()
        dt = time.perf_counter() - t0
        self._host_time += dt
        return dt

    @property
    def comm_time(self) -> float:
        """Total communication seconds so far (reads pending HIP events back once)."""
        if self._events:
            self._events[-1][1].synchronize()
            self._host_time += sum(s.elapsed_time(e) for s, e in self._events) * 1e-3
            self._events = []
        return self._host_time
