"""Inter-layer model parallelism (lab 4): stage-per-GPU pipeline over P2P.

Reference: codes/task4/model.py — a driver process (rank 0) owns data and loss;
``SubNetConv`` lives on worker1 and ``SubNetFC`` on worker2 (``rpc.remote``,
model.py:54-55); every step is a blocking ``rpc_sync`` chain that relays the
(B,400) activation *through the driver* (B8), runs ``dist_autograd.backward``
and two remote ``DistributedOptimizer`` steps (model.py:68-87).  There is no
micro-batching, so the stages never overlap.

MI355X-native design (this module):
* one process per stage (rank i = stage i, its own GPU); the data/loss "driver"
  role is co-located with the first stage (inputs) and the last stage (labels +
  loss), so activations go stage→stage directly, never via a relay;
* activations and activation-gradients move over a stage transport
  (:mod:`dmlab.parallel.p2p`): RCCL P2P over xGMI with one process group per direction,
  or the native xGMI peer-memory channel (``transport="xgmi"``: the sender's kernel writes
  straight into the receiver's device ring); gloo on the CPU;
* every receive is posted one micro-batch AHEAD of the compute that consumes it and waited
  for only where the data is used (a device-side stream wait, never a host sync); message
  shapes are negotiated once and cached (``static_shapes``, default on: the labs' batches
  have one shape);
* GPipe (all-forward, all-backward) or 1F1B micro-batch schedules so stage i
  computes micro-batch m+1 while stage i+1 works on m;
* each stage steps its own fused optimiser locally (no optimiser RPC);
* ``timing=True`` brackets each stage's compute with HIP events, so a step reports its
  compute time and the bubble (the fraction of the step a stage sits idle).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import env
from .p2p import PGTransport, XGMITransport


class PipelineStage:
    """One stage of a linear pipeline.

    ``module``    : this stage's sub-network (a :class:`~dmlab.nn.program.Program` or
                    any ``nn.Module``); ``loss_fn`` is used on the last stage only.
    ``ranks``     : the global ranks of all stages in order (default: 0..P-1).
    ``transport`` : ``"pg"`` (torch.distributed P2P: RCCL / gloo), ``"xgmi"`` (native
                    peer-memory channels, GPU only) or a transport object.
    """

    def __init__(self, module, optimizer, loss_fn=None, ranks=None, device=None,
                 schedule="1f1b", group=None, static_shapes=True, transport="pg",
                 cap_bytes=1 << 20, timing=False):
        self.module = module
        self.opt = optimizer
        self.loss_fn = loss_fn
        self.ranks = list(ranks) if ranks is not None else list(range(env.get_world_size()))
        self.rank = env.get_rank()
        self.idx = self.ranks.index(self.rank)
        self.P = len(self.ranks)
        self.first = self.idx == 0
        self.last = self.idx == self.P - 1
        self.prev = self.ranks[self.idx - 1] if not self.first else None
        self.next = self.ranks[self.idx + 1] if not self.last else None
        self.device = device or env.device()
        if transport == "pg":
            self.p2p = PGTransport(self.ranks, static_shapes)
        elif transport == "xgmi":
            links = [(self.ranks[i], self.ranks[i + 1]) for i in range(self.P - 1)]
            links += [(self.ranks[i + 1], self.ranks[i]) for i in range(self.P - 1)]
            if self.P > 2:
                links.append((self.ranks[0], self.ranks[-1]))  # labels
            self.p2p = XGMITransport(links, cap_bytes=cap_bytes, group=group, device=self.device)
        else:
            self.p2p = transport
        assert schedule in ("gpipe", "1f1b")
        self.schedule = schedule
        self._pending = []
        self._posted = {}
        self.timing = timing and torch.cuda.is_available() and self.device.type == "cuda"
        self._events = []
        self.history = []  # (start, end, compute events) of every timed step
        self._linear = False  # no receive posted ahead (captured steps)
        self._graph = None
        self._time_replays = False

    def selfcheck(self, corrupt=None) -> dict:
        """One ping-pong per adjacent stage pair over this stage's transport, payloads checked
        both ways (:func:`dmlab.parallel.selfcheck.p2p_selfcheck`); collective over the
        default group.  Returns {"p2p_selfcheck": "pass" | "FAIL"}."""
        from dmlab.parallel.selfcheck import p2p_selfcheck

        res = "pass"
        for i in range(self.P - 1):
            a, b = self.ranks[i], self.ranks[i + 1]
            peer = b if self.rank == a else a if self.rank == b else None
            r = p2p_selfcheck(self.p2p, self.rank, peer, self.device, first=self.rank == a,
                              corrupt=corrupt)
            if r["p2p_selfcheck"] != "pass":
                res = "FAIL"
        return {"p2p_selfcheck": res}

    # -------------------------------------------------------------- pieces
    def _post_recv(self, tag, m, src, ahead=False):
        """Post the receive of message (tag, m) now; consumed later by _take.  A receive
        posted AHEAD of its use waits until the message shape is cached (the first step
        negotiates shapes with a blocking header receive, which must not run ahead of the
        schedule: the peer may still need a message from this rank first)."""
        k = (tag, m)
        if k in self._posted:
            return
        if ahead and (self._linear or not self.p2p.known(k)):
            return
        self._posted[k] = self.p2p.recv(src, k, self.device)

    def _take(self, tag, m, src):
        self._post_recv(tag, m, src)
        buf, w = self._posted.pop((tag, m))
        w.wait()
        return buf

    def _labels(self, y, n_micro):
        """Labels travel from the data owner (first stage) to the last stage."""
        if self.P == 1:
            return y.chunk(n_micro)
        if self.first:
            self._pending.extend(self.p2p.send(y, self.ranks[-1], ("labels", 0)))
            return None
        if self.last:
            return self._take("labels", 0, self.ranks[0]).to(self.device).chunk(n_micro)
        return None

    def _timed(self, fn):
        if not self.timing:
            return fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn()
        e.record()
        self._events.append((s, e))
        return out

    def _fwd(self, m, xs, ys, saved, losses, n_micro):
        if self.first:
            inp = xs[m]
        else:
            inp = self._take("act", m, self.prev)
            if m + 1 < n_micro:
                self._post_recv("act", m + 1, self.prev, ahead=True)  # lands during compute m
            inp = inp.to(self.device).requires_grad_(True)
        out = self._timed(lambda: self.module(inp))
        if self.last:
            loss = self._timed(lambda: self.loss_fn(out, ys[m]) / len(ys))
            losses.append(loss.detach())
            saved[m] = (inp, loss)
        else:
            self._pending.extend(self.p2p.send(out.detach(), self.next, ("act", m)))
            saved[m] = (inp, out)

    def _bwd(self, m, saved, n_micro):
        inp, out = saved.pop(m)
        if self.last:
            self._timed(lambda: out.backward())
        else:
            g = self._take("grad", m, self.next)
            if m + 1 < n_micro:
                self._post_recv("grad", m + 1, self.next, ahead=True)
            self._timed(lambda: out.backward(g.to(self.device).to(out.dtype)))
        if not self.first:
            self._pending.extend(self.p2p.send(inp.grad, self.prev, ("grad", m)))

    def _drain(self):
        for w in self._pending:
            w.wait()
        self._pending.clear()

    # -------------------------------------------------------------- step
    def train_step(self, x=None, y=None, n_micro: int = 1):
        """One optimisation step over ``n_micro`` micro-batches.  ``x``/``y`` are
        needed on the first stage only.  Returns the mean loss on the last stage
        (a 0-d tensor) and None elsewhere."""
        if self.timing:
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            self._events = []
            t0.record()
        self.opt.zero_grad()
        xs = x.chunk(n_micro) if self.first else None
        ys = self._labels(y, n_micro) if (self.first or self.last) else None
        saved, losses = {}, []
        if self.schedule == "gpipe" or self.P == 1:
            for m in range(n_micro):
                self._fwd(m, xs, ys, saved, losses, n_micro)
            for m in range(n_micro):
                self._bwd(m, saved, n_micro)
        else:  # 1F1B: warm up (P - idx - 1) forwards, then alternate, then drain
            warm = min(self.P - self.idx - 1, n_micro)
            f = b = 0
            for _ in range(warm):
                self._fwd(f, xs, ys, saved, losses, n_micro)
                f += 1
            while f < n_micro:
                self._fwd(f, xs, ys, saved, losses, n_micro)
                f += 1
                self._bwd(b, saved, n_micro)
                b += 1
            while b < n_micro:
                self._bwd(b, saved, n_micro)
                b += 1
        self._drain()
        self.opt.step()
        if self.timing:
            t1.record()
            self._step_events = (t0, t1, list(self._events))
            self.history.append(self._step_events)
        if self.last:
            return torch.stack(losses).sum()
        return None

    # -------------------------------------------------------------- hipGraph
    def capture(self, x=None, y=None, n_micro: int = 1, warmup: int = 2):
        """Capture one whole ``train_step`` (micro-batch schedule, channel kernels, backward,
        optimiser) into a hipGraph; :meth:`replay` then runs a step as ONE graph launch, so
        the per-micro-batch host work (a Python schedule, ~15 kernel launches and the
        stream/event hops per message) is gone.  Needs the xGMI transport (its message
        counters live on the device) and every rank capturing with the same ``n_micro`` and
        ``warmup``.

        The captured step is one linear chain in program order: the channel kernels run
        inline on the step's stream and no receive is posted ahead.  A graph executes its
        independent branches in an order of the runtime's choosing; with receives that spin
        on a peer, a branch order other than program order could wait on a message the peer
        sends only after this stage's skipped-over work (a cross-process deadlock that the
        bounded waits would turn into a timeout).  Program order with blocking receives and
        buffered sends is deadlock-free for GPipe and 1F1B."""
        if not isinstance(self.p2p, XGMITransport):
            raise ValueError("PipelineStage.capture needs transport='xgmi'")
        self._linear, self.p2p.inline = True, True
        self._sx = x.detach().clone() if self.first else None
        self._sy = y.detach().clone() if self.first else None
        self._n_micro = n_micro
        timed, self.timing = self.timing, False
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):  # shapes negotiated, optimiser state allocated
                loss = self.train_step(self._sx, self._sy, n_micro)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize(self.device)
        self._graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._graph):
            self._gout = self.train_step(self._sx, self._sy, n_micro)
        self._time_replays = timed
        return loss  # of the last warm-up step (the warm-up steps are real updates)

    def replay(self, x=None, y=None):
        """One captured step on new data (first stage: ``x``/``y``; others: nothing).  With
        ``timing`` the step is bracketed by events (no per-compute events inside a graph:
        :meth:`step_stats` then reports the step time only)."""
        if self._graph is None:
            raise RuntimeError("PipelineStage.replay: no captured step; call capture() first")
        if self.first:
            self._sx.copy_(x, non_blocking=True)
            self._sy.copy_(y, non_blocking=True)
        if self._time_replays:
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
        self._graph.replay()
        if self._time_replays:
            t1.record()
            self._step_events = (t0, t1, [])
            self.history.append(self._step_events)
        return self._gout

    def step_stats(self, skip=None):
        """(step ms, compute ms, bubble fraction): of the last timed step, or averaged over
        the timed steps after the first ``skip`` (synchronises once).  Captured steps carry
        no compute events: compute and bubble are None."""
        steps = [self._step_events] if skip is None else self.history[skip:]
        steps[-1][1].synchronize()
        tot = comp = 0.0
        for t0, t1, evs in steps:
            tot += t0.elapsed_time(t1)
            comp += sum(s.elapsed_time(e) for s, e in evs)
        n = len(steps)
        if not any(evs for _, _, evs in steps):
            return tot / n, None, None
        return tot / n, comp / n, (max(0.0, 1.0 - comp / tot) if tot > 0 else 0.0)

    @torch.no_grad()
    def forward_only(self, x=None):
        """Inference through the pipeline; returns logits on the last stage."""
        if self.first:
            h = x
        else:
            h = self._take("eval_act", 0, self.prev).to(self.device)
        out = self.module(h)
        if not self.last:
            for w in self.p2p.send(out, self.next, ("eval_act", 0)):
                w.wait()
            return None
        return out
