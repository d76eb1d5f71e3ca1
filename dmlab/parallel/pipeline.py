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
* activations and activation-gradients move with ``torch.distributed`` P2P
  (``isend``/``irecv`` — RCCL over xGMI on GPUs; gloo on CPU, with a host staging
  copy if a gloo group is used for device tensors);
* GPipe (all-forward, all-backward) or 1F1B micro-batch schedules so stage i
  computes micro-batch m+1 while stage i+1 works on m;
* each stage steps its own fused optimiser locally (no optimiser RPC).

The tensor shape of every message is fixed by the model; it is negotiated once
with a small header message and cached.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import env


class P2P:
    """Point-to-point transport between adjacent stages.

    Every message is preceded by a 16-word shape header unless ``static_shapes``
    is set, in which case the header is exchanged once per tag and cached (use it
    when every micro-batch has the same shape)."""

    def __init__(self, group=None, static_shapes=False):
        self.group = group
        self.gloo = dist.get_backend(group) == "gloo"
        self.static = static_shapes
        self._shapes = {}

    def _dev_out(self, t):
        return t.cpu() if (self.gloo and t.is_cuda) else t

    def send(self, t: torch.Tensor, dst: int, tag: str):
        """Non-blocking (header and payload are both isend) so opposite-direction
        sends of a 1F1B schedule can never deadlock; returns the works to wait on."""
        t = t.contiguous()
        works = []
        if not self.static or tag not in self._shapes:
            hdr = torch.tensor([t.dim()] + list(t.shape) + [_DT.index(t.dtype)], dtype=torch.long)
            hdr = torch.cat([torch.tensor([hdr.numel()]), hdr])
            hdr = self._pad(hdr)
            if not self.gloo:
                hdr = hdr.to(t.device)
            works.append(dist.isend(hdr, dst, group=self.group))
            self._shapes[tag] = (tuple(t.shape), t.dtype)
        works.append(dist.isend(self._dev_out(t), dst, group=self.group))
        return works

    @staticmethod
    def _pad(h):
        out = torch.zeros(16, dtype=torch.long)
        out[: h.numel()] = h
        return out

    def recv(self, src: int, tag: str, device):
        if not self.static or tag not in self._shapes:
            hdr = torch.zeros(16, dtype=torch.long,
                              device="cpu" if self.gloo else device)
            dist.recv(hdr, src, group=self.group)
            hdr = hdr.cpu()
            nd = int(hdr[1])
            shape = tuple(int(v) for v in hdr[2:2 + nd])
            dtype = _DT[int(hdr[2 + nd])]
            self._shapes[tag] = (shape, dtype)
        shape, dtype = self._shapes[tag]
        dev = torch.device("cpu") if self.gloo else device
        buf = torch.empty(shape, dtype=dtype, device=dev)
        work = dist.irecv(buf, src, group=self.group)
        return buf, work


_DT = [torch.float32, torch.bfloat16, torch.float16, torch.int64]


class PipelineStage:
    """One stage of a linear pipeline.

    ``module``  : this stage's sub-network (a :class:`~dmlab.nn.program.Program` or
                  any ``nn.Module``); ``loss_fn`` is used on the last stage only.
    ``ranks``   : the global ranks of all stages in order (default: 0..P-1).
    """

    def __init__(self, module, optimizer, loss_fn=None, ranks=None, device=None,
                 schedule="1f1b", group=None, static_shapes=False):
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
        self.p2p = P2P(group, static_shapes)
        assert schedule in ("gpipe", "1f1b")
        self.schedule = schedule
        self._pending = []

    # -------------------------------------------------------------- pieces
    def _labels(self, y, n_micro):
        """Labels travel from the data owner (first stage) to the last stage."""
        if self.P == 1:
            return y.chunk(n_micro)
        if self.first:
            self._pending.extend(self.p2p.send(y, self.ranks[-1], "labels"))
            return None
        if self.last:
            buf, w = self.p2p.recv(self.ranks[0], "labels", self.device)
            w.wait()
            return buf.to(self.device).chunk(n_micro)
        return None

    def _fwd(self, m, xs, ys, saved, losses):
        if self.first:
            inp = xs[m]
        else:
            buf, w = self.p2p.recv(self.prev, "act", self.device)
            w.wait()
            inp = buf.to(self.device).requires_grad_(True)
        out = self.module(inp)
        if self.last:
            loss = self.loss_fn(out, ys[m]) / len(ys)
            losses.append(loss.detach())
            saved[m] = (inp, loss)
        else:
            self._pending.extend(self.p2p.send(out.detach(), self.next, "act"))
            saved[m] = (inp, out)

    def _bwd(self, m, saved):
        inp, out = saved.pop(m)
        if self.last:
            out.backward()
        else:
            buf, w = self.p2p.recv(self.next, "grad", self.device)
            w.wait()
            out.backward(buf.to(self.device).to(out.dtype))
        if not self.first:
            self._pending.extend(self.p2p.send(inp.grad, self.prev, "grad"))

    def _drain(self):
        for w in self._pending:
            w.wait()
        self._pending.clear()

    # -------------------------------------------------------------- step
    def train_step(self, x=None, y=None, n_micro: int = 1):
        """One optimisation step over ``n_micro`` micro-batches.  ``x``/``y`` are
        needed on the first stage only.  Returns the mean loss on the last stage
        (a 0-d tensor) and None elsewhere."""
        self.opt.zero_grad()
        xs = x.chunk(n_micro) if self.first else None
        ys = self._labels(y, n_micro) if (self.first or self.last) else None
        saved, losses = {}, []
        if self.schedule == "gpipe" or self.P == 1:
            for m in range(n_micro):
                self._fwd(m, xs, ys, saved, losses)
            for m in range(n_micro):
                self._bwd(m, saved)
        else:  # 1F1B: warm up (P - idx - 1) forwards, then alternate, then drain
            warm = min(self.P - self.idx - 1, n_micro)
            f = b = 0
            for _ in range(warm):
                self._fwd(f, xs, ys, saved, losses)
                f += 1
            while f < n_micro:
                self._fwd(f, xs, ys, saved, losses)
                f += 1
                self._bwd(b, saved)
                b += 1
            while b < n_micro:
                self._bwd(b, saved)
                b += 1
        self._drain()
        self.opt.step()
        if self.last:
            return torch.stack(losses).sum()
        return None

    @torch.no_grad()
    def forward_only(self, x=None):
        """Inference through the pipeline; returns logits on the last stage."""
        if self.first:
            h = x
        else:
            buf, w = self.p2p.recv(self.prev, "eval_act", self.device)
            w.wait()
            h = buf.to(self.device)
        out = self.module(h)
        if not self.last:
            for w in self.p2p.send(out, self.next, "eval_act"):
                w.wait()
            return None
        return out
