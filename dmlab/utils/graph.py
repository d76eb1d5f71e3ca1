"""hipGraph capture of a whole training step (HIP graphs instead of a tracing compiler).

The reference's loop is launch- and sync-bound (~60 kernel launches,
8 collectives and a ``loss.item()`` per LeNet step).  A dmlab step is already a
fixed sequence of native launches (explicit forward/backward programs, fused
optimiser), so the whole iteration — forward, backward with its bucketed RCCL
all-reduces, and the optimiser update — is captured once into a hipGraph and
replayed with a single launch per step.

Requirements honoured by the engine: no host synchronisation inside a step, all
temporaries from the caching allocator (graph-private pool during capture), and
state that changes every step (weights, momentum, BN running stats) kept in
device tensors.  Inputs are copied into static buffers before each replay, or, with
``bind_inputs=True``, the example inputs ARE the static buffers (a loader that fills
them in place — or one graph per device-resident batch slot — skips the copy).
"""
from __future__ import annotations

import torch


class CapturedStep:
    """``step_fn(*inputs) -> tensor`` captured into a graph after ``warmup`` eager
    iterations on a side stream (so lazy initialisation, allocator growth and the
    optimiser's first-step branch happen outside the capture)."""

    def __init__(self, step_fn, example_inputs, warmup: int = 3, bind_inputs: bool = False):
        self.step_fn = step_fn
        self.static_inputs = [t.detach() if bind_inputs else t.detach().clone()
                              for t in example_inputs]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                step_fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_output = step_fn(*self.static_inputs)
        self.replays = 0

    def __call__(self, *inputs):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not dst and src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        return self.static_output
