"""Stream priorities for the two-stream training step.

A dmlab ResNet step runs its critical path (forward, data gradients, BN backward) on the
caller's stream and the weight gradients on a side stream (``Program._side_stream``).  Both
were created at the default priority, so when both queues hold work the command processor
hands out workgroups to them evenly, although only the critical path bounds the step.
:func:`compute_stream` returns a per-device HIGH-priority stream to run the step on: the
weight gradients then fill the CUs the critical path leaves idle instead of competing for
them on equal terms.
"""
from __future__ import annotations

import torch

_STREAMS: dict[int, torch.cuda.Stream] = {}


def compute_stream(device=None) -> torch.cuda.Stream:
    """The highest-priority stream of ``device`` (created once per device)."""
    dev = torch.cuda.current_device() if device is None else torch.device(device).index
    st = _STREAMS.get(dev)
    if st is None:
        lo, hi = torch.cuda.Stream.priority_range()  # (least, greatest): greatest is smaller
        st = _STREAMS[dev] = torch.cuda.Stream(device=dev, priority=min(lo, hi))
    return st
