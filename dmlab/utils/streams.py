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
_PARTS: dict[tuple, torch.cuda.ExternalStream] = {}


def compute_stream(device=None) -> torch.cuda.Stream:
    """The highest-priority stream of ``device`` (created once per device)."""
    dev = torch.cuda.current_device() if device is None else torch.device(device).index
    st = _STREAMS.get(dev)
    if st is None:
        lo, hi = torch.cuda.Stream.priority_range()  # (least, greatest): greatest is smaller
        st = _STREAMS[dev] = torch.cuda.Stream(device=dev, priority=min(lo, hi))
    return st


def partition_stream(part: int, nparts: int, device=None) -> torch.cuda.ExternalStream:
    """A stream restricted to CU partition ``part`` of ``nparts`` equal contiguous CU ranges.

    Processes sharing one GPU that each run on a different partition do not compete for CUs,
    so each sees a (smaller) device of its own: the lab-4 pipeline uses this to emulate
    one-GPU-per-stage on a one-GPU box (``task4 --cu-partition``).  The stream has its own
    hardware queue carrying the mask (``hipExtStreamCreateWithCUMask``), created once per
    (device, part, nparts) and reused: a new stream per call would leak hardware queues."""
    from dmlab.ops._native import lib

    if not 0 <= part < nparts:
        raise ValueError(f"partition {part} of {nparts}")
    dev = torch.cuda.current_device() if device is None else torch.device(device).index
    key = (dev, part, nparts)
    if key in _PARTS:
        return _PARTS[key]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    lo, hi = part * ncu // nparts, (part + 1) * ncu // nparts
    words = [0] * ((ncu + 31) // 32)
    for c in range(lo, hi):
        words[c // 32] |= 1 << (c % 32)
    with torch.cuda.device(dev):
        ptr = lib().cu_mask_stream(words)
    st = _PARTS[key] = torch.cuda.ExternalStream(ptr, device=torch.device("cuda", dev))
    return st
