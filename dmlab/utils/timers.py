"""Timing helpers: HIP-event phase timers and host wall clocks.

The reference times with ``time.time()`` around the whole run and around the
aggregation (task2/model-mp.py:48,61-66,79) and recommends
``torch.cuda.Event(enable_timing=True)`` (sections/task2.tex:69-80).  With an async
RCCL backend a host clock around a collective measures only its enqueue, so
:class:`PhaseTimer` records HIP events on the stream and resolves them lazily
(one sync at report time, none in the loop).
"""
from __future__ import annotations

import time
from collections import defaultdict

import torch


class PhaseTimer:
    def __init__(self, enabled: bool = True, device=None):
        self.enabled = enabled and torch.cuda.is_available()
        self._open = {}
        self._pairs = defaultdict(list)
        self._host = defaultdict(float)

    def start(self, name):
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._open[name] = e
        else:
            self._open[name] = time.perf_counter()

    def stop(self, name):
        s = self._open.pop(name)
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._pairs[name].append((s, e))
        else:
            self._host[name] += time.perf_counter() - s

    def totals_ms(self) -> dict:
        out = {k: v * 1e3 for k, v in self._host.items()}
        if self._pairs:
            torch.cuda.synchronize()
            for k, ps in self._pairs.items():
                out[k] = out.get(k, 0.0) + sum(a.elapsed_time(b) for a, b in ps)
        return out


class Wall:
    def __init__(self):
        self.t0 = time.perf_counter()

    def elapsed(self):
        return time.perf_counter() - self.t0
