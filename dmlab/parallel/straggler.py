"""Bottleneck-node ("straggler") injection (lab 2 requirement).

Reference: ``bottle_neck_delay = 0.1`` and, commented out, ``if rank == 1:
time.sleep(bottle_neck_delay)`` after aggregation (codes/task2/model-mp.py:47,64-65);
requirement "设置瓶颈节点" (sections/task2.tex:19, checking.tex:22).

Two modes:
* ``host``   — ``time.sleep`` on the straggler rank (the reference behaviour; models
  a slow host / data pipeline);
* ``device`` — a HIP spin kernel that occupies the straggler's GPU stream for the
  given time (models a slow GPU; works inside hipGraph capture, no host sync).
"""
from __future__ import annotations

import time

import torch

from . import env


class Straggler:
    def __init__(self, rank: int | None = None, delay_ms: float = 0.0, mode: str = "host",
                 every: int = 1):
        self.rank = rank
        self.delay_ms = float(delay_ms)
        self.mode = mode
        self.every = max(int(every), 1)
        self.calls = 0
        self.injected_ms = 0.0

    @property
    def active(self) -> bool:
        return self.rank is not None and self.delay_ms > 0 and env.get_rank() == self.rank

    def __call__(self):
        self.calls += 1
        if not self.active or (self.calls % self.every):
            return
        if self.mode == "host":
            time.sleep(self.delay_ms / 1e3)
        elif self.mode == "device":
            from dmlab.ops._native import lib

            lib().spin_us(float(self.delay_ms * 1e3))
        else:
            raise ValueError(self.mode)
        self.injected_ms += self.delay_ms
