"""The training step's compute stream.

The step runs on a HIP stream of high priority (``MILNCE_MAIN_PRIO``, default on; ``0`` keeps the
default stream): the weight gradients overlap the backward chain on a normal-priority side stream
(ops/hip_ops.py), and when both have workgroups waiting for a CU the main chain's are dispatched
first. Same-box A/Bs of the flagship step (profiles/r6_summary.md): +0.3 % and +0.35 %.

Work queued on the current stream before the context (parameter initialisation, broadcasts,
checkpoint loads) is ordered before the priority stream's first kernel, and the previous stream
waits for the priority stream's work at exit, so code after the loop sees finished results.
"""
from __future__ import annotations

import os

import torch

_MAIN_PRIO = os.environ.get("MILNCE_MAIN_PRIO", "1") != "0"


class MainStream:
    """Context manager: run the enclosed steps on a high-priority stream of ``device``."""

    def __init__(self, device, enabled: bool = None):
        self.device = torch.device(device)
        self.enabled = (_MAIN_PRIO if enabled is None else bool(enabled)) and self.device.type == "cuda"
        self.stream = None
        self._ctx = None
        self._prev = None

    def __enter__(self):
        if not self.enabled:
            return self
        self._prev = torch.cuda.current_stream(self.device)
        lo, hi = torch.cuda.Stream.priority_range()
        self.stream = torch.cuda.Stream(device=self.device, priority=min(lo, hi))
        self.stream.wait_stream(self._prev)
        self._ctx = torch.cuda.stream(self.stream)
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        self._ctx.__exit__(*exc)
        self._prev.wait_stream(self.stream)
        return False

    @property
    def priority(self) -> int:
        return self.stream.priority if self.stream is not None else 0
