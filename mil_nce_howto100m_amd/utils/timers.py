"""Step-phase timers on HIP events (no host sync inside the step).

``StepTimer`` records an event pair per phase on the current stream; ``summary()`` synchronises
once and returns mean milliseconds per phase. On CPU it falls back to ``time.perf_counter``.
Phases used by the trainer: ``data``, ``forward``, ``backward``, ``allreduce_wait``,
``optimizer`` (SURVEY.md §5 "HIP-event step timers (fwd/bwd/comm/optimizer)").
The timer is off unless ``enabled=True``: recording events costs a few microseconds per phase.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict, List, Tuple

import torch

from . import roctx


class StepTimer:
    def __init__(self, enabled: bool = False, device: torch.device | None = None):
        self.enabled = enabled
        self.cuda = device is not None and device.type == "cuda" and torch.cuda.is_available()
        self._pending: Dict[str, List[Tuple[object, object]]] = defaultdict(list)
        self._host: Dict[str, List[float]] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            with roctx.range(name):
                yield
            return
        if self.cuda:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            with roctx.range(name):
                yield
            b.record()
            self._pending[name].append((a, b))
        else:
            t0 = time.perf_counter()
            with roctx.range(name):
                yield
            self._host[name].append(1000.0 * (time.perf_counter() - t0))

    def summary(self, reset: bool = True) -> Dict[str, float]:
        out: Dict[str, float] = {}
        if self.cuda and self._pending:
            torch.cuda.synchronize()
            for k, evs in self._pending.items():
                out[k] = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
        for k, v in self._host.items():
            out[k] = sum(v) / len(v)
        if reset:
            self._pending.clear()
            self._host.clear()
        return out
