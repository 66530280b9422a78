"""Hang / failure detection for the training loop.

The reference has none (a crash or a stuck collective simply stalls the job).
``Watchdog`` is a daemon thread fed by ``beat()`` once per step. If no beat arrives for
``timeout_s`` it dumps every thread's Python stack (``faulthandler``) to stderr and to
``<dump_dir>/watchdog_rank<r>.txt``, then — if ``abort`` — exits the process with status 3 so a
launcher (torchrun / the driver) tears the job down and the run can ``--resume`` from the last
step/epoch checkpoint. RCCL's own collective timeout is set through
``init_process_group(timeout=...)`` (``--dist_timeout_s``); this covers host-side hangs too
(data pipeline, deadlocked Python, a rank stuck before its collective).
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Optional


class Watchdog:
    def __init__(self, timeout_s: float, rank: int = 0, dump_dir: str = "", abort: bool = True,
                 poll_s: Optional[float] = None):
        self.timeout_s = float(timeout_s)
        self.rank = rank
        self.dump_dir = dump_dir
        self.abort = abort
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(5.0, self.timeout_s / 10))
        self._last = time.monotonic()
        self._step = -1
        self._stop = threading.Event()
        self.fired = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def start(self) -> "Watchdog":
        if self.timeout_s > 0 and self._thread is None:
            self._thread = threading.Thread(target=self._run, name="milnce-watchdog", daemon=True)
            self._thread.start()
        return self

    def beat(self, step: int = -1) -> None:
        self._last = time.monotonic()
        self._step = step

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle < self.timeout_s:
                continue
            msg = (f"[watchdog] rank {self.rank}: no training progress for {idle:.1f}s "
                   f"(last step {self._step}); dumping stacks\n")
            sys.stderr.write(msg)
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            if self.dump_dir:
                os.makedirs(self.dump_dir, exist_ok=True)
                with open(os.path.join(self.dump_dir, f"watchdog_rank{self.rank}.txt"), "w") as f:
                    f.write(msg)
                    faulthandler.dump_traceback(file=f, all_threads=True)
            self.fired.set()
            if self.abort:
                sys.stderr.flush()
                os._exit(3)
            return
