"""Run logging: the reference's text log line plus a JSONL metrics stream.

``log()`` appends to ``<log_root>/<checkpoint_dir>temp.txt`` exactly like
``main_distributed.py:304-306`` (rank 0 only, fixing the unlocked multi-rank appends of
``:167,173,180``). ``MetricsLogger`` additionally records step, loss, lr, pairs/s and the
step-time breakdown as JSON lines for machine consumption.
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional


def log(output: str, args, rank: int = 0) -> None:
    if rank != 0:
        return
    root = getattr(args, "log_root", "log") or "log"
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, (getattr(args, "checkpoint_dir", "") or "") + "temp.txt"), "a") as f:
        f.write(output + "\n")
    if getattr(args, "verbose", 0) > 1:
        print(output, flush=True)


def train_line(epoch: int, elapsed: float, status: float, loss: float, lr: float) -> str:
    """Same format string as main_distributed.py:213-223."""
    return ("Epoch %d, Elapsed Time: %.3f, Epoch status: %.4f, Training loss: %.4f, Learning rate: %.6f"
            % (epoch, elapsed, status, loss, lr))


class MetricsLogger:
    def __init__(self, path: str = "", rank: int = 0):
        self.path = path if rank == 0 else ""
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)

    def write(self, **kw) -> None:
        if not self.path:
            return
        kw.setdefault("time", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(kw) + "\n")
