"""roctx ranges for rocprofv3 (``--marker-trace``) around the training-step phases.

The reference has no tracing beyond ``time.time()`` around epoch chunks
(``main_distributed.py:205-224``). Here every phase of the step can be bracketed
by a named roctx range so a rocprofv3 timeline shows forward / gather / loss / backward /
all-reduce wait / optimizer per step. Ranges are emitted only when ``MILNCE_ROCTX=1`` (or
``enable()`` is called) and libroctx64 is loadable; otherwise every call is a no-op.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional

_lib: Optional[ctypes.CDLL] = None
_enabled = os.environ.get("MILNCE_ROCTX", "0") == "1"
_tried = False


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
        except OSError:
            continue
        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
        lib.roctxRangePushA.restype = ctypes.c_int
        lib.roctxRangePop.argtypes = []
        lib.roctxRangePop.restype = ctypes.c_int
        lib.roctxMarkA.argtypes = [ctypes.c_char_p]
        lib.roctxMarkA.restype = None
        _lib = lib
        break
    return _lib


def enable(flag: bool = True) -> bool:
    """Turn ranges on/off; returns whether a roctx library is available."""
    global _enabled
    _enabled = bool(flag)
    return _load() is not None


def enabled() -> bool:
    return _enabled and _load() is not None


def push(name: str) -> None:
    if _enabled and _load() is not None:
        _lib.roctxRangePushA(name.encode())


def pop() -> None:
    if _enabled and _load() is not None:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if _enabled and _load() is not None:
        _lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx vocabulary
    push(name)
    try:
        yield
    finally:
        pop()
