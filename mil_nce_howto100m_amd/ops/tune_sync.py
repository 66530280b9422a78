"""Rank-consistent kernel autotuning for data parallelism.

Every conv shape / direction picks its kernel variant and persistent grid by timing the
candidates on first use (``hip_ops._tune``). Timed independently on each rank, 8 GPUs could pick
different kernels for the same layer: a straggler for the max-over-ranks step time, and a
rank-dependent summation order (the box-tiled and the v3 / v4 kernel families accumulate in
different orders). Inside ``region()`` (entered by the Trainer around every training step when
the world size is > 1) rank 0 alone times the candidates and publishes each decision through the
process group's c10d store; the other ranks take it from there and launch the same variant.

Decisions are keyed by a running counter plus the caller's problem signature: every rank makes
the same sequence of tuning calls in a DP step (same model, same per-rank batch shape), and a
rank whose signature differs from rank 0's raises instead of silently using a kernel tuned for
another shape. ``plan_hash()`` digests the decisions this process made (bench.py reports it per
rank). The reference has no autotuning; cuDNN's benchmark mode (``--cudnn_benchmark``,
``main_distributed.py:177-178``) is per process, which is what this replaces for the HIP kernels.
"""
from __future__ import annotations

import contextlib
import hashlib
import json
from typing import Callable, Optional

_STATE = {"store": None, "rank": 0, "world": 1, "active": 0, "n": 0, "prefix": "milnce_tune"}
_HASH = hashlib.sha1()
_COUNT = [0]


def configure(store, rank: int, world: int, prefix: str = "milnce_tune") -> None:
    """Use ``store`` (a c10d Store shared by every rank) for decisions inside ``region()``."""
    _STATE.update(store=store if world > 1 else None, rank=rank, world=world, prefix=prefix)


def configure_from_process_group() -> bool:
    """configure() from the default torch.distributed group (no-op without one)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() <= 1:
        return False
    from torch.distributed import distributed_c10d as c10d
    configure(c10d._get_default_store(), dist.get_rank(), dist.get_world_size())
    return True


@contextlib.contextmanager
def region(enabled: bool = True):
    """Tuning decisions made inside are rank 0's (when configured and ``enabled``)."""
    if not enabled:
        yield
        return
    _STATE["active"] += 1
    try:
        yield
    finally:
        _STATE["active"] -= 1


def synced() -> bool:
    return _STATE["store"] is not None and _STATE["active"] > 0


def decide(sig: str, tune: Callable[[], int]) -> int:
    """The variant code for problem ``sig``: ``tune()`` here, or rank 0's choice when synced."""
    if synced():
        _STATE["n"] += 1
        key = f"{_STATE['prefix']}/{_STATE['n']}"
        store = _STATE["store"]
        if _STATE["rank"] == 0:
            value = int(tune())
            store.set(key, json.dumps([sig, value]))
        else:
            sig0, value = json.loads(store.get(key).decode())
            if sig0 != sig:
                raise RuntimeError(f"rank {_STATE['rank']}: tuning call {_STATE['n']} is for {sig!r}, rank 0 tuned "
                                   f"{sig0!r}: the ranks ran different shapes inside a synced tuning region")
    else:
        value = int(tune())
    _HASH.update(f"{sig}={value};".encode())
    _COUNT[0] += 1
    return value


def plan_hash() -> Optional[str]:
    """Digest of every tuning decision of this process (None before the first)."""
    return _HASH.hexdigest()[:16] if _COUNT[0] else None


def decisions() -> int:
    return _COUNT[0]
