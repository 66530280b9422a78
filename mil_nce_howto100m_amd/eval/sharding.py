"""Multi-GPU evaluation without ``nn.DataParallel`` (``eval_hmdb.py:27,32``,
``eval_msrvtt.py:25,30``, ``eval_youcook.py:24,29``).

One process per GPU: rank r embeds batches r, r+W, r+2W, ... of the (deterministic) eval
stream, then the per-batch results are all-gathered and put back in stream order, so every
rank holds exactly the single-process result (rank 0 prints/fits the probe). Works for any
world size, including 1, and for batch counts not divisible by the world size.
"""
from __future__ import annotations

from typing import Callable, Iterable, Iterator, List, Tuple

import torch.distributed as dist


def shard(batches: Iterable, rank: int, world: int) -> Iterator[Tuple[int, object]]:
    for i, b in enumerate(batches):
        if i % world == rank:
            yield i, b


def gather_in_order(items: List[Tuple[int, object]], world: int) -> List[object]:
    """items: this rank's (batch index, result) pairs -> every rank's results in index order."""
    if world <= 1 or not dist.is_initialized():
        return [r for _, r in sorted(items, key=lambda t: t[0])]
    allv: List[List[Tuple[int, object]]] = [None] * world  # type: ignore[list-item]
    dist.all_gather_object(allv, items)
    flat = [t for part in allv for t in part]
    return [r for _, r in sorted(flat, key=lambda t: t[0])]


def map_sharded(fn: Callable[[object], object], batches: Iterable, rank: int = 0, world: int = 1) -> List[object]:
    return gather_in_order([(i, fn(b)) for i, b in shard(batches, rank, world)], world)
