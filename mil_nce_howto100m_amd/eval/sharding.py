"""Multi-GPU evaluation without ``nn.DataParallel`` (``eval_hmdb.py:27,32``,
``eval_msrvtt.py:25,30``, ``eval_youcook.py:24,29``).

One process per GPU: rank r embeds batches r, r+W, r+2W, ... of the (deterministic) eval
stream, then the per-batch results are all-gathered and put back in stream order, so every
rank holds exactly the single-process result (rank 0 prints/fits the probe). Works for any
world size, including 1, and for batch counts not divisible by the world size.

Real (ffmpeg-decoded) datasets are sharded by batch index BEFORE loading (``sharded_loader``:
each rank's DataLoader only ever decodes its own batches) and arrive as ``PreSharded``
``(batch index, batch)`` pairs; generated streams are sharded by skipping.
"""
from __future__ import annotations

from typing import Callable, Iterable, Iterator, List, Tuple

import torch.distributed as dist


class PreSharded:
    """An iterable of (global batch index, batch) pairs that already holds only this rank's
    batches."""

    def __init__(self, pairs: Iterable[Tuple[int, object]]):
        self.pairs = pairs

    def __iter__(self):
        return iter(self.pairs)


def shard(batches: Iterable, rank: int, world: int) -> Iterator[Tuple[int, object]]:
    if isinstance(batches, PreSharded):
        yield from batches
        return
    for i, b in enumerate(batches):
        if i % world == rank:
            yield i, b


class _RankBatches:
    """Batch sampler: sequential batches of ``batch_size`` dataset indices, this rank's only."""

    def __init__(self, n: int, batch_size: int, rank: int, world: int):
        self.ids = [i for i in range((n + batch_size - 1) // batch_size) if i % world == rank]
        self.n, self.bs = n, batch_size

    def __iter__(self):
        for i in self.ids:
            yield list(range(i * self.bs, min(self.n, (i + 1) * self.bs)))

    def __len__(self):
        return len(self.ids)


def sharded_loader(dataset, batch_size: int, workers: int, rank: int = 0, world: int = 1,
                   convert: Callable[[object], object] = lambda b: b) -> PreSharded:
    """Decode only this rank's batches of ``dataset`` (sequential batching, no shuffling)."""
    import torch.utils.data as tud
    bs = _RankBatches(len(dataset), batch_size, rank, world)
    loader = tud.DataLoader(dataset, batch_sampler=bs, num_workers=workers)
    return PreSharded((i, convert(b)) for i, b in zip(bs.ids, loader))


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
