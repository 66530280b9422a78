"""Training data feeds: the on-device synthetic generator or the real HowTo100M pipeline.

Real data (``--synthetic 0``) follows the reference (``main_distributed.py:102-141, 185-187``,
``video_loader.py:12-160``):

* ``HowTo100MDataset`` items (ffmpeg decode, nearest-caption candidates);
* ``EpochRankSampler``: ``DistributedSampler`` semantics (a seeded per-epoch permutation padded to
  a multiple of the world size, rank-strided, ``set_epoch``) plus a start offset so a mid-epoch
  checkpoint resumes on the next unseen batch instead of replaying the epoch;
* ``DataLoader(batch_size=local, drop_last=True, pin_memory, num_workers=num_thread_reader /
  ngpus)`` (the reference divides both per GPU, ``main_distributed.py:88-90``);
* ``DevicePrefetcher``: the H2D copy of batch i+1 and its conversion to the stem's native layout
  (uint8 ``[b, T, H, W, 4]``) run on a side HIP stream while step i computes; the compute stream
  waits on an event before using the batch.

Both feeds expose ``steps_per_epoch`` and ``epoch(epoch, start_step)`` yielding device batches
``{"video", "text", ...}`` so the trainer's loop is the same for both.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Iterator, Optional

import torch
from torch.utils.data import DataLoader, Sampler


class EpochRankSampler(Sampler):
    """Rank-strided sampler over a seeded per-epoch permutation (DistributedSampler semantics)."""

    def __init__(self, n: int, rank: int = 0, world: int = 1, shuffle: bool = True, seed: int = 0):
        self.n, self.rank, self.world, self.shuffle, self.seed = n, rank, world, shuffle, seed
        self.epoch = 0
        self.start = 0  # samples of this rank's shard to skip (mid-epoch resume)
        self.per_rank = int(math.ceil(n / float(world)))

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def set_start(self, samples: int) -> None:
        self.start = max(0, int(samples))

    def indices(self) -> list:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g).tolist()
        else:
            order = list(range(self.n))
        total = self.per_rank * self.world
        order += order[: total - len(order)]  # pad by wrapping, like DistributedSampler
        return order[self.rank:total:self.world]

    def __iter__(self):
        return iter(self.indices()[self.start:])

    def __len__(self) -> int:
        return max(0, self.per_rank - self.start)


def _collate_layout(video: torch.Tensor, device: torch.device) -> torch.Tensor:
    """uint8 [b, T, H, W, 3] (host) -> device [b, T, H, W, 4] with a zero 4th channel."""
    v = video.to(device, non_blocking=True)
    out = torch.zeros(v.shape[:-1] + (4,), dtype=torch.uint8, device=device)
    out[..., :3] = v
    return out


class DevicePrefetcher:
    """Iterate a DataLoader with the next batch's H2D copy + layout conversion overlapped with
    the current step (side stream + event on GPU; plain conversion on CPU)."""

    def __init__(self, loader, device: torch.device):
        self.loader, self.device = loader, device
        self.cuda = device.type == "cuda"
        self.stream = torch.cuda.Stream(device=device) if self.cuda else None

    def _convert(self, b: Dict) -> Dict:
        out = dict(b)
        out["video"] = _collate_layout(b["video"], self.device)
        out["text"] = b["text"].to(self.device, non_blocking=True)
        return out

    def __iter__(self) -> Iterator[Dict]:
        it = iter(self.loader)
        if not self.cuda:
            for b in it:
                yield self._convert(b)
            return
        nxt = self._stage(it)
        while nxt is not None:
            batch, ev = nxt
            torch.cuda.current_stream(self.device).wait_event(ev)
            for t in batch.values():
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(torch.cuda.current_stream(self.device))
            nxt = self._stage(it)  # issue the following copy before handing this batch out
            yield batch

    def _stage(self, it):
        try:
            b = next(it)
        except StopIteration:
            return None
        with torch.cuda.stream(self.stream):
            batch = self._convert(b)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return batch, ev


class PrefetchedBatches:
    """``batch(step)`` of an on-device generator (SyntheticClips / SyntheticSequences) with the next
    step's batch generated on a side stream while the current step runs, as a DataLoader's workers
    prefetch: every call still generates one batch (the next one), the step only waits for the
    event of its own. The side stream starts each batch after the work queued so far (the previous
    step), so it overlaps the current step's forward; the batch tensors are recorded on the
    consuming stream for the allocator."""

    def __init__(self, data, device: torch.device):
        self.data, self.device = data, device
        self.stream = torch.cuda.Stream(device=device)
        self.next = None
        self.epoch_len = getattr(data, "epoch_len", 0)

    def __len__(self) -> int:
        return len(self.data)

    def batch(self, step: int) -> Dict:
        main = torch.cuda.current_stream(self.device)
        if self.next is not None and self.next[0] == step:
            _, b, ev = self.next
            main.wait_event(ev)
            for t in b.values():
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(main)
        else:
            b = self.data.batch(step)
        self.stream.wait_stream(main)
        with torch.cuda.stream(self.stream):
            nb = self.data.batch(step + 1)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.next = (step + 1, nb, ev)
        return b


class SyntheticFeed:
    def __init__(self, data):
        self.data = data
        self.steps_per_epoch = len(data)

    @property
    def epoch_len(self) -> int:
        return self.data.epoch_len

    def epoch(self, epoch: int, start_step: int = 0) -> Iterator[Dict]:
        for i in range(start_step, self.steps_per_epoch):
            yield self.data.batch(epoch * self.steps_per_epoch + i)


class HowTo100MFeed:
    def __init__(self, dataset, local_bs: int, rank: int, world: int, device: torch.device, workers: int,
                 pin_memory: bool, seed: int, max_steps: int = 0):
        self.ds, self.b, self.device = dataset, local_bs, device
        self.sampler = EpochRankSampler(len(dataset), rank, world, shuffle=True, seed=seed)
        self.loader = DataLoader(dataset, batch_size=local_bs, sampler=self.sampler, drop_last=True,
                                 num_workers=workers, pin_memory=pin_memory and device.type == "cuda",
                                 persistent_workers=False)
        full = self.sampler.per_rank // local_bs
        self.steps_per_epoch = min(full, max_steps) if max_steps else full
        self.epoch_len = len(dataset)

    def epoch(self, epoch: int, start_step: int = 0) -> Iterator[Dict]:
        self.sampler.set_epoch(epoch)
        self.sampler.set_start(start_step * self.b)
        if hasattr(self.ds, "set_epoch"):
            self.ds.set_epoch(epoch)  # workers get a fresh copy of the dataset per epoch
        for i, batch in enumerate(DevicePrefetcher(self.loader, self.device), start=start_step):
            if i >= self.steps_per_epoch:
                break
            yield batch


def _resolve(path: str) -> str:
    """Reference paths are relative to the script dir (video_loader.py:36); accept cwd too."""
    if not path or os.path.exists(path):
        return path
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    cand = os.path.join(root, path)
    return cand if os.path.exists(cand) else path


def build_train_feed(args, ctx, local_bs: int):
    """The training data feed selected by ``--synthetic`` (1: on-device generator, 0: HowTo100M)."""
    from .synthetic import SyntheticClips, SyntheticSequences
    loss = getattr(args, "loss", "milnce")
    if args.synthetic:
        clips_per_step = local_bs
        if loss != "milnce":
            if local_bs % args.seq_len:
                raise ValueError(f"--batch_size per GPU ({local_bs}) must be a multiple of --seq_len ({args.seq_len})")
        data = SyntheticClips(clips_per_step, args.num_frames, args.video_size, args.num_candidates,
                              args.max_words, args.vocab_size, seed=args.seed, device=ctx.device,
                              rank=ctx.rank, world_size=ctx.world_size, epoch_len=args.synthetic_len)
        if loss != "milnce":
            # --batch_size counts clips (as in bench.py): local_bs // seq_len sequences per GPU
            data = SyntheticSequences(local_bs // args.seq_len, args.seq_len, data)
        feed = SyntheticFeed(data)
        if args.steps_per_epoch:
            feed.steps_per_epoch = min(feed.steps_per_epoch, args.steps_per_epoch)
        return feed
    if loss != "milnce":
        raise ValueError("--synthetic 0 provides HowTo100M clip+caption batches (video_loader.py); the soft-DTW "
                         "losses need sequence batches, which only the synthetic generator provides")
    from .datasets import HowTo100MDataset, Tokenizer
    csv, vroot, croot = _resolve(args.train_csv), _resolve(args.video_path), _resolve(args.caption_root)
    for what, p in (("--train_csv", csv), ("--video_path", vroot), ("--caption_root", croot)):
        if not os.path.exists(p):
            raise FileNotFoundError(f"{what} {p!r} does not exist (--synthetic 0 needs the HowTo100M files)")
    tok = Tokenizer(getattr(args, "token_to_word_path", ""), max_words=args.max_words)
    ds = HowTo100MDataset(csv, vroot, croot, tok, min_time=args.min_time, fps=args.fps, num_frames=args.num_frames,
                          size=args.video_size, crop_only=bool(args.crop_only), center_crop=bool(args.centercrop),
                          random_flip=bool(args.random_flip), num_candidates=args.num_candidates, seed=args.seed)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(ctx.world_size)))
    workers = max(0, args.num_thread_reader // max(1, local_world))
    return HowTo100MFeed(ds, local_bs, ctx.rank, ctx.world_size, ctx.device, workers, bool(args.pin_memory),
                         args.seed, args.steps_per_epoch)
