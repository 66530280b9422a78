"""On-device synthetic clip + caption generator (replaces the ffmpeg loader's role).

The reference decodes HowTo100M with one ffmpeg subprocess per clip (``video_loader.py:58-95``)
and needs ~40 CPU cores per 4 GPUs (README.md:118). Here a batch is produced directly in HBM
in the stem's native layout (uint8 ``[B, T, H, W, 4]``: RGB + a zero pad channel), so the
benchmark measures the model, not the host.

The data has learnable structure so "loss decreases" is a meaningful check: every sample
belongs to one of ``num_classes`` latent classes; the class sets the clip's colour, the
spatial frequency and drift of a moving grating, and the first few word slots of each of its
K captions (class-specific token ids), the rest of the words are random. Samples are a pure
function of (seed, sample index), so a DistributedSampler-like rank stride gives disjoint,
reproducible shards. On GPU the video is produced by a HIP kernel (``csrc/misc.hip (synth_video_kernel)``).
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional

import torch

from .. import ops


M32 = 0xFFFFFFFF
_SYNTH_META = os.environ.get("MILNCE_SYNTH_META", "1") != "0"


def _mix(x: torch.Tensor) -> torch.Tensor:
    """32-bit integer hash on int64 tensors; bit-identical to ``mix32`` in csrc/misc.hip (synth_video_kernel)."""
    x = x & M32
    x = (((x >> 16) ^ x) * 0x45D9F3B) & M32
    x = (((x >> 16) ^ x) * 0x45D9F3B) & M32
    return ((x >> 16) ^ x) & 0x7FFFFFFF


class SyntheticClips:
    def __init__(self, batch_size: int, num_frames: int = 16, size: int = 200, num_candidates: int = 4,
                 max_words: int = 20, vocab_size: int = 66250, num_classes: int = 64, seed: int = 1,
                 device: torch.device = torch.device("cpu"), rank: int = 0, world_size: int = 1,
                 epoch_len: int = 1238911, layout: str = "native"):
        self.b, self.t, self.s = batch_size, num_frames, size
        self.k, self.w, self.vocab = num_candidates, max_words, vocab_size
        self.ncls, self.seed, self.device = num_classes, seed, device
        self.rank, self.world = rank, world_size
        self.epoch_len = epoch_len
        self.layout = layout
        self.class_words = 4  # leading word slots carrying the class

    def __len__(self) -> int:
        """Batches per epoch per rank (drop_last=True, main_distributed.py:136)."""
        return max(1, self.epoch_len // (self.b * self.world))

    def sample_ids(self, step: int) -> torch.Tensor:
        base = (step * self.world + self.rank) * self.b
        return torch.arange(base, base + self.b, device=self.device, dtype=torch.int64)

    def labels(self, ids: torch.Tensor) -> torch.Tensor:
        return _mix(ids * 7919 + self.seed) % self.ncls

    def text(self, ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        b = ids.shape[0]
        kk = torch.arange(self.k, device=self.device).view(1, self.k, 1)
        ww = torch.arange(self.w, device=self.device).view(1, 1, self.w)
        h = _mix(ids.view(b, 1, 1) * 1000003 + kk * 8191 + ww * 131 + self.seed)
        rand_tok = 1 + (h % (self.vocab - 1))
        cls_tok = 1 + ((labels.view(b, 1, 1) * self.class_words + ww) % (self.vocab - 1))
        tok = torch.where(ww < self.class_words, cls_tok, rand_tok)
        return tok.long()

    def video(self, ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        if self.device.type == "cuda" and ops.use_hip(torch.empty(0, device=self.device)):
            from ..ops import hip_ops
            v = hip_ops.synth_video(labels.to(torch.int32), ids.to(torch.int32), self.t, self.s, self.seed)
        else:
            v = self._video_torch(ids, labels)
        if self.layout == "reference":
            v = v[..., :3].permute(0, 4, 1, 2, 3).contiguous()
        return v

    def _video_torch(self, ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """Reference implementation of csrc/misc.hip (synth_video_kernel) (same formula)."""
        b, t, s = ids.shape[0], self.t, self.s
        lab = labels.view(b, 1, 1, 1, 1).float()
        tt = torch.arange(t, device=self.device).view(1, t, 1, 1, 1).float()
        yy = torch.arange(s, device=self.device).view(1, 1, s, 1, 1).float()
        xx = torch.arange(s, device=self.device).view(1, 1, 1, s, 1).float()
        ch = torch.arange(3, device=self.device).view(1, 1, 1, 1, 3).float()
        freq = 0.05 + 0.01 * torch.remainder(lab, 7.0)
        drift = 0.5 + 0.25 * torch.remainder(lab, 5.0)
        color = 64.0 + 48.0 * torch.remainder(lab * 3.0 + ch * 5.0, 4.0)
        wave = torch.sin(freq * (xx + yy * (1.0 + 0.1 * ch)) + drift * tt)
        hid = _mix(ids.view(b, 1, 1, 1, 1) * 65537 + (tt.long() * s + yy.long()) * s + xx.long())
        noise = (hid % 64).float() - 32.0
        v = torch.clamp(color + 60.0 * wave + noise, 0.0, 255.0).to(torch.uint8)
        pad = torch.zeros((b, t, s, s, 1), dtype=torch.uint8, device=self.device)
        return torch.cat([v, pad], dim=-1).contiguous()

    def batch(self, step: int) -> Dict[str, torch.Tensor]:
        if self.device.type == "cuda" and _SYNTH_META and ops.use_hip(torch.empty(0, device=self.device)):
            # labels + captions in one launch, then the video kernel (same formulas as below)
            from ..ops import hip_ops
            base = (step * self.world + self.rank) * self.b
            tok, labels, lab32, ids32 = hip_ops.synth_meta(base, self.b, self.k, self.w, self.vocab, self.ncls,
                                                           self.seed, self.class_words, self.device)
            v = hip_ops.synth_video(lab32, ids32, self.t, self.s, self.seed)
            if self.layout == "reference":
                v = v[..., :3].permute(0, 4, 1, 2, 3).contiguous()
            return {"video": v, "text": tok, "label": labels}
        ids = self.sample_ids(step)
        labels = self.labels(ids)
        return {"video": self.video(ids, labels), "text": self.text(ids, labels), "label": labels}


class SyntheticSequences:
    """Sequences of ``seq_len`` consecutive clips with start/end times, for the soft-DTW loss
    family (loss.py:20-134 assume such a loader; the reference ships none)."""

    def __init__(self, batch_size: int, seq_len: int, clips: SyntheticClips, clip_sec: float = 3.2):
        self.b, self.n, self.clips, self.clip_sec = batch_size, seq_len, clips, clip_sec
        self.epoch_len = clips.epoch_len

    def __len__(self) -> int:
        return max(1, self.epoch_len // (self.b * self.n * self.clips.world))

    def batch(self, step: int) -> Dict[str, torch.Tensor]:
        c = self.clips
        base = (step * c.world + c.rank) * self.b
        seq_ids = torch.arange(base, base + self.b, device=c.device, dtype=torch.int64)
        ids = (seq_ids.view(-1, 1) * self.n + torch.arange(self.n, device=c.device).view(1, -1)).reshape(-1)
        labels = c.labels(ids)
        video = c.video(ids, labels)
        text = c.text(ids, labels)[:, 0]  # one caption per step
        start = (torch.arange(self.n, device=c.device).float() * self.clip_sec).view(1, -1).expand(self.b, -1)
        return {"video": video, "text": text, "label": labels.view(self.b, self.n),
                "start": start.contiguous(), "end": (start + self.clip_sec).contiguous()}


class SyntheticEvalSet:
    """Labelled multi-window clips for the eval pipelines (linear probe / retrieval).

    Video v has latent class ``labels(v)``; each of its ``num_clip`` windows is a different
    sample of that class; its caption carries the class words. ``split{1,2,3}`` mimic the HMDB
    CSV (1 = train, 2 = test, 0 = unused). Layout per batch: video uint8 [b, nc, T, S, S, 4].
    """

    def __init__(self, num_videos: int, num_clip: int = 4, num_frames: int = 16, size: int = 64,
                 num_classes: int = 8, max_words: int = 30, vocab_size: int = 66250, seed: int = 3,
                 device: torch.device = torch.device("cpu")):
        self.n, self.nc = num_videos, num_clip
        self.clips = SyntheticClips(1, num_frames, size, 1, max_words, vocab_size, num_classes, seed, device)

    def batches(self, batch_size: int):
        c = self.clips
        for s in range(0, self.n, batch_size):
            vids = torch.arange(s, min(self.n, s + batch_size), device=c.device)
            labels = c.labels(vids)
            ids = (vids.view(-1, 1) * 1000 + torch.arange(self.nc, device=c.device).view(1, -1)).reshape(-1)
            video = c.video(ids, labels.repeat_interleave(self.nc))
            b = vids.shape[0]
            video = video.view((b, self.nc) + tuple(video.shape[1:]))
            text = c.text(vids * 1000 + 7, labels)[:, 0]
            split = [(((vids + k) % 3) != 0).long() + ((vids + k) % 3 == 0).long() * 2 for k in range(3)]
            yield {"video": video, "text": text, "label": [f"class{int(l)}" for l in labels.tolist()],
                   "split1": split[0].cpu(), "split2": split[1].cpu(), "split3": split[2].cpu()}
