"""Real-data datasets (HowTo100M train, HMDB-51, MSR-VTT, YouCook2) and the tokenizer.

Sampling logic follows the reference loaders:
  * HowTo100M (``video_loader.py:12-160``): random caption, its window extended to ``min_time``,
    the K temporally nearest captions as MIL candidates, random seek inside the window;
  * HMDB (``hmdb_loader.py``): whole video, ``num_clip`` windows at linspace(0, T - num_frames),
    label = class with the ``_test`` suffix stripped, split1..3; (the reference's flip is a
    no-op bug, §2.10 item 9; here ``with_flip`` really doubles the windows with flipped copies);
  * MSR-VTT / YouCook2 (``msrvtt_loader.py``, ``youcook_loader.py``): ``num_clip`` windows at
    linspace(start, max(start, end - num_sec - 0.4)), caption tokens (max 30 words).

Decoding uses an ``ffmpeg`` binary through a subprocess (crop/scale/fps/hflip filters as in the
reference) and returns uint8 clips **channels-last** ``[T, H, W, 3]`` (batched: the stem's
native layout after a zero 4th channel is appended on device). ffmpeg is not shipped with this
image; without it these datasets raise a clear error and the synthetic generators are used.
"""
from __future__ import annotations

import json
import os
import random
import re
import shutil
import subprocess
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
from torch.utils.data import Dataset


class Tokenizer:
    """Word -> token id (index in dict.npy + 1; 0 = padding), regex ``[\\w']+`` split."""

    def __init__(self, token_to_word_path: str = "", max_words: int = 20, words: Optional[Sequence[str]] = None):
        self.max_words = max_words
        self.word_to_token: Dict[str, int] = {}
        if words is None and token_to_word_path and os.path.isfile(token_to_word_path):
            words = np.load(token_to_word_path, allow_pickle=False)
        for i, t in enumerate(words if words is not None else []):
            self.word_to_token[str(t)] = i + 1

    def __call__(self, sentence) -> torch.Tensor:
        ids = [self.word_to_token[w] for w in re.findall(r"[\w']+", str(sentence)) if w in self.word_to_token]
        out = torch.zeros(self.max_words, dtype=torch.long)
        ids = ids[: self.max_words]
        if ids:
            out[: len(ids)] = torch.tensor(ids, dtype=torch.long)
        return out


def ffmpeg_available() -> bool:
    return shutil.which("ffmpeg") is not None


def decode_clip(path: str, size: int, fps: Optional[float] = None, start: Optional[float] = None,
                duration: Optional[float] = None, crop_only: bool = False, center_crop: bool = True,
                hflip: bool = False, rng: Optional[random.Random] = None) -> np.ndarray:
    """ffmpeg decode -> uint8 [T, size, size, 3]."""
    if not ffmpeg_available():
        raise RuntimeError("ffmpeg not found: real-video datasets need it; use the synthetic generators")
    rng = rng or random
    aw, ah = (0.5, 0.5) if center_crop else (rng.uniform(0, 1), rng.uniform(0, 1))
    filters = []
    if fps:
        filters.append(f"fps={fps}")
    if crop_only:
        filters.append(f"crop={size}:{size}:(iw-{size})*{aw}:(ih-{size})*{ah}")
    else:
        filters.append(f"crop=min(iw\\,ih):min(iw\\,ih):(iw-min(iw\\,ih))*{aw}:(ih-min(iw\\,ih))*{ah}")
        filters.append(f"scale={size}:{size}")
    if hflip:
        filters.append("hflip")
    cmd = ["ffmpeg", "-loglevel", "quiet"]
    if start is not None:
        cmd += ["-ss", str(start)]
    if duration is not None:
        cmd += ["-t", str(duration)]
    cmd += ["-i", path, "-vf", ",".join(filters), "-f", "rawvideo", "-pix_fmt", "rgb24", "pipe:"]
    out = subprocess.run(cmd, capture_output=True, check=True).stdout
    return np.frombuffer(out, np.uint8).reshape(-1, size, size, 3)


def _fit_frames(v: np.ndarray, n: int, size: int) -> np.ndarray:
    if v.shape[0] < n:
        v = np.concatenate([v, np.zeros((n - v.shape[0], size, size, 3), np.uint8)], 0)
    return v[:n]


class HowTo100MDataset(Dataset):
    """Random choices (caption, seek, crop, flip) are drawn from a generator seeded by
    (seed, epoch, index) -- not the process-global ``random`` of the reference -- so an item is the
    same whichever worker loads it and a resumed run sees exactly the data of an uninterrupted one."""

    def __init__(self, csv: str, video_root: str, caption_root: str, tokenizer: Tokenizer, min_time: float = 5.0,
                 fps: int = 10, num_frames: int = 32, size: int = 224, crop_only: bool = True,
                 center_crop: bool = False, random_flip: bool = True, num_candidates: int = 4, seed: int = 0):
        import pandas as pd
        self.seed, self.epoch = int(seed), 0
        self.csv = pd.read_csv(csv)
        self.video_root, self.caption_root, self.tok = video_root, caption_root, tokenizer
        self.min_time, self.fps, self.num_frames, self.size = min_time, fps, num_frames, size
        self.num_sec = num_frames / float(fps)
        self.crop_only, self.center_crop, self.random_flip = crop_only, center_crop, random_flip
        self.k = num_candidates

    def __len__(self):
        return len(self.csv)

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    @staticmethod
    def nearest_candidates(starts, ends, ind: int, k: int) -> int:
        """First index of the k temporally nearest captions around ind (video_loader.py:119-133)."""
        start, end, n = ind, ind, 1
        while n < k:
            if start == 0:
                return 0
            if end == len(starts) - 1:
                return start - (k - n)
            if ends[end] - starts[start - 1] < ends[end + 1] - starts[start]:
                start -= 1
            else:
                end += 1
            n += 1
        return start

    def _text(self, cap: dict, rng: random.Random):
        starts, ends, texts = cap["start"], cap["end"], cap["text"]
        ind = rng.randint(0, len(texts) - 1)
        if self.k == 1:
            words = self.tok(texts[ind])
        else:
            words = torch.zeros(self.k, self.tok.max_words, dtype=torch.long)
            c0 = self.nearest_candidates(starts, ends, ind, self.k)
            for i in range(self.k):
                words[i] = self.tok(texts[max(0, min(len(texts) - 1, c0 + i))])
        s, e = starts[ind], ends[ind]
        if e - s < self.min_time:
            diff = self.min_time - e + s
            s = max(0, s - diff / 2)
            e = s + self.min_time
        return words, int(s), int(e)

    def __getitem__(self, idx):
        vf = self.csv["video_path"][idx]
        vid = vf.split(".")[0]
        with open(os.path.join(self.caption_root, vid + ".json")) as f:
            cap = json.load(f)
        rng = random.Random((self.seed * 1000003 + self.epoch) * 1000003 + int(idx))
        text, s, e = self._text(cap, rng)
        seek = rng.randint(s, int(max(s, e - self.num_sec)))
        flip = self.random_flip and rng.uniform(0, 1) > 0.5
        v = decode_clip(os.path.join(self.video_root, vf), self.size, self.fps, seek, self.num_sec + 0.1,
                        self.crop_only, self.center_crop, flip, rng=rng)
        return {"video": torch.from_numpy(_fit_frames(v, self.num_frames, self.size).copy()), "text": text}


class WindowedClipDataset(Dataset):
    """MSR-VTT / YouCook2 style: ``num_clip`` windows + one caption per row."""

    def __init__(self, csv: str, video_root: str, tokenizer: Tokenizer, num_clip: int = 4, fps: int = 10,
                 num_frames: int = 32, size: int = 224, kind: str = "msrvtt"):
        import pandas as pd
        self.data = pd.read_csv(csv)
        self.root, self.tok, self.nc, self.fps, self.nf, self.size, self.kind = (
            video_root, tokenizer, num_clip, fps, num_frames, size, kind)
        self.num_sec = num_frames / float(fps)

    def __len__(self):
        return len(self.data)

    def _path(self, row) -> str:
        if self.kind == "msrvtt":
            return os.path.join(self.root, row["video_id"] + ".mp4")
        base = os.path.join(self.root, str(row["task"]), row["video_id"])
        for ext in (".mp4", ".mkv", ".webm"):
            if os.path.isfile(base + ext):
                return base + ext
        raise FileNotFoundError(base)

    def __getitem__(self, idx):
        row = self.data.iloc[idx]
        path = self._path(row)
        if self.kind == "msrvtt":
            start, end = 0.0, float(json.loads(subprocess.run(
                ["ffprobe", "-v", "quiet", "-print_format", "json", "-show_format", path],
                capture_output=True, check=True).stdout)["format"]["duration"])
            text = row["sentence"]
        else:
            start, end, text = float(row["start"]), float(row["end"]), row["text"]
        video = torch.zeros(self.nc, self.nf, self.size, self.size, 3, dtype=torch.uint8)
        for i, s in enumerate(np.linspace(start, max(start, end - self.num_sec - 0.4), self.nc)):
            v = decode_clip(path, self.size, self.fps, float(s), self.num_sec + 0.1, False, True)
            video[i] = torch.from_numpy(_fit_frames(v, self.nf, self.size).copy())
        return {"video": video, "text": self.tok(text)}


class HMDBDataset(Dataset):
    def __init__(self, csv: str, video_root: str, num_clip: int = 4, num_frames: int = 32, size: int = 224,
                 with_flip: bool = False):
        import pandas as pd
        self.data = pd.read_csv(csv)
        self.root, self.nc, self.nf, self.size, self.flip = video_root, num_clip, num_frames, size, with_flip

    def __len__(self):
        return len(self.data)

    def meta(self, idx):
        """(label with the ``_test`` suffix stripped, split1, split2, split3) without decoding."""
        row = self.data.iloc[idx]
        label = row["label"][:-5] if row["label"].endswith("_test") else row["label"]
        return label, int(row["split1"]), int(row["split2"]), int(row["split3"])

    def __getitem__(self, idx):
        row = self.data.iloc[idx]
        label = row["label"][:-5] if row["label"].endswith("_test") else row["label"]
        v = decode_clip(os.path.join(self.root, label, row["video_id"]), self.size)
        v = _fit_frames(v, max(self.nf, v.shape[0]), self.size)
        starts = np.linspace(0, v.shape[0] - self.nf, self.nc, dtype=int)
        clips = np.stack([v[s:s + self.nf] for s in starts], 0)
        if self.flip:
            clips = np.concatenate([clips, clips[:, :, :, ::-1]], 0)
        return {"video": torch.from_numpy(clips.copy()), "label": label, "split1": int(row["split1"]),
                "split2": int(row["split2"]), "split3": int(row["split3"])}


def to_model_layout(video_ndhwc3: torch.Tensor) -> torch.Tensor:
    """uint8 [..., T, H, W, 3] -> the stem's native uint8 [..., T, H, W, 4] (zero 4th channel)."""
    pad = torch.zeros(video_ndhwc3.shape[:-1] + (1,), dtype=video_ndhwc3.dtype, device=video_ndhwc3.device)
    return torch.cat([video_ndhwc3, pad], dim=-1)
