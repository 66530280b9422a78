"""Zero-shot text-to-video retrieval (``eval_msrvtt.py:57-76``, ``eval_youcook.py:56-75``).

Each item carries ``num_clip`` windows of one video and one caption. The video embedding is
the mean of the window embeddings; similarity = text . video^T; metrics from
``eval.metrics.compute_metrics``. Runs single-GPU (the reference's ``nn.DataParallel`` is
replaced by one process per GPU; shard the dataset with ``rank/world`` to use more GPUs and
``all_gather`` the embeddings).
"""
from __future__ import annotations

from typing import Iterable

import numpy as np
import torch

from .metrics import compute_metrics


@torch.no_grad()
def embed_retrieval(model, batches: Iterable[dict], device) -> tuple:
    model.eval()
    txt, vid = [], []
    for data in batches:
        text = data["text"].to(device)
        video = data["video"].to(device)
        b, nc = video.shape[0], video.shape[1]
        video = video.reshape((b * nc,) + tuple(video.shape[2:]))
        v, t = model(video, text)
        v = v.float().view(b, nc, -1).mean(dim=1)
        txt.append(t.float().cpu().numpy())
        vid.append(v.cpu().numpy())
    return np.concatenate(txt, 0), np.concatenate(vid, 0)


def evaluate_retrieval(model, batches: Iterable[dict], device) -> dict:
    t, v = embed_retrieval(model, batches, device)
    return compute_metrics(np.dot(t, v.T))
