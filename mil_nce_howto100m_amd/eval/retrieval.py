"""Zero-shot text-to-video retrieval (``eval_msrvtt.py:57-76``, ``eval_youcook.py:56-75``).

Each item carries ``num_clip`` windows of one video and one caption. The video embedding is
the mean of the window embeddings; similarity = text . video^T; metrics from
``eval.metrics.compute_metrics``. The reference's ``nn.DataParallel`` is replaced by one
process per GPU: with ``world > 1`` each rank embeds its shard of the batches and the
embeddings are all-gathered in stream order (``eval/sharding.py``).
"""
from __future__ import annotations

from typing import Iterable

import numpy as np
import torch

from .metrics import compute_metrics


@torch.no_grad()
def embed_retrieval(model, batches: Iterable[dict], device, rank: int = 0, world: int = 1) -> tuple:
    from ..utils.hipgraph import GraphedCallable
    from .linear_probe import _graphs_ok
    from .sharding import map_sharded

    model.eval()
    fwd = GraphedCallable(lambda v, t: model(v, t)) if _graphs_ok(device) else (lambda v, t: model(v, t))

    def one(data):
        text = data["text"].to(device)
        video = data["video"].to(device)
        b, nc = video.shape[0], video.shape[1]
        video = video.reshape((b * nc,) + tuple(video.shape[2:]))
        v, t = fwd(video, text)
        v = v.float().view(b, nc, -1).mean(dim=1)
        return t.float().cpu().numpy(), v.cpu().numpy()

    res = map_sharded(one, batches, rank, world)
    return np.concatenate([r[0] for r in res], 0), np.concatenate([r[1] for r in res], 0)


def evaluate_retrieval(model, batches: Iterable[dict], device, rank: int = 0, world: int = 1) -> dict:
    t, v = embed_retrieval(model, batches, device, rank, world)
    return compute_metrics(np.dot(t, v.T))
