"""HMDB-51 style linear-probe evaluation (``eval_hmdb.py:60-104``).

Features are the 1024-d mixed_5c average-pooled activations (``mode='video', mixed5c=True``)
of ``num_windows`` windows per video. For each of the 3 splits (1 = train, 2 = test,
0 = unused) a LinearSVC(C=100) is fit on every training window; test scores are summed over a
video's windows and arg-maxed; top-1 accuracy per split is reported.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import numpy as np
import torch


@torch.no_grad()
def extract_features(model, batches: Iterable[dict], device, rank: int = 0, world: int = 1):
    """mixed_5c features of every window; with world > 1 each rank embeds its shard of the
    batches and the results are all-gathered in stream order (eval/sharding.py)."""
    from ..utils.hipgraph import GraphedCallable
    from .sharding import map_sharded

    model.eval()
    fwd = GraphedCallable(lambda v: model(v, None, mode="video", mixed5c=True)) if _graphs_ok(device) else \
        (lambda v: model(v, None, mode="video", mixed5c=True))

    def one(data):
        video = data["video"].to(device)
        b, nc = video.shape[0], video.shape[1]
        f = fwd(video.reshape((b * nc,) + tuple(video.shape[2:])))
        return (f.float().view(b, nc, -1).cpu().numpy(), list(data["label"]),
                [np.asarray(data[f"split{k + 1}"]) for k in range(3)])

    res = map_sharded(one, batches, rank, world)
    feats = np.concatenate([r[0] for r in res], 0)
    labels = np.asarray([lab for r in res for lab in r[1]])
    splits = [np.concatenate([r[2][k] for r in res]) for k in range(3)]
    return feats, labels, splits


def _graphs_ok(device) -> bool:
    """HIP-graph replay for the eval forward: GPU with the HIP kernels active (env
    MILNCE_EVAL_GRAPHS=0 disables)."""
    import os
    from .. import ops
    dev = torch.device(device)
    return (dev.type == "cuda" and os.environ.get("MILNCE_EVAL_GRAPHS", "1") != "0"
            and ops.use_hip(torch.empty(0, device=dev)))


def linear_probe(feats: np.ndarray, labels: Sequence, splits: List[np.ndarray], C: float = 100.0,
                 max_iter: int = 1000) -> Dict[str, float]:
    from sklearn import preprocessing
    from sklearn.svm import LinearSVC

    nw, dim = feats.shape[1], feats.shape[2]
    y = preprocessing.LabelEncoder().fit_transform(np.asarray(labels))
    out = {}
    for k, s in enumerate(splits):
        tr, te = np.where(s == 1)[0], np.where(s == 2)[0]
        if len(tr) == 0 or len(te) == 0:
            continue
        clf = LinearSVC(C=C, max_iter=max_iter)
        clf.fit(feats[tr].reshape(-1, dim), y[tr].repeat(nw))
        scores = clf.decision_function(feats[te].reshape(-1, dim))
        scores = scores.reshape(len(te), nw, -1).sum(axis=1)
        out[f"split{k + 1}"] = float(np.mean(np.argmax(scores, axis=1) == y[te]))
    if out:
        out["mean"] = float(np.mean(list(out.values())))
    return out
