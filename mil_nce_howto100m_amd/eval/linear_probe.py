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
def extract_features(model, batches: Iterable[dict], device):
    model.eval()
    feats, labels, splits = [], [], [[], [], []]
    for data in batches:
        video = data["video"].to(device)
        b, nc = video.shape[0], video.shape[1]
        f = model(video.reshape((b * nc,) + tuple(video.shape[2:])), None, mode="video", mixed5c=True)
        feats.append(f.float().view(b, nc, -1).cpu().numpy())
        labels.extend(list(data["label"]))
        for k in range(3):
            splits[k].append(np.asarray(data[f"split{k + 1}"]))
    return np.concatenate(feats, 0), np.asarray(labels), [np.concatenate(s) for s in splits]


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
