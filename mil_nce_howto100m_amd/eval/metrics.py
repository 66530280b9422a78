"""Retrieval metrics (``metrics.py:9-29``): rank of the ground-truth diagonal in each row.

Semantics kept: the rank is the number of entries strictly larger than the diagonal plus the
position among ties (ties with the diagonal each add one entry to ``ind``, exactly like the
reference's ``np.where(sx - d == 0)``), R@k are fractions over ``len(ind)``, MR = median + 1.
"""
from __future__ import annotations

import numpy as np


def compute_metrics(x: np.ndarray) -> dict:
    sx = np.sort(-x, axis=1)
    d = np.diag(-x)[:, np.newaxis]
    ind = np.where(sx - d == 0)[1]
    return {
        "R1": float(np.sum(ind == 0)) / len(ind),
        "R5": float(np.sum(ind < 5)) / len(ind),
        "R10": float(np.sum(ind < 10)) / len(ind),
        "MR": float(np.median(ind) + 1),
    }


def format_metrics(m: dict) -> str:
    return "R@1: {:.4f} - R@5: {:.4f} - R@10: {:.4f} - Median R: {}".format(m["R1"], m["R5"], m["R10"], m["MR"])


def print_computed_metrics(m: dict) -> None:
    print(format_metrics(m))
