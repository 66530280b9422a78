"""Soft-DTW sequence-alignment loss family (``loss.py:20-134``), on the native soft-DTW.

The reference defines these but wires none into an entry point; here ``--loss`` selects them
(BASELINE.json config 4) with a sequence batch (``data.synthetic.SyntheticSequences``).
Semantics are reproduced, with the hard-coded constants generalised:

* ``CDTW`` (``loss.py:20-32``): gathered sequences [W*b, n, d] (the reference has b = 1 per
  rank); for each of this rank's own sequences r (rows rank*b .. rank*b+b-1): pos = sdtw(v[r],
  t[r]), neg = sdtw(v[r] vs every gathered t) (the reference's ``repeat(8, ...)`` is world size 8
  at b = 1); loss = mean_r(pos - logsumexp(neg)). gamma 1e-5, cosine. At b = 1 this is the
  reference's v[rank]; with b > 1 every local sequence (hence every local video embedding, the
  only rows the gather's local-slice backward keeps) gets a gradient.
* ``SDTW_CIDM`` (``loss.py:34-68``): contrastive-IDM regulariser on intra-sequence cosine
  distances (sigma 10 s, lambda 1, weights 1/(|dt|+1)) + sdtw(gamma 0.1, cosine); mean.
* ``SDTW_negative`` (``loss.py:70-91``): sdtw(gamma 0.1, cosine) + sum of exp(<v, t>) over all
  non-matching sequences' steps (matching diagonal blocks contribute exp(0) = 1 each, as the
  reference's zero mask does) / (b - 1). The reference's 160 x 8 x 512 is any b x n x d here.
* ``SDTW_3`` (``loss.py:93-134``): InfoNCE with similarity -sdtw(negative_dot, gamma 0.1) over
  all b^2 pairs — video-video, video-text, text-text — computed from ONE [b*n, b*n] GEMM per
  pair type (no [b^2, n, n, d] expand; ~128 GB at b = 1024 in the reference).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.softdtw import SoftDTW


def _cosine_dist(x, y):
    """1 - cos between every pair of steps: [b, n, d] x [b, m, d] -> [b, n, m] (loss.py:41-48)."""
    nx = x.norm(dim=-1, keepdim=True)
    ny = y.norm(dim=-1, keepdim=True)
    cos = torch.matmul(x, y.transpose(1, 2)) / torch.clamp(nx * ny.transpose(1, 2), min=1e-8)
    return 1.0 - cos


class CDTW(nn.Module):
    def __init__(self, args=None):
        super().__init__()
        self.rank = getattr(args, "rank", 0) if args is not None else 0
        self.world = max(1, getattr(args, "world_size", 1) if args is not None else 1)
        self.sdtw = SoftDTW(True, gamma=1e-5, dist_func="cosine")

    def forward(self, video_embd, text_embd):
        total = text_embd.shape[0]
        b = max(1, total // self.world)  # sequences per rank
        r0 = self.rank * b if self.rank * b < total else 0
        v = video_embd[r0:r0 + b]                                          # [b, n, d] local
        pos = self.sdtw(v, text_embd[r0:r0 + b])                           # [b]
        vv = v.unsqueeze(1).expand(-1, total, -1, -1).reshape((b * total,) + tuple(v.shape[1:]))
        tt = text_embd.unsqueeze(0).expand(b, -1, -1, -1).reshape((b * total,) + tuple(text_embd.shape[1:]))
        neg = self.sdtw(vv.contiguous(), tt.contiguous()).view(b, total)  # [b, W*b]
        return (pos - torch.logsumexp(neg, 1)).mean()


class SDTW_CIDM(nn.Module):
    def __init__(self, args=None, lam: float = 1.0, sigma: float = 10.0):
        super().__init__()
        self.lam, self.sigma = lam, sigma
        self.sdtw = SoftDTW(True, gamma=1e-1, dist_func="cosine")

    def forward(self, video_embd, text_embd, start, end=None):
        distance = (start.unsqueeze(2) - start.unsqueeze(1)).abs()
        y = (distance > self.sigma).float()
        w_ = distance + 1
        w = 1 / w_
        D_x = _cosine_dist(video_embd, video_embd)
        D_y = _cosine_dist(text_embd, text_embd)
        I_x = (y * w_ * F.relu(self.lam - D_x) + (1 - y) * w * D_x).sum(1).sum(1)
        I_y = (y * w_ * F.relu(self.lam - D_y) + (1 - y) * w * D_y).sum(1).sum(1)
        dtw = self.sdtw(video_embd, text_embd)
        return torch.mean(I_x + I_y + dtw)


class SDTW_negative(nn.Module):
    def __init__(self, args=None):
        super().__init__()
        self.sdtw = SoftDTW(True, gamma=1e-1, dist_func="cosine")

    def forward(self, video_embd, text_embd):
        b, n, d = video_embd.shape
        sdtw_loss = self.sdtw(video_embd, text_embd)
        pairwise = torch.matmul(video_embd.reshape(-1, d), text_embd.reshape(-1, d).t())  # [b*n, b*n]
        blk = torch.arange(b * n, device=pairwise.device) // n
        same = blk.view(-1, 1) == blk.view(1, -1)
        e = torch.where(same, torch.ones_like(pairwise), torch.exp(pairwise))
        negative_loss = e.sum(1).view(b, n).sum(1)
        return torch.mean(sdtw_loss + negative_loss / (b - 1))


class SDTW_3(nn.Module):
    def __init__(self, args=None):
        super().__init__()
        self.sdtw = SoftDTW(True, gamma=1e-1, dist_func="negative_dot")

    def _infonce(self, a, b_):
        pos = -self.sdtw(a, b_)
        # reference neg[i, j] = -sdtw(a[j], b_[i]) -> transpose of pairwise(a, b_)
        neg = -self.sdtw.pairwise(a, b_).t()
        return torch.mean(torch.logsumexp(neg, 1) - pos)

    def video_video(self, v):
        return self._infonce(v, v)

    def video_text(self, v, t):
        return self._infonce(v, t)

    def text_text(self, t):
        return self._infonce(t, t)

    def forward(self, video_embd, text_embd):
        return self.video_video(video_embd), self.video_text(video_embd, text_embd), self.text_text(text_embd)
