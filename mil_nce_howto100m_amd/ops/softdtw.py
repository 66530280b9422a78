"""Soft-DTW and hard DTW (``soft_dtw_cuda.py``, ``dtw.py``), MI355X-native.

* GPU: the wavefront DP is a HIP kernel (``csrc/softdtw.hip``), one workgroup per pair, one
  lane per row, R kept for the backward; the backward is the reverse wavefront. The distance
  function is fused into both kernels: they read the GEMM output S = X Y^T (one batched GEMM,
  hipBLASLt — never the reference's ``[B, N, M, D]`` expand; the all-pairs form reads every
  pair's block in place from a single ``[b*n, b*m]`` GEMM output) through f(S, row norms), and
  the backward emits dL/dS and the norm terms directly (``_SoftDTWFusedHIP``).
* CPU: a float64 numpy implementation of the same recursions (the oracle for the GPU kernel,
  mirroring the reference's Numba CPU path ``soft_dtw_cuda.py:185-240``).

Distance functions (``soft_dtw_cuda.py:325-363``): ``cosine`` -> exp(1 - cos) (sic),
``negative_dot`` -> -<x, y>, ``euclidean`` -> exp(||x - y||) (sic), ``negative_cosine``
-> -cos (referenced but undefined in the reference), and ``None`` -> squared Euclidean, the
default the reference docstring promises but never assigns (§2.10 item 13).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import use_hip

# ----------------------------------------------------------------------------------------
# distance matrices via GEMM
# ----------------------------------------------------------------------------------------


def _bmm_t(x, y):
    return torch.matmul(x, y.transpose(-1, -2))


def dist_matrix(x: torch.Tensor, y: torch.Tensor, kind: Optional[str]) -> torch.Tensor:
    """x [..., n, d], y [..., m, d] -> [..., n, m] (fp32, or fp64 for fp64 inputs)."""
    if x.dtype != torch.float64:
        x = x.float()
        y = y.float()
    else:
        y = y.double()
    if kind == "negative_dot":
        return -_bmm_t(x, y)
    if kind in ("cosine", "negative_cosine"):
        nx = x.norm(dim=-1, keepdim=True)
        ny = y.norm(dim=-1, keepdim=True)
        cos = _bmm_t(x, y) / torch.clamp(nx * ny.transpose(-1, -2), min=1e-8)
        return torch.exp(1.0 - cos) if kind == "cosine" else -cos
    xx = (x * x).sum(-1, keepdim=True)
    yy = (y * y).sum(-1, keepdim=True).transpose(-1, -2)
    sq = torch.clamp(xx + yy - 2.0 * _bmm_t(x, y), min=0.0)
    if kind == "euclidean":
        return torch.exp(torch.sqrt(_exact_near(sq, x, y, xx + yy) + 1e-12))
    if kind is None or kind == "sqeuclidean":
        return sq
    raise ValueError(f"unknown dist_func {kind}")


# the Gram form ||x||^2 + ||y||^2 - 2<x, y> of a squared distance is rounding noise below about
# this many ulps of the norms' scale (fp32: r = ||x - y|| ~ 3e-3 for unit rows)
_NEAR_ULPS = 64.0


def _exact_near(sq: torch.Tensor, x: torch.Tensor, y: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """``sq`` with the near-duplicate cells (sq at the Gram form's cancellation level) recomputed
    from the explicit difference sum((x_i - y_j)^2), the reference's form
    (``soft_dtw_cuda.py:326-335``): there the euclidean exp(||x - y||) has the finite gradient
    exp(r) (x - y) / r, which a noise-level r would scale arbitrarily. Differentiable (out-of-place
    index_put); identical rows give sq = 0 and a zero gradient."""
    near = sq <= _NEAR_ULPS * torch.finfo(sq.dtype).eps * scale
    if not bool(near.any()):
        return sq
    idx = near.nonzero(as_tuple=True)
    lead, i, j = idx[:-2], idx[-2], idx[-1]
    diff = x[lead + (i,)] - y[lead + (j,)]
    return sq.index_put(idx, (diff * diff).sum(-1))


# ----------------------------------------------------------------------------------------
# CPU oracle (float64)
# ----------------------------------------------------------------------------------------


def softdtw_forward_np(D: np.ndarray, gamma: float, bandwidth: float):
    B, N, M = D.shape
    R = np.full((B, N + 2, M + 2), np.inf)
    R[:, 0, 0] = 0.0
    for p in range(N + M - 1):
        i = np.arange(max(1, p + 2 - M), min(N, p + 1) + 1)
        j = p + 2 - i
        if bandwidth > 0:
            keep = np.abs(i - j) <= bandwidth
            i, j = i[keep], j[keep]
        if i.size == 0:
            continue
        r0 = -R[:, i - 1, j - 1] / gamma
        r1 = -R[:, i - 1, j] / gamma
        r2 = -R[:, i, j - 1] / gamma
        rmax = np.maximum(np.maximum(r0, r1), r2)
        with np.errstate(invalid="ignore", over="ignore"):
            rsum = np.exp(r0 - rmax) + np.exp(r1 - rmax) + np.exp(r2 - rmax)
            R[:, i, j] = D[:, i - 1, j - 1] - gamma * (np.log(rsum) + rmax)
    return R


def softdtw_backward_np(D: np.ndarray, R: np.ndarray, gamma: float, bandwidth: float) -> np.ndarray:
    B, N, M = D.shape
    Dp = np.zeros((B, N + 2, M + 2))
    Dp[:, 1:N + 1, 1:M + 1] = D
    R = R.copy()
    R[:, :, -1] = -np.inf
    R[:, -1, :] = -np.inf
    R[:, -1, -1] = R[:, -2, -2]
    R[np.isinf(R)] = -np.inf
    E = np.zeros((B, N + 2, M + 2))
    E[:, -1, -1] = 1.0
    for p in range(N + M - 2, -1, -1):
        i = np.arange(max(1, p + 2 - M), min(N, p + 1) + 1)
        j = p + 2 - i
        if bandwidth > 0:
            keep = np.abs(i - j) <= bandwidth
            i, j = i[keep], j[keep]
        if i.size == 0:
            continue
        with np.errstate(invalid="ignore", over="ignore"):
            a = np.exp((R[:, i + 1, j] - R[:, i, j] - Dp[:, i + 1, j]) / gamma)
            b = np.exp((R[:, i, j + 1] - R[:, i, j] - Dp[:, i, j + 1]) / gamma)
            c = np.exp((R[:, i + 1, j + 1] - R[:, i, j] - Dp[:, i + 1, j + 1]) / gamma)
        E[:, i, j] = E[:, i + 1, j] * a + E[:, i, j + 1] * b + E[:, i + 1, j + 1] * c
    return E[:, 1:N + 1, 1:M + 1]


class _SoftDTWCPU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, D, gamma, bandwidth):
        Dn = D.detach().cpu().double().numpy()
        R = softdtw_forward_np(Dn, gamma, bandwidth)
        ctx.save_for_backward(D)
        ctx.R, ctx.gamma, ctx.bw = R, gamma, bandwidth
        return torch.from_numpy(R[:, -2, -2].copy()).to(D.device, D.dtype)

    @staticmethod
    def backward(ctx, g):
        (D,) = ctx.saved_tensors
        E = softdtw_backward_np(D.detach().cpu().double().numpy(), ctx.R, ctx.gamma, ctx.bw)
        E = torch.from_numpy(E).to(D.device, D.dtype)
        return g.view(-1, 1, 1) * E, None, None


# ----------------------------------------------------------------------------------------
# GPU kernels
# ----------------------------------------------------------------------------------------


class _SoftDTWHIP(torch.autograd.Function):
    """D: [P, N, M] (layout 'batch') or [b*n, b*m] (layout 'pairs', P = b*b)."""

    @staticmethod
    def forward(ctx, D, gamma, bandwidth, pairs_b):
        from ._lib import call, ptr, stream
        D = D.float().contiguous()  # the kernel reads fp32 distances (R / E are fp64 inside)
        if pairs_b:
            b = pairs_b
            n, m = D.shape[0] // b, D.shape[1] // b
            P, ld, div, s_i, s_j = b * b, D.shape[1], b, n * D.shape[1], m
        else:
            P, n, m = D.shape
            ld, div, s_i, s_j = m, 1, n * m, 0
        R = torch.empty((P, n + 2, m + 2), dtype=torch.float64, device=D.device)
        out = torch.empty((P,), dtype=torch.float32, device=D.device)
        call("milnce_softdtw_fwd", ptr(D), P, n, m, ld, div, s_i, s_j, float(gamma), float(bandwidth),
             0, None, None, 0, 0, 0, 0, ptr(R), ptr(out), stream())
        ctx.save_for_backward(D, R)
        ctx.meta = (gamma, bandwidth, pairs_b, P, n, m, ld, div, s_i, s_j)
        return out

    @staticmethod
    def backward(ctx, g):
        from ._lib import call, ptr, stream
        D, R = ctx.saved_tensors
        gamma, bw, pairs_b, P, n, m, ld, div, s_i, s_j = ctx.meta
        G = torch.empty((P, n, m), dtype=torch.float32, device=D.device)
        call("milnce_softdtw_bwd", ptr(D), ptr(R), P, n, m, ld, div, s_i, s_j, float(gamma), float(bw),
             0, None, None, 0, 0, 0, 0, None, None, ptr(g.float().contiguous()), ptr(G), stream())
        if pairs_b:
            b = pairs_b
            G = G.view(b, b, n, m).permute(0, 2, 1, 3).reshape(b * n, b * m)
        return G, None, None, None


# distance functions the HIP kernels apply to the GEMM output in place (csrc/softdtw.hip DistKind).
# "euclidean" (DK_EUCLID = 5) is not routed here: its gradient needs the explicit difference at
# near-duplicate rows (_exact_near), so it runs as dist_matrix + the raw-distance kernels.
_DIST_KIND = {"negative_dot": 1, "cosine": 2, "negative_cosine": 3, None: 4, "sqeuclidean": 4}


class _SoftDTWFusedHIP(torch.autograd.Function):
    """Soft-DTW of X, Y with the distance function fused into the wavefront kernels
    (``soft_dtw_cuda.py:325-363``): one GEMM S = X Y^T (hipBLASLt) and per-row norms are the only
    other work; the forward reads D = f(S) cell by cell, the backward writes dS = dL/dD * f'(S) in
    S's layout plus the norm terms as per-row coefficients, so dX = dS Y + ca * X, dY = dS^T X +
    cb * Y (two GEMMs and a row-scaled add). No [P, n, m] elementwise pass runs in ATen.
    Layout 'batch': X [P, n, d], Y [P, m, d]; 'pairs' (pairs_b = b): X [b*n, d], Y [b*m, d], all
    b*b pairs from one [b*n, b*m] GEMM."""

    @staticmethod
    def forward(ctx, X, Y, kind, gamma, bandwidth, pairs_b):
        from ._lib import call, ptr, stream
        Xf, Yf = X.float().contiguous(), Y.float().contiguous()
        d = Xf.shape[-1]
        if pairs_b:
            b = pairs_b
            n, m = Xf.shape[0] // b, Yf.shape[0] // b
            S = torch.mm(Xf, Yf.t())
            P, ld, div, s_i, s_j = b * b, b * m, b, n * b * m, m
            a_si, a_sj, b_si, b_sj = n, 0, 0, m
        else:
            P, n, _ = Xf.shape
            m = Yf.shape[1]
            S = torch.bmm(Xf, Yf.transpose(1, 2))
            ld, div, s_i, s_j = m, 1, n * m, 0
            a_si, a_sj, b_si, b_sj = n, 0, m, 0
        stats = kind >= 2
        sq = int(kind >= 4)
        A = Bs = None
        if stats:
            A = torch.empty((Xf.numel() // d,), dtype=torch.float32, device=X.device)
            Bs = torch.empty((Yf.numel() // d,), dtype=torch.float32, device=X.device)
            call("milnce_rowstat", ptr(Xf), A.numel(), d, sq, ptr(A), stream())
            call("milnce_rowstat", ptr(Yf), Bs.numel(), d, sq, ptr(Bs), stream())
        R = torch.empty((P, n + 2, m + 2), dtype=torch.float64, device=X.device)
        out = torch.empty((P,), dtype=torch.float32, device=X.device)
        call("milnce_softdtw_fwd", ptr(S), P, n, m, ld, div, s_i, s_j, float(gamma), float(bandwidth), kind,
             ptr(A), ptr(Bs), a_si, a_sj, b_si, b_sj, ptr(R), ptr(out), stream())
        ctx.save_for_backward(Xf, Yf, S, R, A, Bs)
        ctx.meta = (kind, gamma, bandwidth, pairs_b, P, n, m, ld, div, s_i, s_j, a_si, a_sj, b_si, b_sj,
                    X.dtype, Y.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        from ._lib import call, ptr, stream
        Xf, Yf, S, R, A, Bs = ctx.saved_tensors
        (kind, gamma, bw, pairs_b, P, n, m, ld, div, s_i, s_j, a_si, a_sj, b_si, b_sj, xdt, ydt) = ctx.meta
        dS = torch.empty_like(S)
        stats = kind >= 2
        ca = torch.zeros_like(A) if stats else None
        cb = torch.zeros_like(Bs) if stats else None
        call("milnce_softdtw_bwd", ptr(S), ptr(R), P, n, m, ld, div, s_i, s_j, float(gamma), float(bw), kind,
             ptr(A), ptr(Bs), a_si, a_sj, b_si, b_sj, ptr(ca), ptr(cb), ptr(g.float().contiguous()), ptr(dS),
             stream())
        if pairs_b:
            dX, dY = torch.mm(dS, Yf), torch.mm(dS.t(), Xf)
        else:
            dX, dY = torch.bmm(dS, Yf), torch.bmm(dS.transpose(1, 2), Xf)
        d = Xf.shape[-1]
        if stats:
            call("milnce_rowscale_add", ptr(dX), ptr(Xf), ptr(ca), ca.numel(), d, stream())
            call("milnce_rowscale_add", ptr(dY), ptr(Yf), ptr(cb), cb.numel(), d, stream())
        return dX.to(xdt), dY.to(ydt), None, None, None, None


def _fused_ok(X: torch.Tensor, Y: torch.Tensor, dist_func, pairs: bool) -> bool:
    """GPU tensors, a distance the kernels implement, rows of whole float4s (the row-statistic
    kernels); ``SoftDTW`` then also checks the sequence length against GPU_MAX_N."""
    return use_hip(X) and dist_func in _DIST_KIND and X.shape[-1] % 4 == 0


GPU_MAX_N = 6600  # csrc/softdtw.hip kSdtwMaxN: the LDS ring holds 3 x (N + 2) doubles


def softdtw_from_dist(D: torch.Tensor, gamma: float, bandwidth: float = 0.0) -> torch.Tensor:
    """Batched soft-DTW value of distance matrices D [B, N, M] -> [B]. Longer-than-LDS sequences
    run on the CPU implementation (the reference falls back to CPU above 1024,
    ``soft_dtw_cuda.py:318``; the HIP kernel goes to ~6.6k rows)."""
    if use_hip(D):
        if D.shape[-2] <= GPU_MAX_N:
            return _SoftDTWHIP.apply(D, gamma, bandwidth, 0)
        return _SoftDTWCPU.apply(D.cpu(), gamma, bandwidth).to(D.device)
    return _SoftDTWCPU.apply(D, gamma, bandwidth)


def softdtw_pairwise_from_dist(Dbig: torch.Tensor, b: int, gamma: float, bandwidth: float = 0.0) -> torch.Tensor:
    """All b*b pairs from one [b*n, b*m] distance matrix -> [b, b], out[i, j] = sdtw(block(i, j))."""
    if use_hip(Dbig) and Dbig.shape[0] // b <= GPU_MAX_N:
        return _SoftDTWHIP.apply(Dbig, gamma, bandwidth, b).view(b, b)
    n, m = Dbig.shape[0] // b, Dbig.shape[1] // b
    D = Dbig.view(b, n, b, m).permute(0, 2, 1, 3).reshape(b * b, n, m)
    return _SoftDTWCPU.apply(D, gamma, bandwidth).view(b, b)


class SoftDTW(torch.nn.Module):
    """Drop-in for the reference ``SoftDTW`` (``soft_dtw_cuda.py:274-386``)."""

    def __init__(self, use_cuda: bool = True, gamma: float = 1.0, normalize: bool = False,
                 bandwidth: Optional[float] = None, dist_func: Optional[str] = None):
        super().__init__()
        self.gamma = gamma
        self.normalize = normalize
        self.bandwidth = 0.0 if bandwidth is None else float(bandwidth)
        self.use_cuda = use_cuda  # device placement follows the inputs
        self.dist_func = dist_func

    def _sdtw(self, X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
        if _fused_ok(X, Y, self.dist_func, False) and X.shape[-2] <= GPU_MAX_N:
            return _SoftDTWFusedHIP.apply(X, Y, _DIST_KIND[self.dist_func], self.gamma, self.bandwidth, 0)
        return softdtw_from_dist(dist_matrix(X, Y, self.dist_func), self.gamma, self.bandwidth)

    def forward(self, X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
        assert X.shape[0] == Y.shape[0] and X.shape[2] == Y.shape[2]
        if self.normalize:
            x = torch.cat([X, X, Y])
            y = torch.cat([Y, X, Y])
            out = self._sdtw(x, y)
            out_xy, out_xx, out_yy = torch.split(out, X.shape[0])
            return out_xy - 0.5 * (out_xx + out_yy)
        return self._sdtw(X, Y)

    def pairwise(self, X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
        """[b, n, d] x [b, m, d] -> [b, b] with out[i, j] = sdtw(X[i], Y[j]); one GEMM."""
        b, n, d = X.shape
        m = Y.shape[1]
        if _fused_ok(X, Y, self.dist_func, True) and n <= GPU_MAX_N:
            return _SoftDTWFusedHIP.apply(X.reshape(b * n, d), Y.reshape(b * m, d), _DIST_KIND[self.dist_func],
                                          self.gamma, self.bandwidth, b).view(b, b)
        Dbig = dist_matrix(X.reshape(b * n, d), Y.reshape(b * m, d), self.dist_func)
        return softdtw_pairwise_from_dist(Dbig, b, self.gamma, self.bandwidth)


# ----------------------------------------------------------------------------------------
# hard DTW (dtw.py)
# ----------------------------------------------------------------------------------------


def _dtw_path_np(cost: np.ndarray) -> np.ndarray:
    B, N, M = cost.shape
    path = np.zeros_like(cost)
    path[:, N - 1, M - 1] = 1
    for b in range(B):
        c = cost[b]
        tc = np.full((N, M), np.inf)
        tc[0, 0] = c[0, 0]
        for i in range(1, N):
            tc[i, 0] = tc[i - 1, 0] + c[i, 0]
        for j in range(1, M):
            tc[0, j] = tc[0, j - 1] + c[0, j]
        for i in range(1, N):
            for j in range(1, M):
                tc[i, j] = min(tc[i - 1, j - 1], tc[i - 1, j], tc[i, j - 1]) + c[i, j]
        i, j = N - 1, M - 1
        while not (i == 0 or j == 0):
            r = tc[i, j] - c[i, j]
            if r == tc[i - 1, j - 1]:
                path[b, i - 1, j - 1] = 1; i -= 1; j -= 1
            elif r == tc[i - 1, j]:
                path[b, i - 1, j] = 1; i -= 1
            elif r == tc[i, j - 1]:
                path[b, i, j - 1] = 1; j -= 1
            else:
                break
        path[b, 0, 0] = 1
    return path


class DTW(torch.nn.Module):
    """Hard-DTW alignment loss of ``dtw.py:5-75``: cosine cost, min-plus DP, backtracked path,
    ``logsumexp(sum_i cost*path) - logsumexp(sum_i cost)`` (gradient through the cost only)."""

    def __init__(self, use_cuda: bool = True):
        super().__init__()
        self.use_cuda = use_cuda

    def forward(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        cost = (1.0 - (dist_matrix(x, y, "negative_cosine") * -1.0)).double()
        with torch.no_grad():
            if use_hip(cost):
                from ._lib import call, ptr, stream
                B, N, M = cost.shape
                c = cost.detach().contiguous()
                tc = torch.empty_like(c)
                path = torch.empty_like(c)
                call("milnce_dtw_path", ptr(c), B, N, M, ptr(tc), ptr(path), stream())
            else:
                path = torch.from_numpy(_dtw_path_np(cost.detach().cpu().numpy())).to(cost.device)
        pos = torch.logsumexp(torch.sum(cost * path, dim=1), dim=1)
        neg = torch.logsumexp(torch.sum(cost, dim=1), dim=1)
        return pos - neg
