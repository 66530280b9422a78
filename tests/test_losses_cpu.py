"""MIL-NCE formula, soft-DTW oracle vs brute force + finite differences, the sDTW loss family."""
import itertools
import math

import numpy as np
import pytest
import torch

from mil_nce_howto100m_amd.ops import aten
from mil_nce_howto100m_amd.ops.softdtw import DTW, SoftDTW, softdtw_backward_np, softdtw_forward_np
from mil_nce_howto100m_amd.losses import sdtw as L


def test_milnce_matches_explicit_formula():
    torch.manual_seed(0)
    B, K, D = 5, 3, 8
    v = torch.randn(B, D, dtype=torch.float64)
    t = torch.randn(B * K, D, dtype=torch.float64)
    x = v @ t.t()
    loss = 0.0
    for i in range(B):
        pos = [x[i, i * K + k] for k in range(K)]
        row = [x[i, j] for j in range(B * K)]
        col = [x[r, i * K + k] for r in range(B) for k in range(K)]
        nom = torch.logsumexp(torch.stack(pos), 0)
        den = torch.logsumexp(torch.stack(row + col), 0)
        loss += den - nom
    assert torch.allclose(aten.milnce_loss(v, t), loss / B)


def _softdtw_bruteforce(D, gamma):
    """Soft-min over ALL monotone alignment paths (exponential; tiny sizes only)."""
    n, m = D.shape

    def paths(i, j):
        if i == 0 and j == 0:
            yield [(0, 0)]
            return
        for di, dj in ((1, 0), (0, 1), (1, 1)):
            pi, pj = i - di, j - dj
            if pi >= 0 and pj >= 0:
                for p in paths(pi, pj):
                    yield p + [(i, j)]

    costs = [sum(D[a, b] for a, b in p) for p in paths(n - 1, m - 1)]
    c = np.array(costs)
    return -gamma * (np.log(np.sum(np.exp(-(c - c.min()) / gamma))) - c.min() / gamma)


def test_softdtw_oracle_equals_path_softmin():
    rng = np.random.default_rng(0)
    D = rng.random((2, 4, 3))
    R = softdtw_forward_np(D, 0.7, 0)
    for b in range(2):
        assert abs(R[b, -2, -2] - _softdtw_bruteforce(D[b], 0.7)) < 1e-10


@pytest.mark.parametrize("bw", [0.0, 2.0])
def test_softdtw_gradient_finite_difference(bw):
    torch.manual_seed(1)
    x = torch.randn(2, 5, 3, dtype=torch.float64, requires_grad=True)
    y = torch.randn(2, 6, 3, dtype=torch.float64)
    sd = SoftDTW(False, gamma=0.3, bandwidth=bw if bw else None, dist_func=None)
    assert torch.autograd.gradcheck(lambda a: sd(a, y), (x,), eps=1e-6, atol=1e-5)


def test_softdtw_normalize_and_pairwise():
    torch.manual_seed(2)
    sd = SoftDTW(False, gamma=0.1, normalize=True, dist_func="negative_dot")
    x = torch.randn(3, 4, 5)
    y = torch.randn(3, 4, 5)  # normalize needs equal lengths (it stacks X, X, Y as in the reference)
    out = sd(x, y)
    sdn = SoftDTW(False, gamma=0.1, dist_func="negative_dot")
    ref = sdn(x, y) - 0.5 * (sdn(x, x) + sdn(y, y))
    assert torch.allclose(out, ref, atol=1e-5)
    pw = sdn.pairwise(x, y)
    for i, j in itertools.product(range(3), range(3)):
        assert abs(pw[i, j] - sdn(x[i:i + 1], y[j:j + 1])[0]) < 1e-5


def test_sdtw_losses_run_and_backprop():
    torch.manual_seed(3)
    b, n, d = 4, 5, 16
    v = torch.randn(b, n, d, requires_grad=True)
    t = torch.randn(b, n, d, requires_grad=True)
    start = torch.arange(n).float().view(1, -1).expand(b, -1) * 3.2
    losses = [L.CDTW()(v, t), L.SDTW_CIDM()(v, t, start), L.SDTW_negative()(v, t), sum(L.SDTW_3()(v, t))]
    for l in losses:
        assert torch.isfinite(l)
        v.grad = None
        l.backward(retain_graph=True)
        assert torch.isfinite(v.grad).all()


def test_sdtw3_matches_reference_expand_formulation():
    torch.manual_seed(4)
    b, n, d = 3, 4, 6
    v = torch.randn(b, n, d)
    t = torch.randn(b, n, d)
    sd = SoftDTW(False, gamma=0.1, dist_func="negative_dot")
    row = v.unsqueeze(0).expand(b, b, n, d).reshape(-1, n, d)
    col = t.unsqueeze(1).expand(b, b, n, d).reshape(-1, n, d)
    neg = -sd(row, col).reshape(b, b)
    pos = -sd(v, t)
    ref = torch.mean(torch.logsumexp(neg, 1) - pos)
    assert torch.allclose(L.SDTW_3().video_text(v, t), ref, atol=1e-5)


def test_sdtw_negative_matches_masked_reference_layout():
    torch.manual_seed(5)
    b, n, d = 6, 3, 8
    v, t = torch.randn(b, n, d), torch.randn(b, n, d)
    pairwise = v.reshape(-1, d) @ t.reshape(-1, d).t()
    # reference (loss.py:75-91) with 160 -> b, 8 -> n, 1288 -> b*n + n
    pw = torch.cat(torch.chunk(pairwise, b, 0), 1)
    pw[:, [(b * n + n) * i + j for i in range(b) for j in range(n)]] = 0.0
    pw = torch.cat(torch.chunk(pw, b, 1), 0)
    neg = torch.exp(pw).sum(1).view(b, n).sum(1)
    sd = SoftDTW(False, gamma=0.1, dist_func="cosine")
    ref = torch.mean(sd(v, t) + neg / (b - 1))
    assert torch.allclose(L.SDTW_negative()(v, t), ref, atol=1e-4)


def test_hard_dtw_runs():
    torch.manual_seed(6)
    x = torch.randn(3, 6, 8, requires_grad=True)
    y = torch.randn(3, 6, 8)
    out = DTW(False)(x, y)
    assert out.shape == (3,) and torch.isfinite(out).all()
    out.mean().backward()
    assert torch.isfinite(x.grad).all()


@pytest.mark.parametrize("r", [1e-3, 3e-4])
def test_softdtw_euclidean_near_duplicate_rows_fp32(r):
    """Near-duplicate rows (r ~ 1e-3, below the fp32 Gram form's cancellation level): the fp32
    euclidean soft-DTW value and gradient match float64, because those cells' distances come from
    the explicit difference (ops/softdtw.py _exact_near; reference soft_dtw_cuda.py:326-335)."""
    from mil_nce_howto100m_amd.ops.softdtw import SoftDTW
    torch.manual_seed(5)
    x0 = torch.randn(2, 8, 16) * 0.25
    u = torch.randn(2, 8, 16)
    y0 = x0 + r * u / u.norm(dim=-1, keepdim=True)
    sd = SoftDTW(False, gamma=0.1, dist_func="euclidean")
    x, y = x0.clone().requires_grad_(True), y0.clone().requires_grad_(True)
    out = sd(x, y)
    out.sum().backward()
    xc, yc = x0.double().requires_grad_(True), y0.double().requires_grad_(True)
    outc = sd(xc, yc)
    outc.sum().backward()
    assert torch.allclose(out.double(), outc, atol=1e-5)
    for g, gc in ((x.grad, xc.grad), (y.grad, yc.grad)):
        assert ((g.double() - gc).norm() / gc.norm()).item() < 1e-4
