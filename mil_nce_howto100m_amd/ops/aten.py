"""ATen reference implementations of every fused op, in the framework's NDHWC layout.

These are the CPU path (gloo plumbing runs, unit tests) and the numerical oracle the HIP
kernels are tested against. They are written with plain differentiable torch ops so autograd
derives the backward; the HIP path (``ops/hip_ops.py``) implements forward *and* backward by
hand. Shapes: activations are ``[B, T, H, W, C]`` (channels-last 3-D).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.nn.functional as F


def to_ncdhw(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 4, 1, 2, 3)


def to_ndhwc(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 2, 3, 4, 1).contiguous()


def conv_bn_relu(x, weight, bn, stride, padding, training: bool, relu: bool = True):
    """conv3d(bias=False) -> BatchNorm3d -> ReLU  (reference STConv3D, s3dg.py:89-111)."""
    y = F.conv3d(to_ncdhw(x), weight.to(x.dtype), None, stride, padding)
    y = F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                     training, bn.momentum, bn.eps)
    if training and bn.num_batches_tracked is not None:
        with torch.no_grad():
            bn.num_batches_tracked.add_(1)
    if relu:
        y = F.relu(y)
    return to_ndhwc(y)


def gate_concat(branches: Sequence[torch.Tensor], fc_weights: Sequence[torch.Tensor],
                fc_biases: Sequence[torch.Tensor]) -> torch.Tensor:
    """SelfGating on each branch (s3dg.py:47-59) followed by channel concat (s3dg.py:45)."""
    outs = []
    for z, w, b in zip(branches, fc_weights, fc_biases):
        m = z.to(w.dtype).mean(dim=(1, 2, 3))
        g = torch.sigmoid(F.linear(m, w, b)).to(z.dtype)
        outs.append(z * g[:, None, None, None, :])
    return outs[0] if len(outs) == 1 else torch.cat(outs, dim=-1)


def tf_same_pad(kernel: Sequence[int], stride: Sequence[int]) -> List[Tuple[int, int]]:
    """TF 'SAME' pad amounts per dim (T, H, W) as (before, after); s3dg.py:114-131."""
    pads = []
    for k, s in zip(kernel, stride):
        along = max(k - s, 0)
        pads.append((along // 2, along - along // 2))
    return pads


def maxpool_tf_same(x, kernel, stride):
    """Zero-pad by TF-SAME amounts then MaxPool3d(ceil_mode=True) (s3dg.py:134-146)."""
    (pt0, pt1), (ph0, ph1), (pw0, pw1) = tf_same_pad(kernel, stride)
    y = F.pad(to_ncdhw(x), (pw0, pw1, ph0, ph1, pt0, pt1), value=0.0)
    y = F.max_pool3d(y, kernel, stride, ceil_mode=True)
    return to_ndhwc(y)


def maxpool_s1(x):
    """Inception branch-3 pool: MaxPool3d(3, stride=1, padding=1) (s3dg.py:20)."""
    return to_ndhwc(F.max_pool3d(to_ncdhw(x), 3, 1, 1))


def global_avgpool(x):
    """mean over T, H, W (s3dg.py:323)."""
    return (x.float() if x.dtype in (torch.bfloat16, torch.float16) else x).mean(dim=(1, 2, 3))


def text_relu_max(h: torch.Tensor) -> torch.Tensor:
    """relu then max over words: h [N, W, F] -> [N, F] (s3dg.py:201-202)."""
    return torch.max(F.relu(h), dim=1)[0]


def milnce_loss(video_embd: torch.Tensor, text_embd: torch.Tensor) -> torch.Tensor:
    """MIL-NCE (loss.py:10-18): positives are the K candidates of pair (i, i); the denominator
    is row i of x plus block-column i of x, so positives are counted twice."""
    x = torch.matmul(video_embd, text_embd.t())
    b = video_embd.shape[0]
    x = x.view(b, b, -1)
    eye = torch.eye(b, device=x.device, dtype=x.dtype)
    nominator = (x * eye[:, :, None]).sum(dim=1)
    nominator = torch.logsumexp(nominator, dim=1)
    denominator = torch.cat((x, x.permute(1, 0, 2)), dim=1).view(b, -1)
    denominator = torch.logsumexp(denominator, dim=1)
    return torch.mean(denominator - nominator)


def space_to_depth(x: torch.Tensor) -> torch.Tensor:
    """NDHWC version of s3dg.py:248-253: [B,T,H,W,C] -> [B,T/2,H/2,W/2,8C] with the channel
    order (dt, dh, dw, c) the reference produces (its permute(0,3,5,7,1,2,4,6))."""
    b, t, h, w, c = x.shape
    x = x.view(b, t // 2, 2, h // 2, 2, w // 2, 2, c)
    x = x.permute(0, 1, 3, 5, 2, 4, 6, 7)
    return x.reshape(b, t // 2, h // 2, w // 2, 8 * c)
