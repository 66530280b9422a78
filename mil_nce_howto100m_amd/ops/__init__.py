"""Fused operators of the S3D-G / MIL-NCE hot path.

Dispatch rule (one rule, no per-op fallbacks):
  * tensors on a GPU  -> hand-written HIP kernels in ``libmilnce_hip.so`` (``ops/hip_ops.py``).
    If the library is missing on a GPU box this raises: there is no silent fallback.
  * tensors on CPU    -> the ATen reference implementation (``ops/aten.py``), used for the
    gloo plumbing configuration and as the numerical oracle in tests.

``MILNCE_OPS=aten`` forces the ATen implementation on GPU too; it exists only to A/B the HIP
kernels against MIOpen/hipBLASLt in ``tools/ab_bench.py`` and is never used by bench/smoke.
"""
from __future__ import annotations

import os

import torch

from . import aten

_FORCE_ATEN = os.environ.get("MILNCE_OPS", "") == "aten"


# want_gsum value of the Inception branches: their SelfGating sums may be computed by one pass over
# the whole block inside gate_concat instead of one pass per branch (hip_ops.GSUM_DEFER)
GSUM_DEFER = 2


def use_hip(t: torch.Tensor) -> bool:
    return t.is_cuda and not _FORCE_ATEN


_KEEP_DTYPE = False


def keep_dtype() -> bool:
    """True inside ``force_aten(keep_dtype=True)``: the ATen path on GPU computes in the model's
    parameter dtype (an fp32 reference) instead of bf16 activations."""
    return _KEEP_DTYPE


class force_aten:
    """Context manager: run the ATen implementations on GPU too (A/B comparisons in tests).
    ``keep_dtype=True`` also keeps the activations in the parameters' dtype (fp32 oracle)."""

    def __init__(self, keep_dtype: bool = False):
        self.keep = keep_dtype

    def __enter__(self):
        global _FORCE_ATEN, _KEEP_DTYPE
        self._prev, _FORCE_ATEN = _FORCE_ATEN, True
        self._prev_keep, _KEEP_DTYPE = _KEEP_DTYPE, self.keep

    def __exit__(self, *exc):
        global _FORCE_ATEN, _KEEP_DTYPE
        _FORCE_ATEN = self._prev
        _KEEP_DTYPE = self._prev_keep


def branch_streams_enabled(x: torch.Tensor) -> bool:
    """Inception branches 2 / 3 on a second compute stream (hip_ops "Branch streams")."""
    return use_hip(x) and _hip().branch_streams_enabled(x)


def _hip():
    from . import hip_ops  # imported lazily: loads (and checks) the native library
    return hip_ops


def conv_bn_relu(x, weight, bn, stride, padding, training: bool, want_gsum: bool = False,
                 lazy_out: bool = False):
    """conv -> BN -> ReLU. With ``want_gsum`` also returns the per-(clip, channel) sum of the
    output (fp32 [B, C]) that a following SelfGating needs (None on the ATen path).
    ``lazy_out`` (GPU): the caller feeds the output only to another ``conv_bn_relu``, which may
    apply this BN + ReLU inside its own kernel (the output is then a placeholder)."""
    if use_hip(x):
        return _hip().conv_bn_relu(x, weight, bn, stride, padding, training, want_gsum, lazy_out)
    z = aten.conv_bn_relu(x, weight, bn, stride, padding, training)
    return (z, None) if want_gsum else z


def stem_conv_bn_relu(x, weight, bn, training: bool):
    """S3D-G conv1 unit on the prepared bf16 [B,T,H,W,4] clip (GPU paired-width stem)."""
    return _hip().stem_conv_bn_relu(x, weight, bn, training)


def stem_conv_bn_relu_pool(x, weight, bn, training: bool, pool_k, pool_s):
    """Stem unit + maxpool_2a in one fused op (GPU)."""
    return _hip().stem_conv_bn_relu_pool(x, weight, bn, training, pool_k, pool_s)


def conv1x1_group_bn_relu(x, weights, bns, training: bool, want_gsum0: bool = False):
    """Several 1x1x1 conv -> BN -> ReLU units on the same input (one fused GEMM on GPU).
    Returns the list of outputs and the gating sum of the first (None on the ATen path)."""
    if use_hip(x):
        out = _hip().conv1x1_group_bn_relu(x, weights, bns, training, want_gsum0)
        n = len(weights)
        return list(out[:n]), (out[n] if want_gsum0 else None)
    return [aten.conv_bn_relu(x, w, bn, (1, 1, 1), (0, 0, 0), training) for w, bn in zip(weights, bns)], None


def inception_head(x, weights, bns, training: bool, want_gsum0: bool = False, lazy_out=()):
    """Everything an Inception block computes directly from its input: the 1x1x1 conv-BN-ReLU
    units of branches 0/1a/2a and the branch-3 stride-1 max pool. Returns
    ([z0, z1a, z2a], gating sum of z0 or None, pooled x); one fused op on GPU. ``lazy_out[i]``
    (GPU): z_i feeds only a ``conv_bn_relu``, which may apply its BN + ReLU (placeholder output)."""
    if use_hip(x):
        out = _hip().inception_head(x, weights, bns, training, want_gsum0, lazy_out)
        n = len(weights)
        return list(out[:n]), (out[n] if want_gsum0 else None), out[-1]
    zs = [aten.conv_bn_relu(x, w, bn, (1, 1, 1), (0, 0, 0), training) for w, bn in zip(weights, bns)]
    return zs, None, aten.maxpool_s1(x)


def gate_concat(branches, fc_weights, fc_biases, gsums=None):
    if use_hip(branches[0]):
        return _hip().gate_concat(branches, fc_weights, fc_biases, gsums)
    return aten.gate_concat(branches, fc_weights, fc_biases)


def maxpool_tf_same(x, kernel, stride):
    if use_hip(x):
        return _hip().maxpool3d(x, kernel, stride, tf_same=True)
    return aten.maxpool_tf_same(x, kernel, stride)


def gated_maxpool_tf_same(z, gsum, fc_weight, fc_bias, kernel, stride):
    """SelfGating(z) then a TF-SAME max pool (conv_2c -> gating -> maxpool_3a)."""
    if use_hip(z):
        return _hip().gated_maxpool(z, gsum, fc_weight, fc_bias, kernel, stride)
    return aten.maxpool_tf_same(aten.gate_concat([z], [fc_weight], [fc_bias]), kernel, stride)


def maxpool_s1(x):
    if use_hip(x):
        return _hip().maxpool3d(x, (3, 3, 3), (1, 1, 1), tf_same=False)
    return aten.maxpool_s1(x)


def global_avgpool(x):
    if use_hip(x):
        return _hip().global_avgpool(x)
    return aten.global_avgpool(x)


def text_relu_max(h):
    if use_hip(h):
        return _hip().text_relu_max(h)
    return aten.text_relu_max(h)


def milnce_loss(video_embd, text_embd):
    if use_hip(video_embd):
        return _hip().milnce_loss(video_embd, text_embd)
    return aten.milnce_loss(video_embd, text_embd)


def space_to_depth(x):
    return aten.space_to_depth(x)
