"""S3D-G video tower + word2vec text tower (the reference model, ``s3dg.py:11-328``).

Parameter/buffer names, shapes, default init and ``state_dict`` keys are identical to the
reference (``nn.Conv3d``/``nn.BatchNorm3d``/``nn.Linear`` are used as parameter containers),
so checkpoints load in both directions. The *execution* is different:

  * activations are channels-last ``[B, T, H, W, C]`` (bf16 on GPU) end to end;
  * every ``STConv3D`` unit (conv -> BN(train stats) -> ReLU, ``s3dg.py:107-111``) is one fused
    op; on GPU it is an MFMA implicit-GEMM conv whose epilogue emits BN partial statistics;
  * the four ``SelfGating`` modules of an Inception block and its ``th.cat`` (``s3dg.py:38-45``)
    are one op that writes each gated branch into its channel slice of the block output;
  * the stem reads the clip as width pairs (8 channels), so its 3x7x7 stride-2 conv becomes an
    ordinary 16-B-operand implicit GEMM (``ops.hip_ops.stem_conv_bn_relu``).

"Separable" is the reference's full-channel (2+1)D factorisation — a ``1 x k x k`` conv
followed by a ``k x 1 x 1`` conv, both Cin->Cout dense (``s3dg.py:74-99``), not depthwise.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from .. import ops
from .text import SentenceEmbedding


_FUSE_STEM_POOL = os.environ.get("MILNCE_FUSE_STEM_POOL", "1") != "0"


def _triple(v) -> Tuple[int, int, int]:
    if isinstance(v, (list, tuple)):
        assert len(v) == 3
        return tuple(int(a) for a in v)
    return (int(v),) * 3


class STConv3D(nn.Module):
    """conv -> BN -> ReLU [-> temporal conv -> BN -> ReLU] (``s3dg.py:61-111``)."""

    def __init__(self, input_dim, output_dim, kernel_size, stride=1, padding=0, separable=False):
        super().__init__()
        assert len(kernel_size) == 3
        self.separable = separable
        k = _triple(kernel_size)
        s = _triple(stride)
        p = _triple(padding)
        if separable:
            # s3dg.py:74-99 ; the k[0]==1 separable case NameErrors in the reference and is unused.
            assert k[0] != 1
            self.k1, self.s1, self.p1 = (1, k[1], k[2]), (1, s[1], s[2]), (0, p[1], p[2])
            self.k2, self.s2, self.p2 = (k[0], 1, 1), (s[0], 1, 1), (p[0], 0, 0)
            self.conv1 = nn.Conv3d(input_dim, output_dim, self.k1, self.s1, self.p1, bias=False)
            self.bn1 = nn.BatchNorm3d(output_dim)
            self.conv2 = nn.Conv3d(output_dim, output_dim, self.k2, self.s2, self.p2, bias=False)
            self.bn2 = nn.BatchNorm3d(output_dim)
        else:
            self.k1, self.s1, self.p1 = k, s, p
            self.conv1 = nn.Conv3d(input_dim, output_dim, k, s, p, bias=False)
            self.bn1 = nn.BatchNorm3d(output_dim)

    def forward(self, x, want_gsum: bool = False, lazy_out: bool = False):
        """Returns z, or (z, per-(clip, channel) sum of z) when ``want_gsum`` (GPU path; the
        sum feeds the following SelfGating's global mean for free). ``lazy_out``: z feeds only
        another STConv3D, which may apply this unit's BN + ReLU in its own conv kernel (GPU)."""
        if self.separable:
            # the spatial conv's BN + ReLU is applied by the temporal conv where its kernel can
            z = ops.conv_bn_relu(x, self.conv1.weight, self.bn1, self.s1, self.p1, self.training, lazy_out=True)
            return ops.conv_bn_relu(z, self.conv2.weight, self.bn2, self.s2, self.p2, self.training, want_gsum,
                                    lazy_out=lazy_out)
        return ops.conv_bn_relu(x, self.conv1.weight, self.bn1, self.s1, self.p1, self.training, want_gsum,
                                lazy_out=lazy_out)


class SelfGating(nn.Module):
    """Parameter container for ``x * sigmoid(fc(mean_THW(x)))`` (``s3dg.py:47-59``)."""

    def __init__(self, input_dim):
        super().__init__()
        self.fc = nn.Linear(input_dim, input_dim)

    def forward(self, x, gsum=None):
        return ops.gate_concat([x], [self.fc.weight], [self.fc.bias], None if gsum is None else [gsum])


class InceptionBlock(nn.Module):
    """Four-branch gated Inception block (``s3dg.py:11-45``)."""

    def __init__(self, input_dim, num_outputs_0_0a, num_outputs_1_0a, num_outputs_1_0b,
                 num_outputs_2_0a, num_outputs_2_0b, num_outputs_3_0b, gating=True):
        super().__init__()
        self.conv_b0 = STConv3D(input_dim, num_outputs_0_0a, [1, 1, 1])
        self.conv_b1_a = STConv3D(input_dim, num_outputs_1_0a, [1, 1, 1])
        self.conv_b1_b = STConv3D(num_outputs_1_0a, num_outputs_1_0b, [3, 3, 3], padding=1, separable=True)
        self.conv_b2_a = STConv3D(input_dim, num_outputs_2_0a, [1, 1, 1])
        self.conv_b2_b = STConv3D(num_outputs_2_0a, num_outputs_2_0b, [3, 3, 3], padding=1, separable=True)
        self.conv_b3_b = STConv3D(input_dim, num_outputs_3_0b, [1, 1, 1])
        self.gating = gating
        self.output_dim = num_outputs_0_0a + num_outputs_1_0b + num_outputs_2_0b + num_outputs_3_0b
        if gating:
            self.gating_b0 = SelfGating(num_outputs_0_0a)
            self.gating_b1 = SelfGating(num_outputs_1_0b)
            self.gating_b2 = SelfGating(num_outputs_2_0b)
            self.gating_b3 = SelfGating(num_outputs_3_0b)

    def forward(self, x):
        g = self.gating
        # branches 0, 1a, 2a are 1x1x1 units on the same input: one fused GEMM on GPU
        # (and the branch-3 pool reads it too: one fused op owning every read of x)
        units = (self.conv_b0, self.conv_b1_a, self.conv_b2_a)
        # z1 / z2 feed only the separable units: their BN + ReLU is applied by those convs' kernels
        # the branches' SelfGating sums are taken in one pass over the block (ops.GSUM_DEFER)
        gs = ops.GSUM_DEFER if g else False
        (z0, z1, z2), s0, pooled = ops.inception_head(x, [u.conv1.weight for u in units],
                                                      [u.bn1 for u in units], self.training, want_gsum0=gs,
                                                      lazy_out=(False, True, True))
        b0 = (z0, s0)
        if ops.branch_streams_enabled(x):
            # branches 2 and 3 on a second compute stream next to branch 1 (their backward follows
            # them there); ops.hip_ops "Branch streams"
            from ..ops import hip_ops
            main = torch.cuda.current_stream(x.device)
            side = hip_ops.branch_stream(x.device)
            side.wait_stream(main)
            hip_ops.record_on((z2, pooled), side)
            with torch.cuda.stream(side):
                b2 = self.conv_b2_b(z2, want_gsum=gs)
                b3 = self.conv_b3_b(pooled, want_gsum=gs)
            b1 = self.conv_b1_b(z1, want_gsum=gs)
            main.wait_stream(side)
            hip_ops.record_on([t for t in (*b2, *b3) if isinstance(t, torch.Tensor)], main)
        else:
            b1 = self.conv_b1_b(z1, want_gsum=gs)
            b2 = self.conv_b2_b(z2, want_gsum=gs)
            b3 = self.conv_b3_b(pooled, want_gsum=gs)
        if not g:
            return torch.cat((z0, b1, b2, b3), dim=-1)
        gates = (self.gating_b0, self.gating_b1, self.gating_b2, self.gating_b3)
        zs, sums = zip(b0, b1, b2, b3)
        return ops.gate_concat(list(zs), [m.fc.weight for m in gates], [m.fc.bias for m in gates], list(sums))


# Inception configs (s3dg.py:223-233): (cin-from-previous, 6 widths)
INCEPTION_CFG = [
    ("mixed_3b", (64, 96, 128, 16, 32, 32)),
    ("mixed_3c", (128, 128, 192, 32, 96, 64)),
    ("maxpool_4a", None),
    ("mixed_4b", (192, 96, 208, 16, 48, 64)),
    ("mixed_4c", (160, 112, 224, 24, 64, 64)),
    ("mixed_4d", (128, 128, 256, 24, 64, 64)),
    ("mixed_4e", (112, 144, 288, 32, 64, 64)),
    ("mixed_4f", (256, 160, 320, 32, 128, 128)),
    ("maxpool_5a", None),
    ("mixed_5b", (256, 160, 320, 32, 128, 128)),
    ("mixed_5c", (384, 192, 384, 48, 128, 128)),
]
ALL_BLOCKS = [n for n, c in INCEPTION_CFG if c is not None]


class S3D(nn.Module):
    """S3D-G + text module (``s3dg.py:207-328``).

    ``blocks`` keeps a prefix/subset of the Inception blocks (the "2-block S3D" plumbing
    config of BASELINE.json); the default keeps all nine. Dropped blocks are not created, so a
    reduced model's state_dict is a strict subset of the full one.
    """

    def __init__(self, num_classes=512, gating=True, space_to_depth=False, word2vec_path="",
                 init="uniform", token_to_word_path="", vocab_size=66250,
                 blocks: Optional[Sequence[str]] = None):
        super().__init__()
        self.num_classes = num_classes
        self.space_to_depth = space_to_depth
        if space_to_depth:
            self.conv1 = STConv3D(24, 64, [2, 4, 4], stride=1, padding=(1, 2, 2), separable=False)
        else:
            self.conv1 = STConv3D(3, 64, [3, 7, 7], stride=2, padding=(1, 3, 3), separable=False)
        self.conv_2b = STConv3D(64, 64, [1, 1, 1], separable=False)
        self.conv_2c = STConv3D(64, 192, [3, 3, 3], padding=1, separable=True)
        # The top-level ``gating`` flag is overwritten by this module in the reference
        # (s3dg.py:212 vs :220) so the stem gate is always applied; reproduced.
        self.gating = SelfGating(192)
        self.maxpool_2a = ((1, 3, 3), (1, 2, 2))
        self.maxpool_3a = ((1, 3, 3), (1, 2, 2))
        self.maxpool_4a = ((3, 3, 3), (2, 2, 2))
        self.maxpool_5a = ((2, 2, 2), (2, 2, 2))
        keep = set(ALL_BLOCKS if blocks is None or len(blocks) == 0 else blocks)
        self._plan: List[str] = []
        dim = 192
        for name, cfg in INCEPTION_CFG:
            if cfg is None:
                self._plan.append(name)
                continue
            if name not in keep:
                continue
            blk = InceptionBlock(dim, *cfg)
            setattr(self, name, blk)
            self._plan.append(name)
            dim = blk.output_dim
        self.feature_dim = dim
        self.fc = nn.Linear(dim, num_classes)
        self.text_module = SentenceEmbedding(num_classes, token_to_word_path=token_to_word_path,
                                             word2vec_path=word2vec_path, num_embeddings=vocab_size)
        if init == "kaiming_normal":  # s3dg.py:240-246
            for m in self.modules():
                if isinstance(m, nn.Conv3d):
                    nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")
                elif isinstance(m, nn.BatchNorm3d):
                    nn.init.constant_(m.weight, 1)
                    nn.init.constant_(m.bias, 0)

    # -------------------------------------------------------------------------------------
    def forward(self, video, text, mode="all", mixed5c=False):
        if mode == "all":
            return self.forward_video(video), self.text_module(text)
        if mode == "video":
            return self.forward_video(video, mixed5c=mixed5c)
        if mode == "text":
            return self.text_module(text)
        raise NotImplementedError(mode)

    def prepare_video(self, video: torch.Tensor) -> torch.Tensor:
        """Bring any accepted clip format to the stem's input layout.

        Accepted: reference float ``[B,3,T,H,W]`` in [0,1]; uint8 ``[B,3,T,H,W]`` (raw loader
        output); native uint8 ``[B,T,H,W,4]`` (RGB + zero pad channel, from the synthetic
        generator). GPU stem input: ``[B,T,H,W,4]`` (channel 3 zero, read as width pairs by the
        stem), uint8 for uint8 clips (the stem kernels scale by 1/255 while staging) else bf16;
        CPU: float ``[B,T,H,W,3]``.
        """
        native = video.dim() == 5 and video.shape[-1] == 4 and video.shape[1] != 3
        if video.is_cuda and ops.use_hip(video) and not self.space_to_depth:
            from ..ops import hip_ops
            return hip_ops.prepare_stem_input(video, native)
        if native:
            v = video[..., :3]
        else:
            v = video.permute(0, 2, 3, 4, 1)
        wdt = self.conv1.conv1.weight.dtype
        if v.dtype == torch.uint8:
            v = v.to(wdt) / 255.0
        v = v.contiguous()
        if video.is_cuda and not ops.keep_dtype():
            return v.to(torch.bfloat16)
        return v.to(wdt)

    def forward_video(self, inputs, mixed5c=False):
        net = self.prepare_video(inputs)
        pooled = False
        if self.space_to_depth:
            net = ops.space_to_depth(net)
            net = self.conv1(net)
        elif net.is_cuda and ops.use_hip(net) and _FUSE_STEM_POOL:
            # stem + BN + ReLU + maxpool_2a in one op: the full-resolution ReLU output is never stored
            net = ops.stem_conv_bn_relu_pool(net, self.conv1.conv1.weight, self.conv1.bn1, self.training,
                                             *self.maxpool_2a)
            pooled = True
        elif net.is_cuda and ops.use_hip(net):
            net = ops.stem_conv_bn_relu(net, self.conv1.conv1.weight, self.conv1.bn1, self.training)
        else:
            net = self.conv1(net)
        if self.space_to_depth:
            net = net[:, 1:, 1:, 1:, :].contiguous()
        if not pooled:
            net = ops.maxpool_tf_same(net, *self.maxpool_2a)
        net = self.conv_2b(net, lazy_out=True)  # BN + ReLU applied by conv_2c's kernel where it can
        net, gsum = self.conv_2c(net, want_gsum=True)
        # SelfGating + maxpool_3a (fused on GPU: the full-resolution gate output is never stored)
        net = ops.gated_maxpool_tf_same(net, gsum, self.gating.fc.weight, self.gating.fc.bias, *self.maxpool_3a)
        for name in self._plan:
            if name.startswith("maxpool"):
                net = ops.maxpool_tf_same(net, *getattr(self, name))
            else:
                net = getattr(self, name)(net)
        net = ops.global_avgpool(net)
        if mixed5c:
            return net
        return self.fc(net.to(self.fc.weight.dtype))
