"""MIL-NCE loss module (``loss.py:6-18``).

On GPU the logits GEMM runs on hipBLASLt and the row / block-column logsumexps, positive
extraction and the backward's softmax weights are one HIP kernel each (``csrc/milnce.hip``);
on CPU the reference formula (``ops/aten.py:milnce_loss``) runs. Semantics preserved: no
temperature, no normalisation, positives counted twice in the denominator.
"""
from __future__ import annotations

import torch

from .. import ops


class MILNCELoss(torch.nn.Module):
    def forward(self, video_embd: torch.Tensor, text_embd: torch.Tensor) -> torch.Tensor:
        return ops.milnce_loss(video_embd, text_embd)
