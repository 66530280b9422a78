"""Optimizers over flat buffers + the cosine-with-warmup schedule.

``FlatAdam`` is ``torch.optim.Adam`` semantics (betas 0.9/0.999, eps 1e-8, no weight decay,
``main_distributed.py:154-155``) with its state laid out as three flat fp32 buffers (params,
exp_avg, exp_avg_sq) that parameters and state entries view into. On GPU one HIP kernel
(``csrc/adam.hip``) updates all 11.3 M trainable parameters in a single launch and also folds
in the gradient all-reduce scale. ``state_dict()`` is byte-compatible with torch's Adam
(per-index ``step``/``exp_avg``/``exp_avg_sq``; 309 params in one group, the frozen word2vec
table without state), so reference checkpoints resume here and vice versa.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List

import torch
from torch.optim.lr_scheduler import LambdaLR

from .. import ops


def _adam_defaults(lr: float) -> dict:
    d = dict(lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, maximize=False,
             foreach=None, capturable=False, differentiable=False, fused=None)
    try:
        probe = torch.optim.Adam([torch.zeros(1, requires_grad=True)], lr=lr)
        d = dict(probe.defaults)
    except Exception:
        pass
    return d


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float = 1e-3, grad_scale: float = 1.0):
        params = list(params)
        super().__init__(params, _adam_defaults(lr))
        self.grad_scale = float(grad_scale)
        self.trainable: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        dev = self.trainable[0].device
        total = sum(p.numel() for p in self.trainable)
        self.flat_param = torch.empty(total, dtype=torch.float32, device=dev)
        self.flat_m = torch.zeros(total, dtype=torch.float32, device=dev)
        self.flat_v = torch.zeros(total, dtype=torch.float32, device=dev)
        self.offsets: Dict[int, int] = {}
        off = 0
        # Same layout as parallel.ddp.GradBucketer (reverse registration order ~ backward
        # order) so the all-reduced flat gradient is consumed in place.
        for p in reversed(self.trainable):
            n = p.numel()
            self.flat_param[off:off + n].copy_(p.data.reshape(-1))
            p.data = self.flat_param[off:off + n].view_as(p)
            self.offsets[id(p)] = off
            off += n
        self.step_count = 0
        self._grad_flat = None  # set by bind_flat_grad when grads live in one buffer

    def bind_flat_grad(self, flat_grad: torch.Tensor, offsets: Dict[int, int]) -> None:
        """Use a flat gradient buffer whose layout matches (checked) the param layout."""
        same = all(offsets[id(p)] == self.offsets[id(p)] for p in self.trainable)
        self._grad_flat = flat_grad if same else None

    def _ensure_state(self):
        for p in self.trainable:
            st = self.state[p]
            if "exp_avg" not in st:
                off, n = self.offsets[id(p)], p.numel()
                st["step"] = torch.tensor(float(self.step_count))
                st["exp_avg"] = self.flat_m[off:off + n].view_as(p)
                st["exp_avg_sq"] = self.flat_v[off:off + n].view_as(p)

    def _gather_grad(self) -> torch.Tensor:
        if self._grad_flat is not None:
            return self._grad_flat
        g = torch.zeros_like(self.flat_param)
        for p in self.trainable:
            if p.grad is not None:
                off = self.offsets[id(p)]
                g[off:off + p.numel()].copy_(p.grad.reshape(-1))
        return g

    @torch.no_grad()
    def step(self, closure=None):
        group = self.param_groups[0]
        lr, (b1, b2), eps = group["lr"], group["betas"], group["eps"]
        wd = group.get("weight_decay", 0)
        self.step_count += 1
        self._ensure_state()
        t = self.step_count
        bc1 = 1.0 - b1 ** t
        bc2 = 1.0 - b2 ** t
        g = self._gather_grad()
        if self.flat_param.is_cuda and ops.use_hip(self.flat_param):
            from ..ops import hip_ops
            hip_ops.adam_step(self.flat_param, g, self.flat_m, self.flat_v, lr, b1, b2, eps, wd,
                              bc1, bc2, self.grad_scale)
        else:
            gs = g * self.grad_scale if self.grad_scale != 1.0 else g
            if wd:
                gs = gs + wd * self.flat_param
            self.flat_m.mul_(b1).add_(gs, alpha=1 - b1)
            self.flat_v.mul_(b2).addcmul_(gs, gs, value=1 - b2)
            denom = (self.flat_v.sqrt() / math.sqrt(bc2)).add_(eps)
            self.flat_param.addcdiv_(self.flat_m, denom, value=-lr / bc1)
        for p in self.trainable:
            self.state[p]["step"].fill_(float(t))
        return None

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = []
        for p in self.trainable:
            st = self.state.get(p, {})
            if "exp_avg" in st:
                off, n = self.offsets[id(p)], p.numel()
                self.flat_m[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self.flat_v[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                st["exp_avg"] = self.flat_m[off:off + n].view_as(p)
                st["exp_avg_sq"] = self.flat_v[off:off + n].view_as(p)
                s = st["step"]
                st["step"] = torch.tensor(float(s.item() if torch.is_tensor(s) else s))
                steps.append(int(st["step"].item()))
        if steps:
            self.step_count = max(steps)


class FlatSGD(torch.optim.SGD):
    """SGD with momentum (``main_distributed.py:156-157``, flag ``--momemtum``), with the
    all-reduce scale folded into the update like FlatAdam."""

    def __init__(self, params, lr, momentum, grad_scale: float = 1.0):
        super().__init__(params, lr=lr, momentum=momentum)
        self.grad_scale = float(grad_scale)

    def bind_flat_grad(self, flat_grad, offsets):
        pass

    @torch.no_grad()
    def step(self, closure=None):
        if self.grad_scale != 1.0:
            for g in self.param_groups:
                for p in g["params"]:
                    if p.grad is not None:
                        p.grad.mul_(self.grad_scale)
        return super().step(closure)


def cosine_schedule_with_warmup(optimizer, num_warmup_steps: int, num_training_steps: int,
                                num_cycles: float = 0.5, last_epoch: int = -1) -> LambdaLR:
    """Linear warmup then cosine decay (utils.py:26-38); stepped every batch."""

    def lr_lambda(current_step: int) -> float:
        if current_step < num_warmup_steps:
            return float(current_step) / float(max(1, num_warmup_steps))
        progress = float(current_step - num_warmup_steps) / float(max(1, num_training_steps - num_warmup_steps))
        return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))

    return LambdaLR(optimizer, lr_lambda, last_epoch)
