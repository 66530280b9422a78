"""Link-aware gradient bucket plan for the data-parallel all-reduce (``--bucket_mb auto``).

The reference wraps the model in ``DistributedDataParallel`` with its default 25 MiB buckets
(``main_distributed.py:91``). Here the bucket sizes come from the cost of one all-reduce on the
node's links, so they follow the xGMI topology instead of a fixed constant.

Cost model. RCCL reduces a bucket of S bytes on W ranks with ring steps over the point-to-point
xGMI links (7 per MI355X, ~153 GB/s each), so one bucket costs ``t(S) = a + b * S``: ``a`` is
the 2 (W - 1) ring-step latencies, ``b`` the wire time per byte, 2 (W - 1) / W of the bucket
over the ring's bus bandwidth. The knee ``S_k = a / b`` is the size at which a bucket spends
half its time on latency.

Plan (``plan_buckets``):

* the buckets issued during backward are ``4 * S_k`` (latency <= 20 % of each all-reduce),
  clamped to [4, 64] MiB and to half the gradient, so that at least two buckets exist and the
  first ones overlap the rest of backward;
* the LAST bucket is kept small: it holds the first layers' gradients (the stem), which the
  backward produces last, so its all-reduce runs after the final backward kernel and is exposed
  in the step time. It is ``S_k`` (cost 2a), at least 1 MiB.

``a`` and ``b`` are measured once at start-up (``calibrate``: the all-reduce timed at two sizes
on the run's process group, max over ranks, so every rank derives the same plan; rank 0's plan
is broadcast regardless). Without a process group the analytic xGMI model (``xgmi_model``)
stands in.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Dict, Optional

import torch
import torch.distributed as dist

MIB = 1 << 20
XGMI_LINKS = 7            # xGMI links per MI355X (fully connected 8-GPU node)
XGMI_LINK_GBPS = 153.0    # per link
RING_EFFICIENCY = 0.33    # RCCL ring bus bandwidth / (links in use x link bandwidth), rough
HOP_LATENCY_US = 4.0      # one ring step (launch + hand-off), rough


@dataclass
class LinkModel:
    a_s: float            # seconds per all-reduce independent of size
    b_s_per_byte: float   # seconds per byte of bucket
    source: str           # "measured" or "xgmi-model"

    @property
    def knee_bytes(self) -> float:
        return self.a_s / self.b_s_per_byte if self.b_s_per_byte > 0 else float(64 * MIB)

    def cost_s(self, nbytes: int) -> float:
        return self.a_s + self.b_s_per_byte * nbytes


@dataclass
class BucketPlan:
    bucket_bytes: int
    tail_bytes: int
    world_size: int
    a_us: float
    busbw_gbps: float
    source: str

    def as_dict(self) -> Dict[str, object]:
        d = asdict(self)
        d["bucket_mib"] = round(self.bucket_bytes / MIB, 2)
        d["tail_mib"] = round(self.tail_bytes / MIB, 2)
        return d


def xgmi_model(world: int) -> LinkModel:
    """Analytic ring all-reduce cost on one MI355X node (rough constants above)."""
    w = max(2, int(world))
    bus = RING_EFFICIENCY * min(w - 1, XGMI_LINKS) * XGMI_LINK_GBPS * 1e9  # bytes/s
    a = 2 * (w - 1) * HOP_LATENCY_US * 1e-6
    b = 2.0 * (w - 1) / w / bus
    return LinkModel(a, b, "xgmi-model")


def calibrate(device: torch.device, sizes=(256 << 10, 8 << 20), reps: int = 5, group=None) -> LinkModel:
    """Fit ``t(S) = a + b S`` to the all-reduce of two buffer sizes on the process group. Every
    rank must call it; the times are maxima over ranks, so the fit is the same everywhere."""
    from .comm_probe import _timed
    cuda = device.type == "cuda"
    times = []
    for s in sizes:
        buf = torch.ones(max(1, s // 4), dtype=torch.float32, device=device)
        times.append(_timed(lambda: dist.all_reduce(buf, group=group), reps, cuda))
        del buf
    (s0, s1), (t0, t1) = sizes, times
    b = max((t1 - t0) / (s1 - s0), 1e-15)
    a = max(t0 - b * s0, 0.0)
    return LinkModel(a, b, "measured")


def plan_buckets(grad_bytes: int, world: int, model: Optional[LinkModel] = None,
                 min_bytes: int = 4 * MIB, max_bytes: int = 64 * MIB, min_tail: int = 1 * MIB) -> BucketPlan:
    """Bucket and tail sizes for a ``grad_bytes`` gradient on ``world`` ranks (module docstring)."""
    m = model if model is not None else xgmi_model(world)
    knee = m.knee_bytes
    bucket = int(min(max(4.0 * knee, min_bytes), max_bytes))
    bucket = max(min(bucket, grad_bytes // 2), min_tail)
    tail = int(max(min(knee, bucket), min_tail))
    w = max(2, int(world))
    busbw = 2.0 * (w - 1) / w / m.b_s_per_byte / 1e9 if m.b_s_per_byte > 0 else 0.0
    return BucketPlan(bucket_bytes=int(bucket), tail_bytes=int(tail), world_size=int(world),
                      a_us=round(m.a_s * 1e6, 2), busbw_gbps=round(busbw, 1), source=m.source)


def auto_plan(grad_bytes: int, world: int, device: torch.device, measure: bool = True) -> BucketPlan:
    """The run's plan: measured on the initialised process group when there is one (and
    ``measure``), else the analytic model; rank 0's plan is broadcast so all ranks bucket alike."""
    if world <= 1 or not (dist.is_available() and dist.is_initialized()):
        return plan_buckets(grad_bytes, world)
    model = calibrate(device) if measure else None
    plan = plan_buckets(grad_bytes, world, model)
    sizes = torch.tensor([plan.bucket_bytes, plan.tail_bytes], dtype=torch.int64,
                         device=device if device.type == "cuda" and dist.get_backend() == "nccl" else "cpu")
    dist.broadcast(sizes, 0)
    plan.bucket_bytes, plan.tail_bytes = int(sizes[0].item()), int(sizes[1].item())
    return plan
