"""Process-group bootstrap and the cross-GPU embedding gather.

Replaces the reference's launcher logic (``main_distributed.py:35-75``: UDP probe of 8.8.8.8
for the local IP, ``mp.spawn``, ``init_process_group(tcp://ip:23456)``) and the multi-node
static IP list (``train.py:48-63``) with torchrun-style env rendezvous: one process per GPU,
``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT`` from the environment, backend ``nccl``
(= RCCL over xGMI on ROCm) or ``gloo`` for CPU plumbing.

``all_gather_embeddings`` keeps the reference ``AllGather`` semantics (``utils.py:8-24``):
forward concatenates every rank's rows in rank order; backward returns only the local slice
of the incoming gradient, with no reduction. Video and text embeddings travel in ONE
collective (they are packed into one buffer), halving the latency-bound launches of N4/N5.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_CTX = DistContext()


def context() -> DistContext:
    return _CTX


def init_distributed(backend: str = "nccl", device: str = "auto", timeout_s: int = 1800,
                     init_method: str = "env://") -> DistContext:
    """Initialise from torchrun/env variables. Works with WORLD_SIZE unset (single process)."""
    global _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device == "auto":
        use_cuda = torch.cuda.device_count() > 0
    else:
        use_cuda = device == "cuda"
    if use_cuda:
        # MILNCE_DEVICE_INDEX pins every rank to one device (multi-rank tests on a 1-GPU box,
        # with gloo: RCCL refuses two ranks on one GPU); otherwise rank i owns device i
        idx = int(os.environ.get("MILNCE_DEVICE_INDEX", str(local_rank)))
        if "MILNCE_DEVICE_INDEX" not in os.environ:
            from .launch import check_local_rank
            check_local_rank(local_rank)
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
    else:
        dev = torch.device("cpu")
        if backend == "nccl":
            backend = "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kwargs = dict(backend=backend, init_method=init_method, world_size=world, rank=rank,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = dev
        dist.init_process_group(**kwargs)
    _CTX = DistContext(rank=rank, world_size=world, local_rank=local_rank,
                       backend=backend if world > 1 else "none", device=dev)
    return _CTX


def observed_world_size() -> int:
    """World size as torch.distributed sees it (1 without a process group)."""
    return dist.get_world_size() if dist.is_initialized() else 1


def set_context(ctx: DistContext) -> None:
    global _CTX
    _CTX = ctx


def barrier() -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        if _CTX.device.type == "cuda":
            dist.barrier(device_ids=[_CTX.device.index])
        else:
            dist.barrier()


def destroy() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


_EMB_GATHER = "rccl"


def set_emb_gather(mode: str) -> None:
    """Embedding all-gather path: "rccl" (ring all-gather) or "peer" (one-shot xGMI peer writes,
    parallel/peer.py; same-node process groups only)."""
    global _EMB_GATHER
    if mode not in ("rccl", "peer"):
        raise ValueError(f"unknown embedding gather {mode!r}")
    _EMB_GATHER = mode


class _GatherLocalGrad(torch.autograd.Function):
    """all_gather forward, local-slice backward (utils.py:8-24)."""

    @staticmethod
    def forward(ctx, packed: torch.Tensor, world: int, rank: int):
        ctx.rows = packed.shape[0]
        ctx.rank = rank
        if packed.is_cuda and _EMB_GATHER == "peer":
            from .peer import peer_all_gather
            return peer_all_gather(packed)
        out = packed.new_empty((world * packed.shape[0],) + tuple(packed.shape[1:]))
        if packed.is_cuda and dist.get_backend() == "gloo":
            # gloo over device tensors (multi-rank tests sharing one GPU): gather on the host
            host = out.cpu()
            dist.all_gather_into_tensor(host, packed.contiguous().cpu())
            out.copy_(host)
        else:
            dist.all_gather_into_tensor(out, packed.contiguous())
        ctx.rows = packed.shape[0]
        ctx.rank = rank
        return out

    @staticmethod
    def backward(ctx, grad):
        r = ctx.rows
        return grad[r * ctx.rank: r * (ctx.rank + 1)], None, None


def all_gather_embeddings(video_embd: torch.Tensor, text_embd: torch.Tensor,
                          ctx: Optional[DistContext] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Gather [b, D] video and [b*K, D] text embeddings from every rank in one collective.

    Returns [W*b, D] and [W*b*K, D] in rank-major order, i.e. text rows i*K..i*K+K-1 still
    belong to video row i (loss.py:12).
    """
    ctx = ctx or _CTX
    if ctx.world_size <= 1:
        return video_embd, text_embd
    b = video_embd.shape[0]
    packed = torch.cat([video_embd, text_embd], dim=0)
    out = _GatherLocalGrad.apply(packed, ctx.world_size, ctx.rank)
    rows = packed.shape[0]
    out = out.view(ctx.world_size, rows, -1)
    v = out[:, :b].reshape(ctx.world_size * b, -1)
    t = out[:, b:].reshape(ctx.world_size * (rows - b), -1)
    return v, t


def broadcast_object(obj, src: int = 0):
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def all_reduce_max(value: float) -> float:
    """Max of a host scalar over ranks (used for the bench's timed region)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_CTX.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
