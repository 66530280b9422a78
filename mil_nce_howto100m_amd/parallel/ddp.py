"""Data-parallel gradient synchronisation: flat gradient buffer + bucketed all-reduce.

Replaces ``DistributedDataParallel`` (``main_distributed.py:91``) with an explicit, MI355X-
sized design:

* every trainable parameter's ``.grad`` is a view into ONE flat fp32 buffer laid out in
  (approximate) backward order, so a bucket is a contiguous slice and one RCCL call;
* ``register_post_accumulate_grad_hook`` (or, for gradients a HIP kernel accumulated in place,
  the ``ops.grad_sink`` notification) marks parameters ready; when a bucket's last
  gradient lands its all-reduce is issued asynchronously (RCCL runs on its own HIP stream,
  ordered after the compute stream by an event), overlapping with the rest of backward;
* bucket sizes: ``bucket_bytes`` per bucket in backward order, and optionally a smaller last
  bucket of at most ``tail_bytes`` (the first layers, whose gradients land last, so their
  all-reduce is the exposed one). The trainer's default (``--bucket_mb auto``) takes both from
  ``parallel/bucket_plan.py``: the all-reduce cost measured on the run's process group at
  start-up (or the xGMI link model), buckets at 4x the latency knee, the tail at the knee;
* ``comm_dtype=torch.bfloat16`` (``--grad_comm_dtype bf16``) puts each bucket on the wire as
  bf16 (half the xGMI bytes; the ring then sums in bf16, ~3 significant digits per hop) and
  writes the reduced values back into the fp32 buffer; the default keeps fp32 on the wire;
* the reduction is a SUM; the 1/world_size factor (reference semantics: DDP mean, with
  ``AllGather.backward`` returning only the local slice, ``utils.py:19-24``) or 1 (exact
  full-batch gradient) is folded into the optimizer kernel as ``grad_scale``;
* BN running statistics are broadcast from rank 0 before every forward, like DDP's default
  ``broadcast_buffers=True`` (``main_distributed.py:91``), coalesced into few calls.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


class BucketOrderError(RuntimeError):
    """A gradient slice changed after its bucket's all-reduce was issued (verify mode)."""


class GradBucketer:
    """See the module docstring. ``verify`` (or ``MILNCE_VERIFY_BUCKETS=1``) turns on the
    comm/compute ordering verifier: each bucket is all-reduced from a private copy taken on the
    compute stream at launch, and ``finish`` checks that the local gradient slice still equals
    that copy after backward (any later write, e.g. a kernel that accumulated into a parameter
    after reporting it ready, would silently be lost in normal mode) before installing the
    reduced copy. Costs two extra gradient copies; for debugging only."""

    def __init__(self, params: Sequence[torch.nn.Parameter], world_size: int,
                 bucket_bytes: int = 8 << 20, process_group=None, verify: Optional[bool] = None,
                 comm_dtype: torch.dtype = torch.float32, tail_bytes: Optional[int] = None):
        self.verify = (os.environ.get("MILNCE_VERIFY_BUCKETS", "0") == "1") if verify is None else bool(verify)
        self._snap: Dict[int, torch.Tensor] = {}
        self._comm: Dict[int, torch.Tensor] = {}
        if comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"gradient comm dtype must be fp32 or bf16, got {comm_dtype}")
        self.comm_dtype = comm_dtype
        self.params = [p for p in params if p.requires_grad]
        self.world_size = world_size
        self.group = process_group
        dev = self.params[0].device
        # Backward order is roughly reverse registration order.
        order = list(reversed(self.params))
        total = sum(p.numel() for p in order)
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.offsets: Dict[int, int] = {}
        self.buckets: List[List[int]] = []  # list of [start, end)
        self.bucket_of: Dict[int, int] = {}
        self.bucket_size: List[int] = []
        # the last bucket: the trailing parameters of the backward order (at least one) that fit
        # in tail_bytes; None: no separate tail
        tail_start = len(order)
        if tail_bytes is not None and len(order) > 1:
            acc = 0
            while tail_start > 1 and acc + order[tail_start - 1].numel() * 4 <= tail_bytes:
                tail_start -= 1
                acc += order[tail_start].numel() * 4
            tail_start = min(tail_start, len(order) - 1)
        off = 0
        cur_start, cur_count = 0, 0
        for i, p in enumerate(order):
            n = p.numel()
            if off > cur_start and ((off - cur_start + n) * 4 > bucket_bytes or i == tail_start):
                self.buckets.append([cur_start, off])
                self.bucket_size.append(cur_count)
                cur_start, cur_count = off, 0
            self.offsets[id(p)] = off
            self.bucket_of[id(p)] = len(self.buckets)
            cur_count += 1
            p.grad = self.flat[off:off + n].view_as(p)
            p._milnce_flat_grad = True  # HIP kernels may accumulate into p.grad in place
            off += n
        self.buckets.append([cur_start, off])
        self.bucket_size.append(cur_count)
        self._pending: List[int] = list(self.bucket_size)
        self._ready: set = set()
        self._handles: List[Optional[object]] = [None] * len(self.buckets)
        self.sync_enabled = True  # False: accumulate only (micro-batches before the last)
        self._issue = None  # stream the bucket all-reduces are issued from (GPU)
        self._hooks = []
        if world_size > 1:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        # kernels that write a gradient in place (no AccumulateGrad) report through this sink
        from ..ops import grad_sink
        grad_sink.set_sink(self._on_grad if world_size > 1 else None)

    # ---------------------------------------------------------------------------------
    def views_intact(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == self.flat.data_ptr() + 4 * self.offsets[id(p)]
                   for p in self.params)

    def zero(self) -> None:
        self.flat.zero_()
        self._pending = list(self.bucket_size)
        self._ready = set()
        self._handles = [None] * len(self.buckets)

    def _launch(self, b: int) -> None:
        if self.flat.is_cuda:
            # issued from a stream that waits for the compute stream's work so far AND for the
            # side stream's deferred gradient writes (grad_sink.join), so the compute stream is not
            # made to wait for the side stream at every bucket
            from ..ops import grad_sink
            main = torch.cuda.current_stream(self.flat.device)
            if self._issue is None:
                self._issue = torch.cuda.Stream(device=self.flat.device)
            self._issue.wait_stream(main)
            grad_sink.join(self._issue)
            with torch.cuda.stream(self._issue):
                self._launch_on_current(b)
        else:
            self._launch_on_current(b)

    def _launch_on_current(self, b: int) -> None:
        s, e = self.buckets[b]
        buf = self.flat[s:e]
        if self.verify:  # reduce a private copy; keep another to check the slice against later
            self._snap[b] = buf.clone()
        if self.comm_dtype != torch.float32:  # narrow wire copy, written back in finish()
            buf = self._comm[b] = buf.to(self.comm_dtype)
        elif self.verify:
            buf = self._comm[b] = buf.clone()
        self._handles[b] = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _on_grad(self, p: torch.Tensor) -> None:
        """A parameter's gradient for this step is complete (enqueued on the compute stream).

        Idempotent per step: a parameter whose gradient a HIP kernel wrote in place reports
        through ``ops.grad_sink`` when that kernel is enqueued, and autograd then still runs
        its post-accumulate hook (with nothing to accumulate); counting both would issue the
        bucket's all-reduce while half of its gradients are still missing."""
        if not self.sync_enabled or id(p) in self._ready:
            return
        self._ready.add(id(p))
        b = self.bucket_of[id(p)]
        self._pending[b] -= 1
        if self._pending[b] == 0 and self._handles[b] is None:
            self._launch(b)  # after the side stream's pending gradient writes (see _launch)

    def set_sync(self, enabled: bool) -> None:
        """Gradient accumulation: with sync off, backward passes only accumulate into the flat
        buffer; the pass run with sync on issues every bucket as its last gradient lands."""
        self.sync_enabled = bool(enabled)
        self._pending = list(self.bucket_size)
        self._ready = set()

    def finish(self) -> None:
        """Issue buckets whose params got no gradient this step, then wait for all. Also the
        point where deferred (side-stream) gradient writes are joined into the compute stream,
        so it must run before anything reads the gradients (the trainer calls it before the
        optimizer step, at every world size)."""
        from ..ops import grad_sink
        grad_sink.drain()
        if self.world_size <= 1:
            return
        for b in range(len(self.buckets)):
            if self._handles[b] is None:
                self._launch(b)
        for h in self._handles:
            h.wait()
        if self.flat.is_cuda:  # wire / verify copies made on the issue stream, read here on this one
            cur = torch.cuda.current_stream(self.flat.device)
            for t in list(self._comm.values()) + list(self._snap.values()):
                t.record_stream(cur)
        if self.comm_dtype != torch.float32 and not self.verify:
            for b, (s, e) in enumerate(self.buckets):
                self.flat[s:e].copy_(self._comm[b])
            self._comm.clear()
        if self.verify:
            bad = []
            for b, (s, e) in enumerate(self.buckets):
                d = (self.flat[s:e] - self._snap[b]).abs().max().item() if e > s else 0.0
                if d != 0.0:
                    bad.append((b, d))
                self.flat[s:e].copy_(self._comm[b])
            self._snap.clear()
            self._comm.clear()
            if bad:
                raise BucketOrderError("gradient written after its bucket's all-reduce was issued "
                                       f"(bucket, max |change|): {bad}")


class BufferBroadcaster:
    """Broadcast module buffers (BN running stats, counters) from rank 0 each step.

    At N > 1 the buffers are re-pointed once into one flat tensor per dtype (views, like the
    optimizer's flat parameters; the BN kernels update them in place and checkpoint loads copy
    into them), so each step's broadcast is one collective per dtype with no pack / unpack: a
    coalesced broadcast of the ~300 separate S3D-G buffers re-copies every one of them (one small
    copy launch each) on every step.

    Anything that later replaces a buffer tensor (``model.to()``, ``load_state_dict(assign=True)``,
    a module assigning a new running stat) would detach it from its flat; every call first checks
    that each buffer still is its view (one pointer compare per buffer) and re-flattens otherwise,
    so the broadcast never syncs orphaned copies."""

    def __init__(self, module: torch.nn.Module, world_size: int, bucket_bytes: int = 32 << 20):
        self.world_size = world_size
        self.bucket_bytes = bucket_bytes
        self.module = module
        self.bufs = [b for b in module.buffers()]
        self.flats: List[torch.Tensor] = []
        self.slots: List[tuple] = []  # (owner module, buffer name, expected data_ptr)
        self.reflattens = 0
        if world_size > 1 and self.bufs:
            self._flatten(module)

    def _flatten(self, module: torch.nn.Module) -> None:
        owners = [(m, name, b) for m in module.modules() for name, b in m._buffers.items() if b is not None]
        by_dtype: Dict[torch.dtype, list] = {}
        for m, name, b in owners:
            by_dtype.setdefault((b.dtype, b.device), []).append((m, name, b))
        self.flats, self.slots = [], []
        for (dtype, device), items in by_dtype.items():
            total = sum(b.numel() for _, _, b in items)
            flat = torch.empty(total, dtype=dtype, device=device)
            off = 0
            for m, name, b in items:
                n = b.numel()
                view = flat[off:off + n].view_as(b)
                view.copy_(b)
                m._buffers[name] = view
                self.slots.append((m, name, view.data_ptr()))
                off += n
            self.flats.append(flat)
        self.bufs = [b for b in module.buffers()]

    def views_intact(self) -> bool:
        return all(m._buffers.get(name) is not None and m._buffers[name].data_ptr() == p for m, name, p in self.slots)

    def __call__(self) -> None:
        if self.world_size <= 1 or not self.bufs:
            return
        if self.flats and not self.views_intact():
            self._flatten(self.module)  # a buffer was replaced: its current values move into new flats
            self.reflattens += 1
        if self.flats:
            for f in self.flats:
                dist.broadcast(f, 0)
        else:
            dist._broadcast_coalesced(dist.group.WORLD, self.bufs, self.bucket_bytes, 0)


def broadcast_parameters(module: torch.nn.Module, world_size: int) -> None:
    """Rank-0 broadcast of every parameter and buffer (the DDP constructor's sync, N2)."""
    if world_size <= 1:
        return
    tensors = [p.data for p in module.parameters()] + [b for b in module.buffers()]
    dist._broadcast_coalesced(dist.group.WORLD, tensors, 64 << 20, 0)
