"""Collective timings of the data-parallel step, measured inside a real multi-rank run.

The bench's timed region reports the whole step; this probe, run after it on the same process
group, times the two collectives the step issues so the xGMI behaviour is on record next to the
step time of every N > 1 run (the driver's 2/4/8-GPU scaling runs included):

* the gradient all-reduce: one flat fp32 buffer the size of the model gradient, reduced whole
  (also on a bf16 wire, ``--grad_comm_dtype bf16``) and in the bucketer's bucket slices
  (``parallel/ddp.py``, launched during backward), and
* the embedding all-gather of the MIL-NCE negatives (``parallel/dist.py::all_gather_embeddings``).

Bus bandwidth follows the usual ring convention: all-reduce moves 2 (N-1)/N of the buffer per
rank, all-gather (N-1)/N of the output. xGMI on MI355X is point-to-point (7 links per GPU), so
RCCL's rings are per-link bound: the bucket-sized number shows what one backward bucket costs.
"""
from __future__ import annotations

import time
from typing import Dict, List, Sequence

import torch
import torch.distributed as dist


def _timed(fn, reps: int, cuda: bool) -> float:
    """Mean seconds per call (after one untimed call), max over ranks."""
    fn()
    if cuda:
        torch.cuda.synchronize()
    dist.barrier()
    if cuda:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        sec = a.elapsed_time(b) / 1000.0 / reps
    else:
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        sec = (time.perf_counter() - t0) / reps
    t = torch.tensor([sec], dtype=torch.float64, device="cuda" if cuda else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def probe(grad_numel: int, buckets: Sequence[Sequence[int]], emb_rows: int, emb_dim: int,
          emb_dtype: torch.dtype, device: torch.device, reps: int = 10) -> Dict[str, object]:
    """Times the step's collectives on scratch buffers of the step's sizes (every rank must call)."""
    world = dist.get_world_size()
    cuda = device.type == "cuda"
    flat = torch.ones(grad_numel, dtype=torch.float32, device=device)
    out: Dict[str, object] = {"world_size": world, "backend": dist.get_backend()}
    ar = _timed(lambda: dist.all_reduce(flat), reps, cuda)
    nbytes = grad_numel * 4
    out["grad_mib"] = round(nbytes / 2 ** 20, 2)
    out["allreduce_ms"] = round(ar * 1e3, 3)
    out["allreduce_busbw_gbps"] = round(nbytes * 2 * (world - 1) / world / ar / 1e9, 1)
    # the same gradient on a bf16 wire (--grad_comm_dtype bf16): half the bytes per hop
    flat16 = torch.ones(grad_numel, dtype=torch.bfloat16, device=device)
    ar16 = _timed(lambda: dist.all_reduce(flat16), reps, cuda)
    out["allreduce_bf16_ms"] = round(ar16 * 1e3, 3)
    del flat16
    sizes: List[int] = [int(e) - int(s) for s, e in buckets]
    views = [flat[int(s):int(e)] for s, e in buckets]

    def per_bucket():
        for v in views:
            dist.all_reduce(v)

    bt = _timed(per_bucket, max(2, reps // 2), cuda)
    out["buckets"] = len(sizes)
    out["bucket_mib_max"] = round(max(sizes) * 4 / 2 ** 20, 2) if sizes else 0.0
    out["bucketed_allreduce_ms"] = round(bt * 1e3, 3)
    emb = torch.ones((emb_rows, emb_dim), dtype=emb_dtype, device=device)
    gathered = emb.new_empty((world * emb_rows, emb_dim))
    if cuda and dist.get_backend() == "gloo":  # ranks sharing a GPU in tests: the host path of dist.py
        def gather():
            host = gathered.cpu()
            dist.all_gather_into_tensor(host, emb.cpu())
            gathered.copy_(host)
    else:
        def gather():
            dist.all_gather_into_tensor(gathered, emb)
    ag = _timed(gather, reps, cuda)
    gbytes = gathered.numel() * gathered.element_size()
    out["allgather_kib"] = round(gbytes / 1024, 1)
    out["allgather_ms"] = round(ag * 1e3, 3)
    out["allgather_busbw_gbps"] = round(gbytes * (world - 1) / world / ag / 1e9, 2)
    if cuda:  # the one-shot peer-write path (--emb_gather peer, parallel/peer.py) on the same sizes
        from .peer import PeerAllGather
        pg = PeerAllGather()
        want = gathered.clone()
        ok = True
        try:
            got = pg.gather(emb)
            if want is not None:
                ok = bool(torch.equal(got, want))
            pag = _timed(lambda: pg.gather(emb), reps, cuda)
            out["peer_allgather_ms"] = round(pag * 1e3, 3)
            out["peer_allgather_matches"] = ok
        except Exception as e:  # e.g. no IPC between these processes: recorded, not fatal
            out["peer_allgather_error"] = f"{type(e).__name__}: {e}"[:200]
    return out
