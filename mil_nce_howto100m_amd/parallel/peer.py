"""One-shot peer-write all-gather over xGMI (the MIL-NCE negatives, reference ``utils.py:8-24``).

RCCL's all-gather is a ring: on MI355X's point-to-point xGMI (7 links per GPU, one to each peer
of the node) every byte crosses N-1 hops in sequence, and each hop is one link's bandwidth. The
embedding gather is small (b x D rows per rank) and latency-bound, so this path writes each
rank's slice straight into every peer's receive buffer at once: N-1 direct copies, one per link,
all in flight together, then one completion fence.

* Receive buffers are allocated once per (shape, dtype), two of them (alternating calls), and
  exported to the peers as IPC handles (``torch.multiprocessing.reductions.reduce_tensor``; the
  handles travel through the process group as plain objects). Each rank maps its peers' buffers
  (hipIpcOpenMemHandle under the hood; same-node only).
* ``gather(x)``: rank r copies x into slot r of every peer's buffer and of its own (stream
  ordered on the current stream), then fences: a one-element RCCL all-reduce, which every rank
  enqueues after its copies, so when it completes every slice of every buffer has landed
  (gloo process groups, i.e. ranks sharing one GPU in tests: device sync + host barrier).
  The result is cloned out of the receive buffer, so the caller may keep it.
* Reuse safety: call c writes buffer c % 2. A peer's writes of call c + 2 happen after it passed
  the fence of call c + 1, which this rank enqueued after its clone of call c: no write lands in
  a buffer whose previous contents are still to be read.

``all_gather_embeddings`` (parallel/dist.py) takes this path with ``--emb_gather peer``; the comm
probe (parallel/comm_probe.py) times both. CPU tensors, and groups whose ranks are not all on
one node (checked once per group: every rank's host name and boot id, gathered through the
group), take ``dist.all_gather_into_tensor`` instead: IPC handles cannot be opened across nodes.
"""
from __future__ import annotations

import socket
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist


def _fence(device: torch.device, group=None) -> None:
    if dist.get_backend(group) == "nccl":
        t = torch.zeros(1, dtype=torch.float32, device=device)
        dist.all_reduce(t, group=group)  # ordered after this rank's copies on the current stream
    else:
        torch.cuda.current_stream(device).synchronize()
        dist.barrier(group=group)


def _node_id() -> str:
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return f"{socket.gethostname()}|{boot}"


def same_node(group=None) -> bool:
    """True when every rank of ``group`` runs on this node (collective: call on every rank)."""
    world = dist.get_world_size(group)
    ids: List[Optional[str]] = [None] * world
    dist.all_gather_object(ids, _node_id(), group=group)
    return len(set(ids)) == 1


class PeerAllGather:
    """Same-node all-gather into ``[world * rows, ...]`` by direct peer writes (see module doc)."""

    def __init__(self, group=None):
        self.group = group
        self._bufs: Dict[Tuple, List[List[torch.Tensor]]] = {}  # key -> [parity][rank] buffer views
        self._calls = 0
        self._local: Optional[bool] = None  # all ranks on one node (decided on the first gather)

    def _exchange(self, key, shape, dtype, device) -> List[List[torch.Tensor]]:
        from torch.multiprocessing.reductions import reduce_tensor
        world, rank = dist.get_world_size(self.group), dist.get_rank(self.group)
        mine = [torch.empty((world,) + shape, dtype=dtype, device=device) for _ in range(2)]
        handles = [reduce_tensor(b) for b in mine]
        every: List[Optional[list]] = [None] * world
        dist.all_gather_object(every, handles, group=self.group)
        views = [[None] * world for _ in range(2)]
        for r in range(world):
            for p in range(2):
                if r == rank:
                    views[p][r] = mine[p]
                else:
                    fn, args = every[r][p]
                    views[p][r] = fn(*args)  # the peer's buffer, mapped into this process
        self._bufs[key] = views
        self._keep = getattr(self, "_keep", []) + mine
        return views

    def gather(self, x: torch.Tensor) -> torch.Tensor:
        world, rank = dist.get_world_size(self.group), dist.get_rank(self.group)
        if world == 1:
            return x.clone()
        if self._local is None and x.is_cuda:
            self._local = same_node(self.group)
        if not x.is_cuda or not self._local:
            out = x.new_empty((world * x.shape[0],) + tuple(x.shape[1:]))
            dist.all_gather_into_tensor(out, x.contiguous(), group=self.group)
            return out
        x = x.contiguous()
        key = (tuple(x.shape), x.dtype, x.device.index)
        views = self._bufs.get(key) or self._exchange(key, tuple(x.shape), x.dtype, x.device)
        p = self._calls % 2
        self._calls += 1
        order = [(rank + 1 + k) % world for k in range(world)]  # the next peer first: links not hit in rank order
        nbytes = x.numel() * x.element_size()
        if _native() and nbytes % 16 == 0 and world <= 8:
            import ctypes
            from ..ops._lib import call, stream
            dsts = (ctypes.c_void_p * world)(*[views[p][r][rank].data_ptr() for r in order])
            call("milnce_peer_scatter", x.data_ptr(), ctypes.addressof(dsts), world, nbytes, stream())
        else:
            for r in order:
                views[p][r][rank].copy_(x, non_blocking=True)
        _fence(x.device, self.group)
        return views[p][rank].reshape((world * x.shape[0],) + tuple(x.shape[1:])).clone()


def _native() -> bool:
    try:
        from ..ops import _lib
        _lib.lib()
        return True
    except Exception:  # no HIP library (CPU container): torch copies
        return False


_PEER: Optional[PeerAllGather] = None


def peer_all_gather(x: torch.Tensor) -> torch.Tensor:
    global _PEER
    if _PEER is None:
        _PEER = PeerAllGather()
    return _PEER.gather(x)
