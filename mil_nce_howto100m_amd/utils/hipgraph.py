"""HIP-graph replay of launch-bound forward passes (evaluation / inference).

A small-batch S3D-G forward is a few hundred short kernel launches, so the host, not the GPU,
sets its speed. ``GraphedCallable`` captures ``fn(*tensors)`` once per input signature into a
HIP graph (``torch.cuda.CUDAGraph``, which is hipGraph on ROCm) and replays it: inputs are
copied into the captured static buffers, the graph runs, the static outputs are returned
(cloned, so later replays cannot overwrite what the caller holds). Eager warm-up calls run
before capture, so per-shape conv autotuning and first-launch kernel attributes never happen
inside a capture. Training steps are not captured: they are GPU-bound at the flagship batch.
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import torch


class GraphedCallable:
    def __init__(self, fn: Callable, warmup: int = 2, max_graphs: int = 4):
        self.fn = fn
        self.warmup = warmup
        self.max_graphs = max_graphs
        self._graphs: Dict[Tuple, Tuple] = {}

    @staticmethod
    def _key(tensors) -> Tuple:
        return tuple((tuple(t.shape), t.dtype, t.device) for t in tensors)

    def _capture(self, tensors):
        static_in = [t.clone() for t in tensors]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.fn(*static_in)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_out = self.fn(*static_in)
        return graph, static_in, static_out

    def __call__(self, *tensors):
        if not all(t.is_cuda for t in tensors):
            return self.fn(*tensors)
        key = self._key(tensors)
        entry = self._graphs.get(key)
        if entry is None:
            if len(self._graphs) >= self.max_graphs:
                return self.fn(*tensors)
            entry = self._capture(tensors)
            self._graphs[key] = entry
        graph, static_in, static_out = entry
        for dst, src in zip(static_in, tensors):
            dst.copy_(src)
        graph.replay()
        if isinstance(static_out, (tuple, list)):
            return type(static_out)(o.clone() for o in static_out)
        return static_out.clone()
