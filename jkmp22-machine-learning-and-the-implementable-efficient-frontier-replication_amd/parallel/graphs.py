"""Segmented HIP-graph capture of a multi-rank step (one process per GPU).

A whole grid-search step captures as ONE HIP graph on a single rank (bench.graphed).  With
several ranks the step has collectives in it (the chunk-total all-gather of the window sums,
the utilities all-gather), which stay eager here: while the step function is captured, each
collective (parallel.collectives.all_gather_known) ends the current graph segment, runs
eagerly into a static output tensor and opens the next segment.  A replay is then

    segment 0 graph | collective 0 | segment 1 graph | collective 1 | segment 2 graph

- every kernel between collectives replays from its graph (no host launch work), the
collectives run with the same static buffers the segments were captured against.  The
inputs of a collective are tensors of the preceding segment's graph pool (kept alive by the
recorded op), its outputs live outside the pool, so no later segment can overwrite them.
"""
from __future__ import annotations

import torch

from . import collectives as coll


class SegmentedGraph:
    def __init__(self, device: torch.device):
        self.device = device
        self.stream = torch.cuda.Stream(device=device)
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs: list = []
        self.ops: list = []
        self._cur = None

    def _begin(self) -> None:
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self.pool)
        self._cur = g

    def _end(self) -> None:
        import warnings
        with warnings.catch_warnings():
            # back-to-back collectives leave an empty segment in between (harmless)
            warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
            self._cur.capture_end()
        self.graphs.append(self._cur)
        self._cur = None

    def collective(self, fn, x: torch.Tensor, counts):
        """Called by the collective under capture: close the segment, run the collective
        eagerly into a static tensor, record it, open the next segment."""
        self._end()
        res = fn(None, x, counts)                       # eager, allocates the result shape
        out = torch.empty_like(res)
        out.copy_(res)
        self.ops.append(lambda: fn(out, x, counts))
        self._begin()
        return out

    def capture(self, fn):
        """Warm up ``fn`` once eagerly, then capture it segment-wise; returns the replay."""
        s = self.stream
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            fn()                                      # plans, caches, allocator state
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        with torch.cuda.stream(s):
            self._begin()
            coll.set_capture(self)
            try:
                fn()
            finally:
                coll.set_capture(None)
                if self._cur is not None:
                    self._end()
        torch.cuda.synchronize(self.device)
        return self.replay

    def replay(self) -> None:
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.ops):
                self.ops[i]()
