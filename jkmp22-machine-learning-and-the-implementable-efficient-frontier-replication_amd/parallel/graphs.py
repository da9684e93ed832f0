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

No collective ever runs on the capture stream: the warm-up and every eager collective (at
capture and at replay) run on a separate communication stream, joined to the capture /
replay stream by event waits.  ProcessGroupNCCL (RCCL) records a collective's completion
event on the stream it ran on, and its watchdog thread polls those events; HIP refuses a
query of an event whose stream is capturing (hipErrorCapturedEvent), so an event left on
the capture stream aborted the process as soon as the next segment began capturing.
"""
from __future__ import annotations

import torch

from . import collectives as coll


class SegmentedGraph:
    def __init__(self, device: torch.device):
        self.device = device
        self.stream = torch.cuda.Stream(device=device)      # capture stream (graphs only)
        self.comm = torch.cuda.Stream(device=device)        # warm-up and eager collectives
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs: list = []
        self.ops: list = []
        self._cur = None

    def _begin(self) -> None:
        g = torch.cuda.CUDAGraph()
        # thread-local capture mode: the process group's watchdog thread keeps polling its
        # (non-captured) events while a segment is being captured
        g.capture_begin(pool=self.pool, capture_error_mode="thread_local")
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
        s, c = self.stream, self.comm
        c.wait_stream(s)
        with torch.cuda.stream(c):
            res = fn(None, x, counts)                   # eager, allocates the result shape
            out = torch.empty_like(res)
            out.copy_(res)
        s.wait_stream(c)
        dev = self.device

        def op():
            cur = torch.cuda.current_stream(dev)
            c.wait_stream(cur)
            with torch.cuda.stream(c):
                fn(out, x, counts)
            cur.wait_stream(c)

        self.ops.append(op)
        self._begin()
        return out

    def capture(self, fn):
        """Warm up ``fn`` once eagerly, then capture it segment-wise; returns the replay."""
        s, c = self.stream, self.comm
        cur = torch.cuda.current_stream(self.device)
        c.wait_stream(cur)
        with torch.cuda.stream(c):
            fn()                                      # plans, caches, allocator state
        cur.wait_stream(c)
        torch.cuda.synchronize(self.device)
        s.wait_stream(cur)
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
