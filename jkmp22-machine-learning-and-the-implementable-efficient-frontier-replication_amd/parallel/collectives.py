"""Collectives used by the sharded stages (RCCL on GPU, gloo on CPU).

Every collective here moves MB-scale messages: shard totals of the expanding
window sums (one P x P matrix per g per rank), per-cell utilities, chosen coefficients.
On xGMI these are latency-bound, so the design point is *few* collectives per stage, not
bucketing.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .dist import env


def _comm_device(x: torch.Tensor) -> torch.device:
    """Where a collective on ``x`` must run: gloo takes host tensors (PFML_DIST_BACKEND=gloo:
    several ranks sharing one GPU, a rehearsal of the multi-GPU path where RCCL cannot run),
    RCCL device tensors - so a CPU tensor under RCCL (e.g. the S9 CPU recompute of a failure
    recovery) is staged through this rank's GPU, a device tensor under gloo through the host."""
    e = env()
    if e.backend == "gloo":
        return torch.device("cpu")
    return e.device if e.device.type == "cuda" else x.device


def _staged(x: torch.Tensor) -> bool:
    return x.device != _comm_device(x)


def all_gather_cat(x: torch.Tensor) -> torch.Tensor:
    """Concatenate equally-shaped tensors of every rank along dim 0 (rank order)."""
    e = env()
    if not e.is_dist:
        return x
    if _staged(x):
        return all_gather_cat(x.to(_comm_device(x))).to(x.device)
    x = x.contiguous()
    out = torch.empty((e.world_size * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x)
    return out


def all_gather_varlen(x: torch.Tensor) -> torch.Tensor:
    """Concatenate tensors whose first dimension differs per rank (rank order)."""
    e = env()
    if not e.is_dist:
        return x
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    ns = all_gather_cat(n).cpu().numpy()
    m = int(ns.max())
    pad = torch.zeros((m, *x.shape[1:]), dtype=x.dtype, device=x.device)
    if x.shape[0]:
        pad[: x.shape[0]] = x
    g = all_gather_cat(pad)
    parts = [g[r * m: r * m + int(ns[r])] for r in range(e.world_size)]
    return torch.cat(parts, 0)


# Segmented HIP-graph capture (parallel/graphs.py): while a step is being captured, the
# collectives below end the current graph segment, run eagerly into a static output and
# start the next segment; a replay then alternates segment graphs and these collectives.
_CAPTURE = None


def set_capture(cap) -> None:
    global _CAPTURE
    _CAPTURE = cap


def all_gather_known(x: torch.Tensor, counts) -> torch.Tensor:
    """all_gather_varlen when every rank's first-dim size is already known everywhere (e.g.
    from a plan all ranks share): ONE collective, no size exchange and no host round trip."""
    e = env()
    if not e.is_dist:
        return x
    if _CAPTURE is not None:
        return _CAPTURE.collective(_all_gather_known_into, x, counts)
    return _all_gather_known_into(None, x, counts)


def _all_gather_known_into(out: torch.Tensor | None, x: torch.Tensor, counts) -> torch.Tensor:
    """all_gather_known; with ``out`` the result is copied into that (static) tensor."""
    e = env()
    counts = [int(c) for c in counts]
    if len(counts) != e.world_size or x.shape[0] != counts[e.rank]:
        raise ValueError(f"all_gather_known: rank {e.rank} holds {x.shape[0]} rows, "
                         f"counts {counts}")
    m = max(counts)
    if m == 0:
        return x
    if min(counts) == m and not _staged(x):
        # equal shares (e.g. the chunk totals when the chunks split evenly over the ranks):
        # the rank-order concatenation IS the all-gather output - gathered straight into the
        # (static) destination, no padding, no concatenation, no copy
        if out is None:
            out = torch.empty((e.world_size * m, *x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x.contiguous())
        return out
    pad = x.contiguous()
    if x.shape[0] < m:
        pad = torch.zeros((m, *x.shape[1:]), dtype=x.dtype, device=x.device)
        pad[: x.shape[0]] = x
    g = all_gather_cat(pad)
    res = torch.cat([g[r * m: r * m + counts[r]] for r in range(e.world_size)], 0)
    if out is None:
        return res
    out.copy_(res)
    return out


def exclusive_prefix_sum(total: torch.Tensor) -> torch.Tensor:
    """Sum of ``total`` over all lower ranks (zeros on rank 0): cross-GPU exclusive scan."""
    e = env()
    if not e.is_dist:
        return torch.zeros_like(total)
    g = all_gather_cat(total.unsqueeze(0))
    if e.rank == 0:
        return torch.zeros_like(total)
    return g[: e.rank].sum(0)


def all_reduce_max(v: float, device=None) -> float:
    e = env()
    if not e.is_dist:
        return float(v)
    t = torch.tensor([float(v)], dtype=torch.float64, device=device or e.device)
    t = t.to(_comm_device(t))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum_(t: torch.Tensor) -> torch.Tensor:
    e = env()
    if e.is_dist:
        if _staged(t):
            h = t.to(_comm_device(t))
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def broadcast_object(obj, src: int = 0):
    e = env()
    if not e.is_dist:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src,
                               device=e.device if e.backend == "nccl" else None)
    return box[0]


def contiguous_split(n: int, world: int, rank: int) -> range:
    """Balanced contiguous block of range(n) for ``rank`` (first n % world ranks get +1)."""
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return range(start, start + q + (1 if rank < r else 0))


def weighted_split(weights, world: int) -> list[range]:
    """Contiguous split of items with positive weights into ``world`` near-equal-weight blocks."""
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if world <= 1 or n == 0:
        return [range(0, n)] + [range(n, n)] * (world - 1)
    cum = np.concatenate([[0.0], np.cumsum(w)])
    bounds = [0]
    for r in range(1, world):
        target = cum[-1] * r / world
        b = int(np.searchsorted(cum, target))
        b = min(max(b, bounds[-1]), n)
        bounds.append(b)
    bounds.append(n)
    return [range(bounds[i], bounds[i + 1]) for i in range(world)]


def send_next(x: torch.Tensor) -> None:
    """Point-to-point send to rank + 1 (a pipeline hand-off, e.g. the portfolio recursion's
    w_start vector: N doubles over one xGMI link)."""
    e = env()
    if e.is_dist and e.rank + 1 < e.world_size:
        dist.send(x.to(_comm_device(x)).contiguous(), dst=e.rank + 1)


def recv_prev(like: torch.Tensor) -> torch.Tensor:
    """Receive the tensor ``send_next`` of rank - 1 sent (shape / dtype of ``like``); rank 0
    (and a non-distributed run) gets zeros, so a chain never starts from uninitialised
    memory."""
    e = env()
    out = torch.zeros_like(like)
    if e.is_dist and e.rank > 0:
        if _staged(out):
            h = torch.empty_like(out, device=_comm_device(out))
            dist.recv(h, src=e.rank - 1)
            out.copy_(h)
        else:
            dist.recv(out, src=e.rank - 1)
    return out
