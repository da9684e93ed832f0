"""Process-group setup: one process per GPU, RCCL over xGMI (backend "nccl" on ROCm).

The reference is single-process.  Here every stage is data-parallel over
months or hyper-parameter cells; ranks talk only through a handful of small collectives
(shard totals, utilities, chosen weights), so the layout is the same on 1, 2, 4 or 8 GPUs of
one node.  On CPU-only hosts the same code runs over gloo (tests, world_size > 1).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    # PFML_DIST_FORCE=1: the distributed code path (process group, collectives, segmented
    # graphs) even at world size 1 - on a one-GPU box this is how RCCL itself is exercised
    force: bool = False

    @property
    def is_dist(self) -> bool:
        return ((self.world_size > 1 or self.force) and dist.is_available()
                and dist.is_initialized())

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_ENV: DistEnv | None = None


def init(device: str = "auto", timeout_s: int = 600) -> DistEnv:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*)."""
    global _ENV
    if _ENV is not None:
        return _ENV
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    want_gpu = device in ("auto", "cuda") and torch.cuda.is_available()
    if device == "cuda" and not torch.cuda.is_available():
        raise RuntimeError("device=cuda requested but no HIP device is visible")
    if want_gpu:
        torch.cuda.set_device(lrank % max(1, torch.cuda.device_count()))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    backend = "none"
    force = ws == 1 and os.environ.get("PFML_DIST_FORCE", "0") == "1"
    if ws > 1 or force:
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if dev.type == "cuda" else "gloo"
        # PFML_DIST_BACKEND=gloo with GPUs: ranks may share a device (a rehearsal of the
        # multi-GPU path on a one-GPU box; collectives stage through the host)
        backend = os.environ.get("PFML_DIST_BACKEND", backend)
        if not dist.is_initialized():
            kw = {}
            if dev.type == "cuda" and backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(backend=backend, rank=rank, world_size=ws,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _ENV = DistEnv(rank=rank, world_size=ws, local_rank=lrank, device=dev, backend=backend,
                   force=force)
    return _ENV


def env() -> DistEnv:
    return _ENV if _ENV is not None else DistEnv()


def set_env(e: DistEnv | None) -> None:
    """Install an explicit environment (tests that drive ranks by hand)."""
    global _ENV
    _ENV = e


def barrier() -> None:
    e = env()
    if e.is_dist:
        if e.backend == "nccl":
            dist.barrier(device_ids=[e.device.index])
        else:
            dist.barrier()


def shutdown() -> None:
    global _ENV
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _ENV = None
