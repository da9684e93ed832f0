"""Stage artifacts, done-markers and resume.

The reference's only "checkpoints" are the files each stage writes (SQLite, CSV, pickles).
Here every stage writes into ``<artifact_dir>/<stage>/`` and finishes with a ``_DONE.json``
marker holding the config hash of the settings it depends on; ``Pipeline`` skips a stage
whose marker matches and reruns it (and everything downstream) otherwise.  Sharded stages
write one marker per rank (``_DONE.rank<r>.json``) so a multi-GPU run resumes only the
shards that are missing.  Tensors are stored with ``torch.save`` and loaded with
``weights_only=True``; tables as CSV; arrays as ``.npz`` (no pickle).
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch


class ArtifactStore:
    def __init__(self, root: str):
        self.root = root

    def dir(self, stage: str) -> str:
        p = os.path.join(self.root, stage)
        os.makedirs(p, exist_ok=True)
        return p

    def _marker(self, stage: str, rank: int | None) -> str:
        name = "_DONE.json" if rank is None else f"_DONE.rank{rank}.json"
        return os.path.join(self.root, stage, name)

    def is_done(self, stage: str, key: str, rank: int | None = None) -> bool:
        m = self._marker(stage, rank)
        if not os.path.exists(m):
            return False
        try:
            with open(m, encoding="utf-8") as f:
                return json.load(f).get("key") == key
        except (OSError, ValueError):
            return False

    def mark_done(self, stage: str, key: str, rank: int | None = None, **info) -> None:
        self.dir(stage)
        m = self._marker(stage, rank)
        tmp = m + ".tmp"
        with open(tmp, "w", encoding="utf-8") as f:
            json.dump({"key": key, "time": time.time(), **info}, f, default=str)
        os.replace(tmp, m)

    def invalidate(self, stage: str) -> None:
        d = os.path.join(self.root, stage)
        if os.path.isdir(d):
            for n in os.listdir(d):
                if n.startswith("_DONE"):
                    os.remove(os.path.join(d, n))

    # -- payloads ------------------------------------------------------------------
    def save_tensors(self, stage: str, name: str, tensors: dict) -> str:
        p = os.path.join(self.dir(stage), name + ".pt")
        cpu = {k: (v.detach().cpu() if isinstance(v, torch.Tensor) else
                   torch.as_tensor(v) if isinstance(v, np.ndarray) else v)
               for k, v in tensors.items()}
        tmp = p + ".tmp"
        torch.save(cpu, tmp)
        os.replace(tmp, p)
        return p

    def load_tensors(self, stage: str, name: str, device="cpu") -> dict:
        p = os.path.join(self.root, stage, name + ".pt")
        d = torch.load(p, map_location=device, weights_only=True)
        return d

    def path(self, stage: str, name: str) -> str:
        return os.path.join(self.dir(stage), name)
