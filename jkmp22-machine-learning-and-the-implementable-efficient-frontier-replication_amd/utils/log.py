"""Stage logging + JSONL metrics.

``get_logger(stage)`` returns a stdlib logger that prints the reference's diagnostics (screen
exclusion shares, turnover, ...) so output stays comparable; ``metric(**kv)`` appends a JSON
line (stage timings, solves/s, fallback counts, oracle errors) to ``$PFML_METRICS`` or
``<artifact_dir>/metrics.jsonl`` when configured.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time

_METRICS_PATH: str | None = os.environ.get("PFML_METRICS")


def get_logger(stage: str) -> logging.Logger:
    log = logging.getLogger(f"pfml.{stage}")
    if not logging.getLogger("pfml").handlers:
        h = logging.StreamHandler(sys.stdout)
        h.setFormatter(logging.Formatter("[%(name)s] %(message)s"))
        root = logging.getLogger("pfml")
        root.addHandler(h)
        root.setLevel(os.environ.get("PFML_LOGLEVEL", "INFO"))
        root.propagate = False
    return log


def set_metrics_path(p: str | None) -> None:
    global _METRICS_PATH
    _METRICS_PATH = p


def metric(**kv) -> dict:
    rec = {"ts": time.time(), **kv}
    if _METRICS_PATH:
        os.makedirs(os.path.dirname(os.path.abspath(_METRICS_PATH)), exist_ok=True)
        with open(_METRICS_PATH, "a", encoding="utf-8") as f:
            f.write(json.dumps(rec, default=str) + "\n")
    return rec


class Counters:
    """Numerical-fallback counters reported per stage (Cholesky->LU->pinv, NaN guards...)."""

    def __init__(self):
        self.c: dict[str, int] = {}

    def add(self, key: str, n: int = 1) -> None:
        self.c[key] = self.c.get(key, 0) + int(n)

    def as_dict(self) -> dict:
        return dict(self.c)


COUNTERS = Counters()
