"""Work ledger for the roofline tables: floating-point operations and minimum HBM bytes per
kernel name, summed over a run (tools/roofline_s4.py joins it with a rocprofv3 kernel-stats
table of the same run).

Off by default (one ``if`` per call).  ``PFML_WORK_LEDGER=<file.json>`` turns it on at import
and writes ``{kernel: {"calls", "flops", "bytes"}}`` there at exit.  The names are the
kernels' demangled template names as rocprofv3 prints them, e.g.
``dgemm_kernel<false, false, 64, 64, 2, true>``.
"""
from __future__ import annotations

import atexit
import json
import os

_PATH = os.environ.get("PFML_WORK_LEDGER")
LEDGER: dict | None = {} if _PATH else None


def on() -> bool:
    return LEDGER is not None


def add(kernel: str, flops: float = 0.0, nbytes: float = 0.0, calls: int = 1) -> None:
    if LEDGER is None:
        return
    e = LEDGER.setdefault(kernel, {"calls": 0, "flops": 0.0, "bytes": 0.0})
    e["calls"] += calls
    e["flops"] += float(flops)
    e["bytes"] += float(nbytes)


def _dump() -> None:
    if LEDGER is not None and _PATH:
        with open(_PATH, "w") as f:
            json.dump(LEDGER, f, indent=1, sort_keys=True)


atexit.register(_dump)
