"""Tracing: roctx ranges (visible in rocprofv3 --marker-trace) and stage timers.

The reference only has tqdm bars and prints.  Here every stage and kernel
group is bracketed by a roctx range when tracing is on (``PFML_TRACE=1`` or
``Config.run.profile``), and ``StageTimer`` records device-synchronised wall time per stage
into the JSONL metrics stream (utils/metrics.py).
"""
from __future__ import annotations

import ctypes
import os
import time
from contextlib import contextmanager

import torch

_roctx = None
_enabled = os.environ.get("PFML_TRACE", "0") not in ("0", "", "false")


def enable(flag: bool = True) -> None:
    global _enabled
    _enabled = flag


def _lib():
    global _roctx
    if _roctx is None:
        _roctx = False
        for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so",
                     "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx


def range_push(name: str) -> None:
    if _enabled:
        lib = _lib()
        if lib:
            lib.roctxRangePushA(name.encode())


def range_pop() -> None:
    if _enabled:
        lib = _lib()
        if lib:
            lib.roctxRangePop()


@contextmanager
def trace_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


def sync(device=None) -> None:
    if torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda"):
        torch.cuda.synchronize(device)


class StageTimer:
    """Accumulates synchronised wall time per named stage."""

    def __init__(self, device=None):
        self.device = device
        self.times: dict[str, float] = {}

    @contextmanager
    def __call__(self, name: str):
        sync(self.device)
        t0 = time.perf_counter()
        range_push(name)
        try:
            yield
        finally:
            sync(self.device)
            range_pop()
            self.times[name] = self.times.get(name, 0.0) + time.perf_counter() - t0
