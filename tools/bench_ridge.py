#!/usr/bin/env python3
"""Micro-benchmark of the ridge-grid kernels: wall time vs number of concurrent cells.

Distinguishes a per-reflector latency bound (time flat in #cells) from a memory-system bound
(time grows once the cells' working sets exceed L2 / Infinity Cache)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.ops.ridge import ridge_grid  # noqa: E402


def run(ncells, n, reps=3):
    dev = torch.device("cuda", 0)
    P = 513
    S = max(1, ncells // 4)
    X = torch.randn(S, 600, P, dtype=torch.float64, device=dev)
    SD = X.transpose(1, 2) @ X
    Sr = torch.randn(S, P, dtype=torch.float64, device=dev)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64,
                      device=dev)
    src = np.arange(ncells) % S
    nn = np.full(ncells, n)
    sc = np.full(ncells, 1e-3)
    ridge_grid(SD, Sr, src, nn, sc, lv)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        ridge_grid(SD, Sr, src, nn, sc, lv)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def timing(n=513):
    """Per-phase cycle split of the cooperative band reduction: 8 phase slots for workgroup 0
    (the QR one) and 1 of cell 0, plus the banded solve's forward / backward cycles."""
    from pfml.ops import _native as nat
    dev = torch.device("cuda", 0)
    ncells = int(os.environ.get("PFML_TIMING_CELLS", "1"))
    buf = torch.zeros(ncells * 16 + 16, dtype=torch.int64, device=dev)
    nat.hip_lib().pfml_ridge_set_timing(buf.data_ptr())
    run(ncells, n, reps=1)
    torch.cuda.synchronize()
    nat.hip_lib().pfml_ridge_set_timing(None)
    allb = buf.cpu().numpy()
    names = ["init_panel0", "U", "X_partials", "sync_wait", "C_sums_W", "update",
             "lookahead_qr", "end_sync"]
    out = {"K": os.environ.get("PFML_COOP_K", "auto"), "cells": ncells}
    for w in (0, 1):
        t = allb[w * 8:(w + 1) * 8]
        tot = max(1, int(t.sum()))
        out[f"wg{w}"] = {nm: f"{int(v)} cyc ({100.0 * v / tot:.1f}%)" for nm, v in zip(names, t)}
        out[f"wg{w}_total_cyc"] = tot
    out.update({"solve_fwd_cyc": int(allb[ncells * 16]),
                "solve_bwd_cyc": int(allb[ncells * 16 + 1])})
    return out


if __name__ == "__main__":
    if "--timing" in sys.argv:
        print(json.dumps(timing(), indent=1))
        sys.exit(0)
    out = {}
    ncs = [int(x) for x in os.environ.get("PFML_BENCH_CELLS", "1,8,32,106,212").split(",")]
    for n in (513, 257):
        for nc in ncs:
            out[f"n{n}_cells{nc}_ms"] = round(run(nc, n), 3)
            print(n, nc, out[f"n{n}_cells{nc}_ms"], flush=True)
    print(json.dumps(out))
