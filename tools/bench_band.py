#!/usr/bin/env python3
"""Band-reduction ridge grid: wall time per launch vs number of n = 513 cells, for the
single-workgroup and the multi-workgroup reduction (PFML_BAND_MODE).  With few cells per
GPU (the 8-GPU strong-scaling case: ~14 big cells per rank) the single-workgroup form is
latency-bound by one CU per cell."""
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
    S = max(1, min(ncells, 8))
    X = torch.randn(S, 600, P, dtype=torch.float64, device=dev)
    SD = X.transpose(1, 2) @ X
    Sr = torch.randn(S, P, dtype=torch.float64, device=dev)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64,
                      device=dev)
    src = np.arange(ncells) % S
    nn = np.full(ncells, n)
    sc = np.full(ncells, 1e-3)
    ridge_grid(SD, Sr, src, nn, sc, lv, repair=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        ridge_grid(SD, Sr, src, nn, sc, lv, repair=False)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


if __name__ == "__main__":
    cells = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "1,14,28,106").split(",")]
    out = {}
    for mode in ("single", "multi"):
        os.environ["PFML_BAND_MODE"] = mode
        for c in cells:
            for n in (513, 257):
                out[f"{mode}_n{n}_cells{c}_ms"] = round(run(c, n), 3)
    print(json.dumps(out))
