#!/usr/bin/env python3
"""Library DGEMM rate (torch.matmul fp64 -> rocBLAS/hipBLASLt) and the in-house fp64 GEMM on
large square shapes: the empirical fp64 MFMA ceiling the roofline table quotes against."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pfml.ops.gemm import gemm  # noqa: E402


def rate(fn, flops, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return flops * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12


out = {}
dev = torch.device("cuda", 0)
for n in (2048, 4096, 8192):
    a = torch.randn(n, n, dtype=torch.float64, device=dev)
    b = torch.randn(n, n, dtype=torch.float64, device=dev)
    c = torch.empty(n, n, dtype=torch.float64, device=dev)
    f = 2.0 * n ** 3
    out[f"n{n}"] = {"library": round(rate(lambda: torch.matmul(a, b, out=c), f), 2),
                    "own": round(rate(lambda: gemm(a, b, out=c, backend="own"), f), 2)}
    print(n, out[f"n{n}"], flush=True)
print(json.dumps(out))
