#!/usr/bin/env python3
"""Validation-utility kernel (csrc/quadform.hip) in isolation, at the headline shapes:
12 validation months x 106 (g, year) cells for each p (n = 513 / 257 / 129 / 65), 101 lambdas.
Prints ms per launch and the achieved fp64 rate (symmetric half of D_t B counted)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.ops.ridge import quadform_utilities  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    T, P, L, C = 120, 513, 101, 106
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(T, 64, P, generator=g, dtype=torch.float64, device=dev)
    D = X.transpose(1, 2) @ X / 64
    R = torch.randn(T, P, generator=g, dtype=torch.float64, device=dev)
    beta = torch.randn(C, L, P, generator=g, dtype=torch.float64, device=dev) * 0.01
    out = {}
    for n in (513, 257, 129, 65):
        jc = np.repeat(np.arange(C), 12)
        jm = (np.arange(C * 12) * 7) % T
        jn = np.full(C * 12, n)
        quadform_utilities(D, R, beta, jc, jm, jn)
        torch.cuda.synchronize()
        reps = 5
        t = time.perf_counter()
        for _ in range(reps):
            quadform_utilities(D, R, beta, jc, jm, jn)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / reps * 1e3
        flops = len(jc) * (n * n + n * 64) * 101 * 2 / 2      # upper block triangle
        out[f"n{n}_ms"] = round(ms, 3)
        out[f"n{n}_tflops"] = round(flops / ms / 1e9, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
