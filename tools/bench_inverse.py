#!/usr/bin/env python3
"""SPD inverse on the m_func shape ([256, 490, 490] fp64): recursive Schur-complement blocks,
fused symmetric Gauss-Jordan steps
(csrc/spd_inverse.hip, 3 launches per block) vs the generic block steps (pivot kernel + fused
GEMMs + copies) interleaved in one process (torch.linalg.inv / rocSOLVER getrf-batched fails to allocate
at this batch)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.ops.linalg import spd_inverse  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, n = 256, 490
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn((B, n + 40, n), generator=g, dtype=torch.float64, device=dev)
    A = X.transpose(1, 2) @ X / n + 0.05 * torch.eye(n, dtype=torch.float64, device=dev)
    I = torch.eye(n, dtype=torch.float64, device=dev)
    res = {}
    fns = {"recursive": ("recursive", lambda: spd_inverse(A)),
           "fused_sym": ("sym", lambda: spd_inverse(A)), "generic": ("generic", lambda: spd_inverse(A)),
           "generic128": ("generic128", lambda: spd_inverse(A))}
    for k, (envv, f) in fns.items():
        os.environ["PFML_SPD_INV"] = envv
        out = f()
        res[k + "_resid"] = float((out @ A - I).abs().max())
    ts = {k: [] for k in fns}
    for _ in range(3):
        for k, (envv, f) in fns.items():
            os.environ["PFML_SPD_INV"] = envv
            f()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                f()
            torch.cuda.synchronize()
            ts[k].append((time.perf_counter() - t) / 5)
    for k, v in ts.items():
        res[k + "_ms"] = round(1000 * min(v), 3)
        res[k + "_tflops_2n3"] = round(2.0 * B * n ** 3 / min(v) / 1e12, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
