#!/usr/bin/env python3
"""Ridge-grid kernel debugging: relative error of the GPU tridiagonalisation variants vs the
CPU reference for one cell per size (PFML_RIDGE_VARIANT is read per call)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.ops.ridge import ridge_grid  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    lv = torch.tensor([0.0] + list(np.exp(np.linspace(-10, 10, 100))), dtype=torch.float64)
    out = {}
    for n in [int(a) for a in (sys.argv[1:] or ["9", "17", "33", "65", "129", "257", "513"])]:
        X = torch.randn(2 * n + 40, n, dtype=torch.float64, generator=g)
        SD = (X.T @ X)[None]
        if os.environ.get("DEBUG_INDEF"):      # indefinite: small lambdas take the LU repair
            SD = SD - 0.5 * torch.linalg.eigvalsh(SD[0]).max() * torch.eye(n, dtype=SD.dtype)
        Sr = torch.randn(1, n, dtype=torch.float64, generator=g)
        args = (np.array([0]), np.array([n]), np.array([0.01]))
        ref = ridge_grid(SD, Sr, *args, lv)
        for var, mode in (("u", ""), ("f", ""), ("band", "")):
            os.environ["PFML_RIDGE_VARIANT"] = var
            got = ridge_grid(SD.to(dev), Sr.to(dev), *args, lv.to(dev)).cpu()
            rel = ((got - ref).norm(dim=-1) / ref.norm(dim=-1)).max().item()
            out[f"n{n}_{var}{mode}"] = float(f"{rel:.3e}")
            print(n, var, mode, rel, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
