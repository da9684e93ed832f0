#!/usr/bin/env python3
"""Residual max |X A - I| of the batched SPD inverses (ops/linalg.py: one-triangle
spd_inverse_sym, two-sided spd_inverse_into) over batch sizes up to the S4 production batch,
with the batch indices of the worst matrices.

    python tools/micro/spd_inverse_check.py [n] [B ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pfml.ops.linalg as la  # noqa: E402
from tools.micro.spd_inverse_levels import spd_batch  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 490
    Bs = [int(b) for b in sys.argv[2:]] or [8, 64, 256, 512, 715]
    dev = torch.device("cuda", 0)
    eye = torch.eye(n, dtype=torch.float64, device=dev)
    for B in Bs:
        A = spd_batch(B, n, dev)
        rec = {"B": B, "n": n}
        for name in ("sym", "two_sided"):
            st = torch.zeros(B, dtype=torch.int32, device=dev)
            if name == "sym":
                X = A.clone()
                la.spd_inverse_sym(X, st)
            else:
                X = torch.empty_like(A)
                la.spd_inverse_into(A, X, st)
            r = (torch.bmm(X, A) - eye).abs().amax((1, 2))
            bad = torch.nonzero(r > 1e-10).flatten()
            rec[name] = {"max_res": float(r.max()), "n_bad": int(bad.numel()),
                         "first_bad": bad[:8].tolist(), "status": int(st.sum())}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
