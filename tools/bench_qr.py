#!/usr/bin/env python3
"""Panel-QR micro-benchmark: band_panel_hh (csrc/ridge_band.hip) in isolation.

Cycles per m x 16 panel factorisation (the band reduction's serial step, once per panel on
the critical chain of every ridge cell), column-by-column Householder with the panel in LDS,
with ``nblocks`` workgroups factoring at once (1: latency alone; 106: the one-GPU grid's big
cells), plus the numerics: Q = I - V T V' orthogonal and Q' P = [R; 0] to fp64 rounding.
(A CholeskyQR2 + Householder-reconstruction form measured 45-60 % slower per panel,
profiles/r04_qr_bench_dpp.jsonl, and was removed.)

    python tools/bench_qr.py [m ...]            (default m = 497 241 113)
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.ops import _native as nat  # noqa: E402

nat.register_hip("pfml_band_qr_bench", [C.c_void_p, C.c_int, C.c_int, C.c_int,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p])


def panels(nblocks: int, m: int, kind: str, seed: int = 0) -> torch.Tensor:
    """Panels like the band reduction's: columns of a window-sum matrix D = X'X (kind 'full':
    X of 700 rows, full rank; 'deficient': 90 rows, rank-deficient columns)."""
    g = torch.Generator().manual_seed(seed)
    nobs = 700 if kind != "deficient" else 90
    X = torch.randn(nblocks, nobs, m + 16, generator=g, dtype=torch.float64)
    D = X.transpose(1, 2) @ X / nobs
    P = D[:, 16:, :16].contiguous()               # rows below the diagonal block
    if kind == "dup":                             # exactly dependent columns: CholeskyQR2
        P[:, :, 5] = P[:, :, 3]                   # must hand the panel to Householder
        P[:, :, 9] = 0.0
    return P


def run(m: int, nblocks: int, kind: str, reps: int = 20) -> dict:
    dev = torch.device("cuda", 0)
    P = panels(nblocks, m, kind).to(dev)
    lda = m + 16
    A = torch.zeros(nblocks, lda, lda, dtype=torch.float64, device=dev)
    V = torch.zeros(nblocks, m, 16, dtype=torch.float64, device=dev)
    T = torch.zeros(nblocks, 16, 16, dtype=torch.float64, device=dev)
    cyc = torch.zeros(nblocks, 8, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    nat.check(nat.hip_lib().pfml_band_qr_bench(P.data_ptr(), m, nblocks, reps,
                                               A.data_ptr(), V.data_ptr(), T.data_ptr(),
                                               cyc.data_ptr(), st), "pfml_band_qr_bench")
    torch.cuda.synchronize()
    # numerics of block 0: Q = I - V T V', Q' P = [R; 0]
    Pc, Vc, Tc = P[0].cpu(), V[0].cpu(), T[0].cpu()
    R = torch.triu(A[0, 16:16 + 16, :16].cpu()) if m >= 16 else None
    Q = torch.eye(m, dtype=torch.float64) - Vc @ Tc @ Vc.T
    orth = (Q.T @ Q - torch.eye(m, dtype=torch.float64)).abs().max().item()
    QP = Q.T @ Pc
    rerr = None
    if R is not None:
        ref = torch.zeros_like(QP)
        ref[:16] = R
        rerr = ((QP - ref).abs().max() / Pc.abs().max()).item()
    c = cyc.float()[0].tolist()                   # block 0 (the others: cycles_max)
    return {"m": m, "blocks": nblocks, "panel": kind, "cycles_per_panel": int(c[0]),
            "cycles_max": int(cyc[:, 0].max()), "orth_err": orth, "qp_err": rerr,
            "load": int(c[1]), "columns": int(c[2]), "g_t": int(c[3]), "col_own": int(c[4]),
            "col_barrier": int(c[5]), "col_chain_update": int(c[6])}


if __name__ == "__main__":
    ms = [int(x) for x in sys.argv[1:]] or [497, 241, 113]
    out = []
    for m in ms:
        for nb in (1, 106):
            for kind in (("full", "deficient", "dup") if nb == 1 else ("full",)):
                r = run(m, nb, kind)
                out.append(r)
                print(json.dumps(r), flush=True)
