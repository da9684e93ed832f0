#!/usr/bin/env python3
"""Accuracy of the device m_func forms (ops/linalg.py) at the production shape: the
Denman-Beavers square root vs a symmetric eigendecomposition, and m = diag(a) m_tilde diag(1/a)
vs the reference-form torch m_func (LU inverses, convergence-checked sqrtm), for the
Denman-Beavers switches DB_SYM (one-triangle inverse) and DB_SYMPROD (one-triangle Y M^-1).
Prints one JSON line per arm (max relative errors).

    python tools/micro/mfunc_accuracy.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pfml.ops.linalg as la  # noqa: E402


def case(B=6, N=496, K=25, n=489, tc=True, seed=1):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(B, N, K))
    X[:, n:] = 0.0
    F = np.stack([np.cov(rng.normal(size=(K, 300))) * 21e-4 for _ in range(B)])
    iv = rng.uniform(0.01, 0.03, (B, N)) ** 2 * 21
    iv[:, n:] = 1.0
    S = np.einsum("bik,bkl,bjl->bij", X, F, X) + np.stack([np.diag(v) for v in iv])
    S = 0.5 * (S + S.transpose(0, 2, 1))
    w = np.linspace(3e9, 1e10, B)
    lam = 0.2 / rng.uniform(1e7, 1e9, (B, N)) if tc else np.full((B, N), 1e-16)
    lam[:, n:] = 10.0 / w[:, None]
    mask = np.zeros((B, N))
    mask[:, :n] = 1.0
    t = lambda v: torch.tensor(v, dtype=torch.float64)                      # noqa: E731
    return (t(S), t(lam), t(w), t(np.full(B, 0.002)), 0.007, 10.0, 10), t(mask)


def main():
    dev = torch.device("cuda", 0)
    out = {}
    refs = {}
    for tc in (True, False):
        args, mask = case(tc=tc)
        refs[tc] = (args, mask, la.m_func_reference(*args, mask=mask))
    for arm, (dbs, dbp) in {"base": (False, False), "db_sym": (True, False),
                            "db_symprod": (False, True), "both": (True, True)}.items():
        la.DB_SYM, la.DB_SYMPROD = dbs, dbp
        rec = {}
        for tc, (args, mask, ref) in refs.items():
            dargs = [x.to(dev) if isinstance(x, torch.Tensor) else x for x in args]
            mt, a = la.m_tilde(*dargs, mask=mask.to(dev), sigma_exact_sym=False)
            got = (mt * a.unsqueeze(-1) / a.unsqueeze(-2)).cpu()
            rec[f"m_rel_tc{int(tc)}"] = float((got - ref).abs().max() / ref.abs().max())
        # the square root alone vs eigh
        g = torch.Generator().manual_seed(3)
        Xs = torch.randn(4, 496, 496, generator=g, dtype=torch.float64)
        ev = torch.logspace(-6, 0, 496, dtype=torch.float64)
        Q, _ = torch.linalg.qr(Xs)
        S = Q @ torch.diag_embed(ev.expand(4, -1)) @ Q.transpose(1, 2)
        S = 0.5 * (S + S.transpose(1, 2))
        ref = Q @ torch.diag_embed(ev.sqrt().expand(4, -1)) @ Q.transpose(1, 2)
        Sd = S.to(dev).contiguous()
        ws = [torch.empty_like(Sd) for _ in range(4)]
        st = torch.zeros(4, dtype=torch.int32, device=dev)
        root = la._db_sqrt(Sd, la.DB_ITERS, la.DB_SCALED_ITERS, st, ws).cpu()
        rec["sqrt_rel_vs_eigh"] = float((root - ref).abs().max() / ref.abs().max())
        out[arm] = rec
        print(json.dumps({arm: rec}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
