#!/usr/bin/env python3
"""Bitwise A/B of two builds of the SPD-inverse kernels (csrc/spd_inverse.hip: the 64-leaf
Gauss-Jordan, the one-launch 65..128-row node, the one-triangle recursive inverse) and of the
pivoted LU solve (csrc/lu_solve.hip).

    PFML_HIP_LIB=<lib A> python tools/micro/inverse_ab.py save A.json
    PFML_HIP_LIB=<lib B> python tools/micro/inverse_ab.py save B.json
    python tools/micro/inverse_ab.py cmp A.json B.json

``save`` inverts fixed-seed SPD batches (n = 490: nodes of 128 and 106 rows; n = 100: one
node; n = 64 and 37: a single leaf) with ``spd_inverse_sym`` and stores the results and the
launch times (the results as SHA-256 digests); ``cmp`` reports per case whether the digests
match (bitwise equal).
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pfml.ops.linalg as la  # noqa: E402

# (batches large enough that the GPU, not the Python launch path, sets the time)
CASES = [(192, 490), (2048, 100), (4096, 64), (4096, 37)]


def _spd(B, n, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    X = torch.randn(B, n, n + 32, generator=g, dtype=torch.float64, device=dev)
    A = X @ X.transpose(1, 2) / (n + 32) + 1e-3 * torch.eye(n, dtype=torch.float64, device=dev)
    return 0.5 * (A + A.transpose(1, 2))


def save(path):
    dev = torch.device("cuda", 0)
    out, times = {}, {}
    for k, (B, n) in enumerate(CASES):
        A = _spd(B, n, dev, k)
        X = torch.empty_like(A)
        st = torch.zeros(B, dtype=torch.int32, device=dev)
        la.spd_inverse_sym(X, st, src=A)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            la.spd_inverse_sym(X, st, src=A)
        e1.record()
        torch.cuda.synchronize()
        err = float((torch.bmm(X, A) - torch.eye(n, dtype=A.dtype, device=dev)).abs().max())
        out[f"{B}x{n}"] = hashlib.sha256(X.cpu().numpy().tobytes()).hexdigest()
        times[f"{B}x{n}"] = {"ms": round(e0.elapsed_time(e1) / reps, 4), "max_abs_XA_minus_I": err,
                             "status": int(st.sum())}
    # the pivoted LU solve of augmented [B | A] rows (csrc/lu_solve.hip, the S4 const^-1 Omega
    # form: one- and two-level), general A (partial pivoting active)
    for k, (B, n, m, two) in enumerate([(64, 490, 258, True), (64, 490, 258, False),
                                        (24, 137, 66, True)]):
        g = torch.Generator(device=dev).manual_seed(100 + k)
        Wz = m + n + (la.LU_PANEL_COLS if two else 0)
        M0 = torch.randn(B, n, Wz, generator=g, dtype=torch.float64, device=dev)
        M = M0.clone()
        st = torch.zeros(B, dtype=torch.int32, device=dev)
        z0 = m + n if two else None
        la.solve_augmented(M, n, m, a0=m, b0=0, status=st, z0=z0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            M.copy_(M0)
            la.solve_augmented(M, n, m, a0=m, b0=0, status=st, z0=z0)
        e1.record()
        torch.cuda.synchronize()
        X = M[:, :, :m]
        res = float((torch.bmm(M0[:, :, m:m + n], X) - M0[:, :, :m]).abs().max())
        key = f"lu{'2' if two else '1'}_{B}x{n}x{m}"
        out[key] = hashlib.sha256(X.contiguous().cpu().numpy().tobytes()).hexdigest()
        times[key] = {"ms_incl_copy": round(e0.elapsed_time(e1) / 10, 4), "max_abs_residual": res,
                      "status": int(st.sum())}
    with open(path, "w") as f:
        json.dump(out, f)
    print(json.dumps({"lib": os.environ.get("PFML_HIP_LIB", "in-tree"), "cases": times}))


def cmp(pa, pb):
    with open(pa) as fa, open(pb) as fb:
        a, b = json.load(fa), json.load(fb)
    res = {k: a[k] == b[k] for k in a}
    print(json.dumps({"sha256_equal": res, "bitwise_equal": all(res.values())}))


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
