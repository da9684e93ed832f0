#!/usr/bin/env python3
"""Where the time of one batched one-triangle SPD inverse (ops/linalg.py spd_inverse_sym) goes
at the S4 production shape (B months of n = 490): every GEMM launch of the recursion timed on
its own (events around each call, synchronised), grouped by role and shape, the remainder being
the leaf inverses.  One JSON line per group plus the total and the achieved TF/s (n^3 flops per
matrix).

    python tools/micro/spd_inverse_levels.py [B] [n]
"""
import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pfml.ops.linalg as la  # noqa: E402


def spd_batch(B, n, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    X = torch.randn(B, n, n + 32, generator=g, dtype=torch.float64, device=dev)
    A = X @ X.transpose(1, 2) / n + 0.5 * torch.eye(n, dtype=torch.float64, device=dev)
    return 0.5 * (A + A.transpose(1, 2))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 715
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 490
    dev = torch.device("cuda", 0)
    A = spd_batch(B, n, dev)
    st = torch.zeros(B, dtype=torch.int32, device=dev)
    X = A.clone()
    la.spd_inverse_sym(X, st)                                   # warm-up (buffers, code)
    torch.cuda.synchronize()
    reps = 3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        X.copy_(A)
        la.spd_inverse_sym(X, st)
    e1.record()
    torch.cuda.synchronize()
    err = float((torch.bmm(X[:4], A[:4]) - torch.eye(n, device=dev, dtype=torch.float64))
                .abs().max())
    e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e2.record()
    for _ in range(reps):
        X.copy_(A)
    e3.record()
    torch.cuda.synchronize()
    total = (e0.elapsed_time(e1) - e2.elapsed_time(e3)) / reps
    # per-GEMM timing (synchronised launches)
    groups = defaultdict(lambda: [0, 0.0, 0.0])
    real = la.gemm_fused

    def timed(Aop, Bop, C, **kw):
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = real(Aop, Bop, C, **kw)
        e.record()
        torch.cuda.synchronize()
        M, N = C.shape[-2], C.shape[-1]
        K = Aop.shape[-2] if kw.get("trans_a") else Aop.shape[-1]
        role = "sym" if kw.get("sym") else ("mirror" if kw.get("mirror_out") is not None
                                            else "plain")
        key = f"{role}{'_tb' if kw.get('trans_b') else ''} {M}x{N}x{K}"
        g = groups[key]
        g[0] += 1
        g[1] += s.elapsed_time(e)
        g[2] += 2.0 * B * M * N * K * (0.5 if kw.get("sym") else 1.0)
        return out
    la.gemm_fused = timed
    X.copy_(A)
    la.spd_inverse_sym(X, st)
    la.gemm_fused = real
    gsum = 0.0
    for k, (c, ms, fl) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        gsum += ms
        print(json.dumps({"gemm": k, "calls": c, "ms": round(ms, 3),
                          "tflops": round(fl / (ms * 1e-3) / 1e12, 1)}), flush=True)
    print(json.dumps({"B": B, "n": n, "total_ms": round(total, 3), "gemm_ms_sync": round(gsum, 3),
                      "rest_ms (leaves + launch)": round(total - gsum, 3),
                      "tflops_n3": round(B * n ** 3 / (total * 1e-3) / 1e12, 1),
                      "max_abs_XA_minus_I": err}))


if __name__ == "__main__":
    main()
