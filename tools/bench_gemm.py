#!/usr/bin/env python3
"""fp64 batched GEMM: the hand-written MFMA kernel (csrc/gemm_f64.hip) vs torch (rocBLAS)
on the S4 shapes (Horner chain, risk / tc products, Sigma build)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.ops.gemm import gemm  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for (b, M, N, K, ta) in [(64, 500, 1526, 500, False), (64, 500, 1026, 500, False),
                             (64, 513, 513, 500, True), (64, 500, 500, 500, False),
                             (8, 3000, 4026, 3000, False)]:
        A = torch.randn((b, K, M) if ta else (b, M, K), dtype=torch.float64, device=dev)
        B = torch.randn((b, K, N), dtype=torch.float64, device=dev)
        C = torch.randn((b, M, N), dtype=torch.float64, device=dev)
        fl = 2.0 * b * M * N * K
        t_own = timeit(lambda: gemm(A, B, trans_a=ta, beta=1.0, out=C))
        At = A.transpose(1, 2) if ta else A
        t_blas = timeit(lambda: torch.baddbmm(C, At, B, out=C))
        key = f"b{b}_m{M}_n{N}_k{K}{'_ta' if ta else ''}"
        out[key] = {"own_tflops": round(fl / t_own / 1e12, 2),
                    "rocblas_tflops": round(fl / t_blas / 1e12, 2)}
        del A, B, C
    print(json.dumps(out))


if __name__ == "__main__":
    main()
