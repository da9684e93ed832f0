#!/usr/bin/env python3
"""fp64 batched GEMM on the S4 shapes: the hand-written MFMA kernel (csrc/gemm_f64.hip, each
tile config, with and without the Horner fusions) vs rocBLAS (torch.baddbmm), interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24).  Random operands."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.ops.gemm import gemm_fused  # noqa: E402


def timeit(fn, reps=5):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = torch.device("cuda", 0)
    shapes = [  # (batch, M, N, K, trans_a, horner_fusion)
        (122, 490, 2006, 490, False, True),     # Horner step with the lag-1 block R (GP + 2N)
        (256, 496, 1522, 496, False, True),     # Horner step, 2 distinct g (GP = 1026)
        (256, 496, 1010, 496, False, True),     # Horner step, compat (GP = 514)
        (256, 496, 496, 496, False, False),     # x^2, DB products, inverse * Omega
        (256, 514, 514, 496, True, False),      # risk / tc: omega' (Sigma omega)
        (256, 496, 1522, 64, False, False),     # rank-64 elimination update
        (8, 3000, 4026, 3000, False, False),    # 3000-stock stress
    ]
    out = {}
    for (b, M, N, K, ta, fused) in shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        A = torch.rand((b, K, M) if ta else (b, M, K), generator=g, dtype=torch.float64, device=dev) - 0.5
        B = torch.rand((b, K, N), generator=g, dtype=torch.float64, device=dev) - 0.5
        C = torch.empty((b, M, N), dtype=torch.float64, device=dev)
        ks = torch.rand((b, K), generator=g, dtype=torch.float64, device=dev) + 0.5
        E = torch.rand((b, M, N - M), generator=g, dtype=torch.float64, device=dev)
        fl = 2.0 * b * M * N * K
        At = A.transpose(1, 2) if ta else A
        res = {}
        fns = {"rocblas": lambda: torch.bmm(At, B, out=C)}
        for cfg in (1, 2, 3):
            fns[f"own{cfg}"] = (lambda cfg=cfg: gemm_fused(A, B, C, trans_a=ta, tile_cfg=cfg))
            if fused:
                fns[f"own{cfg}_fused"] = (lambda cfg=cfg: gemm_fused(
                    A, B, C, trans_a=ta, k_scale=ks, addend=E, addend_cols=N - M,
                    diag_col0=N - M, tile_cfg=cfg))
        for f in fns.values():
            f()
        # correctness of the plain product vs rocBLAS
        ref = torch.bmm(At, B)
        gemm_fused(A, B, C, trans_a=ta)
        err = float((C - ref).abs().max() / ref.abs().max())
        ts = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                ts[k].append(timeit(f))
        for k, v in ts.items():
            res[k] = round(fl / min(v) / 1e12, 2)
        res["max_rel_err_vs_rocblas"] = err
        key = f"b{b}_m{M}_n{N}_k{K}{'_ta' if ta else ''}"
        out[key] = res
        print(key, res, flush=True)
        del A, B, C, E, ks
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
