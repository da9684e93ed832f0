#!/usr/bin/env python3
"""The in-house fp64 GEMM (csrc/gemm_f64.hip) on the S4 Horner shape and a large square, each
tile config, a few launches each: the program a `rocprofv3 --pmc` / `--kernel-trace` pass runs
(tools/gpu_run.sh step dgemmpmc), and a TF/s table when run alone.

    python tools/micro/dgemm_shapes.py [reps]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pfml.ops.gemm import gemm_fused  # noqa: E402

SHAPES = [  # name, batch, M, N, K, horner fusion
    ("horner", 256, 496, 1522, 496, True),
    ("square8192", 1, 8192, 8192, 8192, False),
    ("square2048", 4, 2048, 2048, 2048, False),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    cfgs = [int(c) for c in os.environ.get("PFML_DGEMM_CFGS", "1,3,4,5").split(",")]
    dev = torch.device("cuda", 0)
    out = {}
    for name, b, M, N, K, fused in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        A = torch.rand((b, M, K), generator=g, dtype=torch.float64, device=dev) - 0.5
        B = torch.rand((b, K, N), generator=g, dtype=torch.float64, device=dev) - 0.5
        C = torch.empty((b, M, N), dtype=torch.float64, device=dev)
        kw = {}
        if fused:
            kw = dict(k_scale=torch.rand((b, K), generator=g, dtype=torch.float64, device=dev) + 0.5,
                      addend=torch.rand((b, M, N - M), generator=g, dtype=torch.float64, device=dev),
                      addend_cols=N - M, diag_col0=N - M)
        ref = torch.bmm(A * kw["k_scale"].unsqueeze(1), B) if fused else torch.bmm(A, B)
        if fused:
            ref[:, :, :N - M] += kw["addend"]
            ref[:, :, N - M:] += torch.eye(M, dtype=torch.float64, device=dev)
        fl = 2.0 * b * M * N * K
        for cfg in cfgs:
            gemm_fused(A, B, C, tile_cfg=cfg, **kw)
            err = float((C - ref).abs().max() / ref.abs().max())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                gemm_fused(A, B, C, tile_cfg=cfg, **kw)
            e1.record()
            torch.cuda.synchronize()
            tf = fl * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12
            out[f"{name}_cfg{cfg}"] = {"tflops": round(tf, 2), "rel_err": err}
            print(name, cfg, out[f"{name}_cfg{cfg}"], flush=True)
        del A, B, C, ref, kw
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
