#!/usr/bin/env python3
"""The in-house fp64 GEMM (csrc/gemm_f64.hip) on the S4 shapes and a large square, each tile
config, a few launches each: the program a `rocprofv3 --pmc` / `--kernel-trace` pass runs
(tools/gpu_run.sh step dgemmpmc), and a TF/s table when run alone.

Shapes: the Horner step of (24) (m_tilde x [S | I | R], k-scaled, addend + identity
epilogue), the recursive SPD inverse's Schur GEMMs at the top level of n = 490 (W = X11 A12,
S = A22 - A21 W, X12, X21 = -X22 W', X11 -= X12 W'), the Denman-Beavers product Y M^-1, and
large squares.  Configs (PfmlGemmEpi.tile_cfg): 1 128x128, 3 64x64 (register staging),
6 / 7 / 8 LDS-DMA 128x128 / 64x64 / 128x64.

    python tools/micro/dgemm_shapes.py [reps]        PFML_DGEMM_CFGS=3,6,7,8  PFML_DGEMM_SHAPES=..
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pfml.ops.gemm import gemm_fused  # noqa: E402

SHAPES = [  # name, batch, M, N, K, trans_a, trans_b, horner fusion
    ("horner", 256, 490, 2006, 490, False, False, True),
    ("horner_plain", 256, 490, 2006, 490, False, False, False),
    ("horner_ks", 256, 490, 2006, 490, False, False, "ks"),
    ("inv_W", 384, 256, 234, 256, False, False, False),
    ("inv_S", 384, 234, 234, 256, False, False, False),
    ("inv_X21", 384, 234, 256, 234, False, True, False),
    ("inv_X11", 384, 256, 256, 234, False, True, False),
    ("inv_S_sym", 384, 234, 234, 256, False, False, "sym"),
    ("inv_X11_sym", 384, 256, 256, 234, False, True, "sym"),
    ("inv_X12_mirror", 384, 256, 234, 234, False, False, "mirror"),
    ("inv_h128", 384, 128, 128, 128, False, False, False),
    ("db_prod", 256, 490, 490, 490, False, False, False),
    ("gram_tn", 128, 514, 514, 490, True, False, False),
    # K sweep at equal flops (per-tile prologue / epilogue vs main-loop cost)
    ("k256", 256, 512, 2048, 256, False, False, False),
    ("k512", 128, 512, 2048, 512, False, False, False),
    ("k1024", 64, 512, 2048, 1024, False, False, False),
    ("k4096", 16, 512, 2048, 4096, False, False, False),
    ("square8192", 1, 8192, 8192, 8192, False, False, False),
    ("square2048", 4, 2048, 2048, 2048, False, False, False),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    cfgs = [int(c) for c in os.environ.get("PFML_DGEMM_CFGS", "3,6,7,8,9,10,11").split(",")]
    pick = os.environ.get("PFML_DGEMM_SHAPES")
    shapes = [s for s in SHAPES if not pick or s[0] in pick.split(",")]
    dev = torch.device("cuda", 0)
    out = {}
    for name, b, M, N, K, ta, tb, fused in shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        A = torch.rand((b, K, M) if ta else (b, M, K), generator=g, dtype=torch.float64,
                       device=dev) - 0.5
        B = torch.rand((b, N, K) if tb else (b, K, N), generator=g, dtype=torch.float64,
                       device=dev) - 0.5
        C = torch.empty((b, M, N), dtype=torch.float64, device=dev)
        kw = dict(trans_a=ta, trans_b=tb)
        mode, fused = (fused if isinstance(fused, str) else ""), fused is True
        if mode == "sym":
            kw.update(sym=True)
        elif mode == "ks":
            kw.update(k_scale=torch.rand((b, K), generator=g, dtype=torch.float64, device=dev) + 0.5)
        elif mode == "mirror":
            kw.update(mirror_out=torch.empty((b, N, M), dtype=torch.float64, device=dev))
        if fused:
            kw.update(k_scale=torch.rand((b, K), generator=g, dtype=torch.float64, device=dev) + 0.5,
                      row_scale=torch.rand((b, M), generator=g, dtype=torch.float64, device=dev) + 0.5,
                      addend=torch.rand((b, M, N - 2 * M), generator=g, dtype=torch.float64,
                                        device=dev),
                      addend_cols=N - 2 * M, diag_col0=N - 2 * M)
        opa = A.transpose(1, 2) if ta else A
        opb = B.transpose(1, 2) if tb else B
        if fused:
            ref = torch.bmm(opa * kw["k_scale"].unsqueeze(1), opb) * kw["row_scale"].unsqueeze(-1)
            ref[:, :, :N - 2 * M] += kw["addend"]
            ref[:, :, N - 2 * M:N - M] += torch.eye(M, dtype=torch.float64, device=dev)
        elif mode == "ks":
            ref = torch.bmm(opa * kw["k_scale"].unsqueeze(1), opb)
        else:
            ref = torch.bmm(opa, opb)
        if mode == "sym":
            ref = torch.tril(ref) + torch.tril(ref, -1).transpose(1, 2)
        fl = 2.0 * b * M * N * K          # (sym: the full product's flops, for comparison)
        for cfg in cfgs:
            C.fill_(float("nan"))                     # no stale result can pass the check
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
