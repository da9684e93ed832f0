"""fp64 batched GEMM with fused diagonal scalings.

``gemm(A, B)`` computes ``alpha * diag(rs) @ op(A) @ op(B) @ diag(cs) + beta * C`` for 2-D or
3-D (batched) fp64 tensors.  On CPU it is the torch fp64 oracle.  On a HIP device:

* a product with a fused diagonal scaling runs ``pfml_dgemm`` (csrc/gemm_f64.hip,
  v_mfma_f64_16x16x4_f64, scales in the epilogue);
* a plain product (no scaling) is a library GEMM and goes to rocBLAS through torch
  (``baddbmm``), which sustains 40-66 TF/s fp64 on the S4 shapes against 19-40 TF/s for the
  hand-written tile (tools/bench_gemm.py, profiles/r01_gemm_own_vs_rocblas.json).

``backend="own"`` (or PFML_GEMM=own) forces the hand-written kernel, ``"blas"`` rocBLAS.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _native as nat

_P, _I, _L, _D = C.c_void_p, C.c_int, C.c_int64, C.c_double
nat.register_hip("pfml_gemm_lowp", [_I, _I, _I, _I, _I, _I, _I, _D, _P, _L, _L, _P, _L, _L, _D,
                                    _P, _L, _L, _P, _P, _P])
LOWP_FORMATS = {"bf16": 1, "fp8": 2}


def _as3(x):
    return x.unsqueeze(0) if x.dim() == 2 else x


def _bstride(x3, batch):
    return 0 if (x3.shape[0] == 1 and batch > 1) else x3.stride(0)


def _blas_gemm(A3, B3, trans_a, trans_b, alpha, beta, C3) -> None:
    a = A3.transpose(1, 2) if trans_a else A3
    b = B3.transpose(1, 2) if trans_b else B3
    if a.shape[0] != C3.shape[0]:
        a = a.expand(C3.shape[0], -1, -1)
    if b.shape[0] != C3.shape[0]:
        b = b.expand(C3.shape[0], -1, -1)
    if beta == 0.0:
        torch.bmm(a, b, out=C3) if alpha == 1.0 else C3.copy_(torch.bmm(a, b).mul_(alpha))
    else:
        C3.baddbmm_(a, b, beta=beta, alpha=alpha)


def gemm(A: torch.Tensor, B: torch.Tensor, *, trans_a: bool = False, trans_b: bool = False,
         alpha: float = 1.0, beta: float = 0.0, out: torch.Tensor | None = None,
         row_scale: torch.Tensor | None = None, col_scale: torch.Tensor | None = None,
         backend: str = "auto") -> torch.Tensor:
    squeeze = A.dim() == 2 and B.dim() == 2 and (out is None or out.dim() == 2)
    A3, B3 = _as3(A), _as3(B)
    batch = max(A3.shape[0], B3.shape[0])
    M = A3.shape[2] if trans_a else A3.shape[1]
    K = A3.shape[1] if trans_a else A3.shape[2]
    N = B3.shape[1] if trans_b else B3.shape[2]
    Kb = B3.shape[2] if trans_b else B3.shape[1]
    if K != Kb:
        raise ValueError(f"gemm: inner dims {K} vs {Kb}")
    if out is None:
        if beta != 0.0:
            raise ValueError("beta != 0 needs out=")
        out = torch.empty((batch, M, N), dtype=A.dtype, device=A.device)
    C3 = _as3(out)
    rs3 = None if row_scale is None else (row_scale.unsqueeze(0) if row_scale.dim() == 1 else row_scale)
    cs3 = None if col_scale is None else (col_scale.unsqueeze(0) if col_scale.dim() == 1 else col_scale)

    if backend == "auto":
        backend = os.environ.get("PFML_GEMM", "auto")
    if (nat.is_device(A) and backend != "own" and rs3 is None and cs3 is None
            and C3.stride(-1) == 1 and (backend == "blas" or A.dtype == torch.float64)):
        _blas_gemm(A3, B3, trans_a, trans_b, float(alpha), float(beta), C3)
    elif nat.is_device(A):
        if A.dtype != torch.float64:
            raise TypeError("pfml_dgemm is fp64-only")
        # a transposed view is consumed as-is by flipping the operand's transpose flag
        if A3.stride(-1) != 1:
            if A3.stride(-2) == 1:
                A3, trans_a = A3.transpose(1, 2), not trans_a
            else:
                A3 = A3.contiguous()
        if B3.stride(-1) != 1:
            if B3.stride(-2) == 1:
                B3, trans_b = B3.transpose(1, 2), not trans_b
            else:
                B3 = B3.contiguous()
        if C3.stride(-1) != 1:
            raise ValueError("gemm output must have unit inner stride")
        lib = nat.hip_lib()
        err = lib.pfml_dgemm(
            int(trans_a), int(trans_b), M, N, K, batch, float(alpha),
            A3.data_ptr(), A3.stride(1), _bstride(A3, batch),
            B3.data_ptr(), B3.stride(1), _bstride(B3, batch), float(beta),
            C3.data_ptr(), C3.stride(1), C3.stride(0),
            nat.ptr(rs3), 0 if rs3 is None else _bstride(rs3, batch),
            nat.ptr(cs3), 0 if cs3 is None else _bstride(cs3, batch),
            nat.stream_of(A))
        nat.check(err, "pfml_dgemm")
    else:
        a = A3.transpose(1, 2) if trans_a else A3
        b = B3.transpose(1, 2) if trans_b else B3
        r = torch.matmul(a, b)
        if rs3 is not None:
            r = r * rs3.unsqueeze(-1)
        if cs3 is not None:
            r = r * cs3.unsqueeze(-2)
        r = alpha * r
        if beta != 0.0:
            r = r + beta * C3
        C3.copy_(r.expand_as(C3))
    return out.squeeze(0) if squeeze and out.dim() == 3 else out


def _quantize(x: torch.Tensor, fmt: str) -> torch.Tensor:
    """CPU oracle of the kernel's operand rounding (bf16 RNE; e4m3 of x * 448 / amax)."""
    if fmt == "bf16":
        return x.float().to(torch.bfloat16).double()
    amax = float(x.abs().max())
    s = 448.0 / amax if amax > 0 else 1.0
    q = (x.float() * s).clamp(-448, 448).to(torch.float8_e4m3fn).double()
    return q / s


def gemm_lowp(A: torch.Tensor, B: torch.Tensor, fmt: str, *, trans_a: bool = False,
              trans_b: bool = False, alpha: float = 1.0, beta: float = 0.0,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """alpha op(A) op(B) + beta C with bf16 / fp8-e4m3 operands and fp32 accumulation
    (csrc/gemm_lowp.hip); fp64 in and out.  CPU: the same operand rounding in torch."""
    code = LOWP_FORMATS[fmt]
    squeeze = A.dim() == 2 and B.dim() == 2 and (out is None or out.dim() == 2)
    A3, B3 = _as3(A), _as3(B)
    batch = max(A3.shape[0], B3.shape[0])
    M = A3.shape[2] if trans_a else A3.shape[1]
    K = A3.shape[1] if trans_a else A3.shape[2]
    N = B3.shape[1] if trans_b else B3.shape[2]
    if out is None:
        out = torch.empty((batch, M, N), dtype=torch.float64, device=A.device)
    C3 = _as3(out)
    if nat.is_device(A):
        A3 = A3.contiguous() if A3.stride(-1) != 1 else A3
        B3 = B3.contiguous() if B3.stride(-1) != 1 else B3
        amax_a = A3.abs().amax().reshape(1).double() if fmt == "fp8" else None
        amax_b = B3.abs().amax().reshape(1).double() if fmt == "fp8" else None
        nat.check(nat.hip_lib().pfml_gemm_lowp(
            code, int(trans_a), int(trans_b), M, N, K, batch, float(alpha),
            A3.data_ptr(), A3.stride(1), _bstride(A3, batch),
            B3.data_ptr(), B3.stride(1), _bstride(B3, batch), float(beta),
            C3.data_ptr(), C3.stride(1), C3.stride(0), nat.ptr(amax_a), nat.ptr(amax_b),
            nat.stream_of(A)), "pfml_gemm_lowp")
    else:
        a = _quantize(A3, fmt)
        b = _quantize(B3, fmt)
        a = a.transpose(1, 2) if trans_a else a
        b = b.transpose(1, 2) if trans_b else b
        r = alpha * torch.matmul(a, b)
        if beta != 0.0:
            r = r + beta * C3
        C3.copy_(r.expand_as(C3))
    return out.squeeze(0) if squeeze and out.dim() == 3 else out


def gemm_fp32(A: torch.Tensor, B: torch.Tensor, *, trans_a: bool = False,
              trans_b: bool = False, alpha: float = 1.0, beta: float = 0.0,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """alpha op(A) op(B) + beta C with fp32 operands and accumulation (rocBLAS sgemm: the f32
    MFMA runs at twice the fp64 rate on gfx950), fp64 in and out."""
    a = A.to(torch.float32)
    b = B.to(torch.float32)
    if trans_a:
        a = a.transpose(-1, -2)
    if trans_b:
        b = b.transpose(-1, -2)
    C = torch.matmul(a, b).to(torch.float64)
    if alpha != 1.0:
        C.mul_(alpha)
    if out is None:
        return C
    if beta == 0.0:
        out.copy_(C)
    else:
        out.mul_(beta).add_(C)
    return out


def gemm_prec(A: torch.Tensor, B: torch.Tensor, precision: str = "fp64", **kw) -> torch.Tensor:
    """``gemm`` at the configured precision: fp64 (production) or an fp32 / bf16 / fp8
    experiment."""
    if precision in LOWP_FORMATS:
        return gemm_lowp(A, B, precision, **kw)
    if precision == "fp32":
        return gemm_fp32(A, B, **kw)
    return gemm(A, B, **kw)
