"""fp64 batched GEMM with fused diagonal scalings.

``gemm(A, B)`` computes ``alpha * diag(rs) @ op(A) @ op(B) @ diag(cs) + beta * C`` for 2-D or
3-D (batched) fp64 tensors.  On CPU it is the torch fp64 oracle.  On a HIP device every
product runs ``pfml_dgemm`` (csrc/gemm_f64.hip, v_mfma_f64_16x16x4_f64, scales in the
epilogue): 54 TF/s plain and 51.5 TF/s with the fused Horner epilogue on the S4 shapes, against
56-61 TF/s for rocBLAS (profiles/r02_gemm_own_vs_rocblas.txt) - the engine has no library GEMM
on its paths.  ``backend="blas"`` (or PFML_GEMM=blas) routes an unscaled product to rocBLAS
through torch, as an explicit A/B only.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _native as nat
from ..utils import work as _work

_P, _I, _L, _D = C.c_void_p, C.c_int, C.c_int64, C.c_double


class _Epi(C.Structure):
    """Mirror of ``PfmlGemmEpi`` (csrc/gemm_f64.hip)."""
    _fields_ = [("alpha", _D), ("beta", _D), ("rs", _P), ("srs", _L), ("cs", _P), ("scs", _L),
                ("ks", _P), ("sks", _L), ("E", _P), ("lde", _L), ("sE", _L), ("e_cols", _I),
                ("diag_col0", _I), ("dval", _D), ("dv", _P), ("sdv", _L), ("has_diag", _I),
                ("es", _P), ("ses", _L), ("sincos", _I), ("sym", _I), ("Ct", _P), ("ldct", _L),
                ("sCt", _L), ("erow", _P), ("serow", _L), ("ecm", _P), ("ecs", _P),
                ("secm", _L), ("os", _P), ("sos", _L), ("tile_cfg", _I), ("ms", _I), ("ns", _I)]


nat.register_hip("pfml_dgemm_ex", [_I, _I, _I, _I, _I, _I, _P, _L, _L, _P, _L, _L, _P, _L, _L,
                                   C.POINTER(_Epi), _P])
nat.register_hip("pfml_gemm_epi_size", [])
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


def _ledger(ta, tb, M, N, K, batch, A3, B3, C3, ks=None, sks=0, sincos=False, cfg=0,
            extra_bytes=0, sym=False):
    """Work-ledger entry of one pfml_dgemm_ex launch under the kernel name its dispatch picks
    (the tile / vector-width / k-scale choice of csrc/gemm_f64.hip, mirrored); a symmetric
    launch counts the flops of the tiles it runs (on and below the diagonal)."""
    cfg = 0 if cfg < 0 else (cfg or _TILE_DEFAULT)          # -1: pfml_dgemm (always auto)
    if cfg == 0:
        cfg = _auto_cfg(M, N, K, sym, batch)
    if cfg == 1 and sincos:
        cfg = 3
    if sym and cfg in (2, 8, 10):
        cfg = 3 if cfg == 2 else 7
    lda, ldb = A3.stride(1), B3.stride(1)
    sa, sb = _bstride(A3, batch), _bstride(B3, batch)
    a_cont, b_cont = (M if ta else K), (K if tb else N)
    vec = (a_cont % 2 == 0 and b_cont % 2 == 0 and lda % 2 == 0 and ldb % 2 == 0
           and sa % 2 == 0 and sb % 2 == 0 and A3.data_ptr() % 16 == 0
           and B3.data_ptr() % 16 == 0
           and (ks is None or (ks.data_ptr() % 16 == 0 and sks % 2 == 0)))
    # the LDS-DMA forms load the k-scale in 16-byte pairs: they also need an even K
    if cfg in (6, 7, 8, 9, 10, 11) and not (vec and not sincos and min(M, N, K) >= 2 and
                                            (ks is None or K % 2 == 0)):
        cfg = 3
    bm, bn = {1: (128, 128), 2: (128, 64), 6: (128, 128), 8: (128, 64), 9: (128, 128),
              10: (128, 64), 11: (128, 128)}.get(cfg, (64, 64))
    bk, nbuf = {4: (32, 1), 5: (32, 2)}.get(cfg, (16, 2))
    b = lambda v: "true" if v else "false"                                  # noqa: E731
    if cfg in (6, 7, 8, 9, 10, 11):
        wm, wn = (4, 2) if cfg in (9, 11) else (2, 2)
        name = (f"dgemm_glds_kernel<{b(ta)}, {b(tb)}, {bm}, {bn}, {b(ks is not None)}, "
                f"{wm}, {wn}, {3 if cfg >= 10 else 2}>")
    else:
        name = (f"dgemm_kernel<{b(ta)}, {b(tb)}, {bm}, {bn}, {2 if vec else 1}, "
                f"{b(ks is not None)}, {bk}, {nbuf}>")
    na = M * K * (A3.shape[0] if sa else 1)
    nb = K * N * (B3.shape[0] if sb else 1)
    frac = 1.0
    if sym:
        t = -(-M // bm)
        frac = 0.5 * (t + 1) / t
    _work.add(name, 2.0 * batch * M * N * K * frac,
              8.0 * (na + nb + batch * M * N) * frac + extra_bytes)


_SMALL_TILES = int(os.environ.get("PFML_GEMM_SMALL_TILES", "256"))


def _auto_cfg(M: int, N: int, K: int, sym: bool = False, batch: int = 1) -> int:
    """Host mirror of the auto tile choice of pfml_dgemm_ex (tile_cfg 0; the LDS-DMA forms
    fall back to 3 where their 16-byte chunking does not apply, mirrored in _ledger): a launch
    of fewer than PFML_GEMM_SMALL_TILES 128 x 64 tiles takes 64 x 64 tiles (same bits)."""
    cfg = 6 if (M >= 1024 and N >= 1024) else (7 if sym else 8)
    if cfg == 8 and -(-M // 128) * -(-N // 64) * batch < _SMALL_TILES:
        cfg = 7
    return cfg


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
        backend = os.environ.get("PFML_GEMM", "own")
    if (nat.is_device(A) and backend == "blas" and rs3 is None and cs3 is None
            and C3.stride(-1) == 1):
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
        if _work.on():
            _ledger(trans_a, trans_b, M, N, K, batch, A3, B3, C3, cfg=-1,
                    extra_bytes=8.0 * batch * M * N if beta != 0.0 else 0)
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


def _vec3(v, batch):
    """[n] or [B, n] scale vector -> (3-D-compatible tensor, batch stride)."""
    if v is None:
        return None, 0
    v2 = v.unsqueeze(0) if v.dim() == 1 else v
    if v2.stride(-1) != 1:
        v2 = v2.contiguous()
    return v2, (0 if (v2.shape[0] == 1 and batch > 1) else v2.stride(0))


# A/B switch for the auto tile choice (0 auto, 1: 128x128, 2: 128x64, 3: 64x64; 4, 5: BK = 32
# variants, csrc/gemm_f64.hip PfmlGemmEpi), read once
_TILE_DEFAULT = int(os.environ.get("PFML_GEMM_TILE", "0"))
# the same for symmetric-mode products only (square tiles: 3 / 7 64 x 64, 1 / 6 128 x 128)
_SYM_TILE = int(os.environ.get("PFML_SYM_TILE", "0"))


def gemm_fused(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, *, trans_a: bool = False,
               trans_b: bool = False, alpha: float = 1.0, beta: float = 0.0,
               row_scale: torch.Tensor | None = None, col_scale: torch.Tensor | None = None,
               k_scale: torch.Tensor | None = None, addend: torch.Tensor | None = None,
               addend_cols: int | None = None, diag_col0: int | None = None,
               diag_value: float = 1.0, diag_vec: torch.Tensor | None = None,
               addend_row_scale: torch.Tensor | None = None, sincos: bool = False,
               tile_cfg: int = 0, sym: bool = False,
               mirror_out: torch.Tensor | None = None,
               addend_rows: torch.Tensor | None = None,
               addend_col_shift: torch.Tensor | None = None,
               addend_col_scale: torch.Tensor | None = None,
               out_row_scale: torch.Tensor | None = None,
               clip: bool = False) -> torch.Tensor:
    """out = diag(os) (alpha diag(rs) op(A) diag(ks) op(B) diag(cs) + beta out
             + diag(es) addend[:, :, :addend_cols]  (on out's first addend_cols columns)
             + diag(diag_vec or diag_value) placed at out[:, i, diag_col0 + i]).

    ``out_row_scale`` (os, applied last): e.g. the next Horner step's k-scale folded into this
    step's output rows, so that step's main loop needs none.

    ``sym=True``: the result is known to be symmetric (square out): only its lower triangle is
    computed (the output tiles on and below the diagonal) and mirrored, so out comes back
    exactly symmetric (beta / addend read at the lower positions only).  ``mirror_out``
    [.., N, M]: also receives the transpose of the result (X21 = X12' of the SPD inverse).

    Gathered addend (``addend_rows`` [B, M] int64, ``addend_col_shift`` / ``addend_col_scale``
    [B, addend_cols]): the addend row i is (addend[rows[b, i]] - shift[b]) * scale[b] (times
    the addend row scale) - the standardised signals of the Horner steps formed from the panel
    features on the fly.  ``addend`` is then the [R, >= addend_cols] feature table (2-D).

    One launch of csrc/gemm_f64.hip on a HIP device (the Horner step of (24), Sigma = X F X'
    + diag(ivol), ...); the same arithmetic in torch fp64 on CPU.  3-D batched operands
    (batch stride 0 = broadcast); scale vectors are [n] or [B, n].

    ``sincos=True`` (K13): v = alpha op(A) op(B) never stored - out (width >= 2 N + 1) gets
    the row [1, cos v_1, sin v_1, cos v_2, sin v_2, ...] (columns past 2 N + 1 untouched).

    ``clip=True``: out is [.., Ms, Ns] with Ms <= M, Ns <= N - the product is computed at the
    operands' full (e.g. even-padded) size and only its leading Ms x Ns block is read (beta)
    and stored, straight into the final buffer (no padded temporary + copy)."""
    A3, B3, C3 = _as3(A), _as3(B), _as3(out)
    batch = C3.shape[0]
    M = A3.shape[2] if trans_a else A3.shape[1]
    K = A3.shape[1] if trans_a else A3.shape[2]
    N = B3.shape[1] if trans_b else B3.shape[2]
    Ms, Ns = (C3.shape[1], C3.shape[2]) if clip else (M, N)
    if clip and (sincos or Ms > M or Ns > N or mirror_out is not None or Ms < 1 or Ns < 1):
        raise ValueError("gemm_fused(clip): out [.., <= M, <= N], no sincos / mirror_out")
    if sincos:
        if C3.shape[1] != M or C3.shape[2] < 2 * N + 1:
            raise ValueError("gemm_fused(sincos): out must be [.., M, >= 2N + 1]")
    elif (B3.shape[2] if trans_b else B3.shape[1]) != K or tuple(C3.shape[1:]) != (Ms, Ns):
        raise ValueError(f"gemm_fused: shapes {tuple(A3.shape)} {tuple(B3.shape)} -> {tuple(C3.shape)}")
    if addend is not None and addend_cols is None:
        addend_cols = N
    if sym and (M != N or sincos):
        raise ValueError("gemm_fused(sym): square output, no sincos")
    gathered = addend_rows is not None
    if gathered and (addend is None or addend.dim() != 2 or addend_col_shift is None
                     or addend_col_scale is None):
        raise ValueError("gemm_fused: a gathered addend needs a 2-D table, shift and scale")
    E3 = None if addend is None else _as3(addend)
    T3 = None if mirror_out is None else _as3(mirror_out)
    if T3 is not None and (tuple(T3.shape[1:]) != (N, M) or T3.stride(-1) != 1):
        raise ValueError("gemm_fused: mirror_out must be [.., N, M] with unit inner stride")
    if nat.is_device(A):
        for x, nm in ((A3, "A"), (B3, "B"), (C3, "out")):
            if x.stride(-1) != 1:
                raise ValueError(f"gemm_fused: {nm} needs unit inner stride")
        if E3 is not None and E3.stride(-1) != 1:
            raise ValueError("gemm_fused: addend needs unit inner stride")
        rs, srs = _vec3(row_scale, batch)
        cs, scs = _vec3(col_scale, batch)
        ks, sks = _vec3(k_scale, batch)
        dv, sdv = _vec3(diag_vec, batch)
        es, ses = _vec3(addend_row_scale, batch)
        osc, sos = _vec3(out_row_scale, batch)
        er = ecm = ecs = None
        ser = secm = 0
        if gathered:
            er = addend_rows if addend_rows.dim() == 2 else addend_rows.unsqueeze(0)
            ecm = addend_col_shift if addend_col_shift.dim() == 2 else addend_col_shift.unsqueeze(0)
            ecs = addend_col_scale if addend_col_scale.dim() == 2 else addend_col_scale.unsqueeze(0)
            if (er.dtype != torch.int64 or er.stride(-1) != 1 or ecm.stride(-1) != 1
                    or ecs.stride(-1) != 1 or ecm.stride(0) != ecs.stride(0)):
                raise ValueError("gemm_fused: gathered addend layout")
            ser = 0 if er.shape[0] == 1 else er.stride(0)
            secm = 0 if ecm.shape[0] == 1 else ecm.stride(0)
        ep = _Epi(float(alpha), float(beta), nat.ptr(rs), srs, nat.ptr(cs), scs, nat.ptr(ks), sks,
                  nat.ptr(E3), 0 if E3 is None else E3.stride(1),
                  0 if (E3 is None or gathered) else _bstride(E3, batch), int(addend_cols or 0),
                  int(diag_col0 or 0), float(diag_value), nat.ptr(dv), sdv,
                  int(diag_col0 is not None), nat.ptr(es), ses, int(sincos), int(sym),
                  nat.ptr(T3), 0 if T3 is None else T3.stride(1),
                  0 if T3 is None else T3.stride(0), nat.ptr(er), ser, nat.ptr(ecm),
                  nat.ptr(ecs), secm, nat.ptr(osc), sos, int(tile_cfg or (_SYM_TILE if sym else 0) or _TILE_DEFAULT),
                  int(Ms) if clip else 0, int(Ns) if clip else 0)
        if _work.on():
            _ledger(trans_a, trans_b, M, N, K, batch, A3, B3, C3, ks=ks, sks=sks,
                    sincos=sincos, cfg=tile_cfg, sym=sym,
                    extra_bytes=8.0 * batch * M * ((N if beta != 0.0 else 0)
                                                   + (addend_cols or 0 if E3 is not None else 0)
                                                   + (N if T3 is not None else 0)))
        nat.check(nat.hip_lib().pfml_dgemm_ex(
            int(trans_a), int(trans_b), M, N, K, batch,
            A3.data_ptr(), A3.stride(1), _bstride(A3, batch),
            B3.data_ptr(), B3.stride(1), _bstride(B3, batch),
            C3.data_ptr(), C3.stride(1), C3.stride(0), C.byref(ep), nat.stream_of(A)),
            "pfml_dgemm_ex")
        return out
    a = A3.transpose(1, 2) if trans_a else A3
    b = B3.transpose(1, 2) if trans_b else B3
    if k_scale is not None:
        ksv = k_scale if k_scale.dim() == 2 else k_scale.unsqueeze(0)
        b = b * ksv.unsqueeze(-1)
    r = torch.matmul(a, b)
    if row_scale is not None:
        rsv = row_scale if row_scale.dim() == 2 else row_scale.unsqueeze(0)
        r = r * rsv.unsqueeze(-1)
    if col_scale is not None:
        csv = col_scale if col_scale.dim() == 2 else col_scale.unsqueeze(0)
        r = r * csv.unsqueeze(-2)
    r = alpha * r
    if sincos:
        C3[:, :, 0] = 1.0
        C3[:, :, 1:2 * N + 1:2] = torch.cos(r)
        C3[:, :, 2:2 * N + 1:2] = torch.sin(r)
        return out
    if beta != 0.0:
        if clip:
            Cf = torch.zeros((batch, M, N), dtype=C3.dtype, device=C3.device)
            Cf[:, :Ms, :Ns] = C3
            r = r + beta * Cf
        else:
            r = r + beta * C3
    r = r.expand(batch, M, N).clone()
    if E3 is not None and addend_cols:
        if gathered:
            er = addend_rows if addend_rows.dim() == 2 else addend_rows.unsqueeze(0)
            sh = addend_col_shift if addend_col_shift.dim() == 2 else addend_col_shift.unsqueeze(0)
            scl = addend_col_scale if addend_col_scale.dim() == 2 else addend_col_scale.unsqueeze(0)
            Ea = (addend[:, :addend_cols][er] - sh[:, None, :addend_cols]) * \
                scl[:, None, :addend_cols]
        else:
            Ea = E3[:, :, :addend_cols]
        if addend_row_scale is not None:
            esv = addend_row_scale if addend_row_scale.dim() == 2 else addend_row_scale.unsqueeze(0)
            Ea = Ea * esv.unsqueeze(-1)
        r[:, :, :addend_cols] += Ea
    if diag_col0 is not None:
        n = min(M, N - diag_col0)
        ii = torch.arange(n, device=r.device)
        if diag_vec is not None:
            dvv = diag_vec if diag_vec.dim() == 2 else diag_vec.unsqueeze(0)
            r[:, ii, diag_col0 + ii] += dvv[:, :n]
        else:
            r[:, ii, diag_col0 + ii] += diag_value
    if out_row_scale is not None:
        osv = out_row_scale if out_row_scale.dim() == 2 else out_row_scale.unsqueeze(0)
        r = r * osv.unsqueeze(-1)
    if sym:                                     # the lower triangle, mirrored (device form)
        r = torch.tril(r) + torch.tril(r, -1).transpose(-1, -2)
    C3.copy_(r[:, :Ms, :Ns] if clip else r)
    if T3 is not None:
        T3.copy_(r.transpose(-1, -2))
    return out
