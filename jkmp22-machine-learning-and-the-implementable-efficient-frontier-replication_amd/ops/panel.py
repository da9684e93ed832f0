"""Panel signal ops: RFF features (K13) and per-month standardisation (K11/K12).

Device paths run the fused GEMM (csrc/gemm_f64.hip, sincos epilogue) and csrc/panel.hip; CPU
paths are the torch fp64 oracle
of PFML_Input_Data.py:179-185 (cos/sin of X W) and :364-388 (demean, unit L2 norm, 1/vol).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _native as nat
from ..utils import work as _work
from .gemm import gemm_fused, gemm_prec

nat.register_hip("pfml_rff_sincos", [C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int64,
                                     C.c_void_p])
nat.register_hip("pfml_standardize", [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                                      C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                      C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_int64,
                                      C.c_int, C.c_void_p, C.c_int64, C.c_void_p])
nat.register_hip("pfml_date_sums", [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                                    C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p])
nat.register_hip("pfml_excl_stats", [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                                     C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                     C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_void_p])


def rff_features(X: torch.Tensor, W: torch.Tensor, precision: str = "fp64",
                 width: int | None = None, pad_rows: int = 0,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """[R, k] x [k, P/2] -> [R + pad_rows, width] rows [1, cos z1, sin z1, cos z2, sin z2, ...,
    0 ...] (P = 2 (P/2) + 1 real columns; ``width`` >= P pads with zero columns, ``pad_rows``
    appends all-zero rows).  fp64 on a device: ONE launch of the fused GEMM whose epilogue
    writes cos / sin of each accumulator straight into the interleaved row (X W never
    stored); ``precision`` fp32 / bf16 / fp8 (experimental configs): the lowered GEMM, then the
    sincos kernel.  ``out``: a [R + pad_rows, width] (column block) view to write into."""
    R, half = X.shape[0], W.shape[1]
    P = 2 * half + 1
    width = width or P
    if out is not None and (tuple(out.shape) != (R + pad_rows, width) or out.stride(-1) != 1):
        raise ValueError("rff_features: out must be a [R + pad_rows, width] row-major view")
    if nat.is_device(X) and precision == "fp64":
        if out is None:
            out = torch.empty((R + pad_rows, width), dtype=X.dtype, device=X.device)
        if pad_rows:
            out[R:].zero_()
        if width > P:
            out[:R, P:].zero_()
        Xc, Wc = X.contiguous(), W.contiguous()
        # row chunks: the GEMM's epilogue addresses one output with 32-bit byte offsets (< 2 GB)
        ch = max(1, ((1 << 31) // 8 - out.shape[1]) // out.stride(0) - 1)
        for r0 in range(0, R, ch):
            gemm_fused(Xc[r0:r0 + ch], Wc, out[r0:min(R, r0 + ch)], sincos=True)
        return out
    Z = gemm_prec(X, W, precision)
    if nat.is_device(X):
        if out is None:
            out = torch.empty((R + pad_rows, width), dtype=X.dtype, device=X.device)
        if pad_rows:
            out[R:].zero_()
        if width > P:
            out[:R, P:].zero_()
        Zc = Z.contiguous()
        nat.check(nat.hip_lib().pfml_rff_sincos(Zc.data_ptr(), R, half, out.data_ptr(),
                                                out.stride(0), nat.stream_of(X)),
                  "pfml_rff_sincos")
    else:
        if out is None:
            out = torch.zeros((R + pad_rows, width), dtype=X.dtype, device=X.device)
        else:
            out.zero_()
        out[:R, 0].fill_(1.0)
        out[:R, 1:P:2] = torch.cos(Z)
        out[:R, 2:P:2] = torch.sin(Z)
    return out


def standardize_signals(F: torch.Tensor, idx: torch.Tensor, mask: torch.Tensor,
                        vol: torch.Tensor, P: int | None = None, out: torch.Tensor | None = None,
                        n_real: torch.Tensor | None = None,
                        row_scale: torch.Tensor | None = None) -> torch.Tensor:
    """Gather + standardise the signal windows.

    F: [R+1, >= P] panel features (last row all zero, used for padding; P real columns),
    idx: [B, TH, N] rows, mask: [B, N] 1 for real stocks (real rows first), vol: [R+1].
    Returns [B, TH, N, Pw]: ``out`` may be a column block view of a wider buffer (e.g. one g's
    block of the [B, TH, N, G*Pw] S4 signal stack), columns P..Pw-1 come out zero.
    ``row_scale`` [B, N] (unit inner stride): every output row i of month b is multiplied by
    row_scale[b, i] afterwards (a separate rounding step: bitwise the standardised block times
    the scale) - the k-scale of the Horner step that reads the block."""
    B, TH, N = idx.shape
    P = P or F.shape[1]
    if out is None:
        out = torch.empty((B, TH, N, P), dtype=F.dtype, device=F.device)
    Pw = out.shape[-1]
    if nat.is_device(F):
        if out.stride(-1) != 1 or out.stride(1) != N * out.stride(2) or F.stride(-1) != 1:
            raise ValueError("standardize_signals: unsupported output layout")
        if n_real is None:
            n_real = mask.sum(1).to(torch.int32)
        n_real = n_real.to(torch.int32).contiguous()
        rows = idx.to(torch.int64).contiguous()
        _work.add("standardize", 6.0 * B * TH * N * P, 8.0 * B * TH * N * (P + Pw))
        if row_scale is not None and row_scale.stride(-1) != 1:
            raise ValueError("standardize_signals: row_scale needs unit inner stride")
        nat.check(nat.hip_lib().pfml_standardize(
            F.data_ptr(), P, F.stride(0), rows.data_ptr(), n_real.data_ptr(), B, TH, N,
            vol.data_ptr(), out.data_ptr(), out.stride(2), out.stride(1), Pw, None, 0, 1,
            nat.ptr(row_scale), 0 if row_scale is None else row_scale.stride(0),
            nat.stream_of(F)), "pfml_standardize")
        return out
    F = F[:, :P]
    S = F[idx]                                                  # [B, TH, N, P]
    m = mask.view(B, 1, N, 1)
    n = mask.sum(1).view(B, 1, 1, 1)
    mean = (S * m).sum(2, keepdim=True) / n
    mean[..., 0].fill_(0.0)                                     # constant is not demeaned
    S = (S - mean) * m
    norm = torch.sqrt(1.0 / (S * S).sum(2, keepdim=True))
    S = S * norm
    v = vol[idx].unsqueeze(-1)
    out.zero_()
    out[..., :P] = S / v
    if row_scale is not None:
        out.mul_(row_scale.view(B, 1, N, 1))
    return out


def signal_stats(F: torch.Tensor, idx: torch.Tensor, mask: torch.Tensor, P: int,
                 out: torch.Tensor, n_real: torch.Tensor | None = None) -> torch.Tensor:
    """The column means and scales of ``standardize_signals`` without the standardised values:
    out [B, TH, 2, >= Pw] (row 0 the means - 0 for the constant - row 1 the unit-norm scales;
    columns P.. zero), so that (F[idx] - mean) * scale / vol is formed where it is consumed
    (the Horner GEMM's gathered addend, models/pfml_inputs.py).  Same kernel, same sums."""
    B, TH, N = idx.shape
    Pw = out.shape[-1]
    if nat.is_device(F):
        if out.stride(-1) != 1 or out.stride(-2) != out.stride(1) // 2 or \
                out.stride(1) * TH != out.stride(0) or F.stride(-1) != 1:
            raise ValueError("signal_stats: unsupported output layout")
        if n_real is None:
            n_real = mask.sum(1).to(torch.int32)
        n_real = n_real.to(torch.int32).contiguous()
        rows = idx.to(torch.int64).contiguous()
        _work.add("standardize", 4.0 * B * TH * N * P, 8.0 * B * TH * N * P)
        nat.check(nat.hip_lib().pfml_standardize(
            F.data_ptr(), P, F.stride(0), rows.data_ptr(), n_real.data_ptr(), B, TH, N,
            F.data_ptr(), None, 0, 0, Pw, out.data_ptr(), out.stride(-2), 0, None, 0,
            nat.stream_of(F)), "pfml_standardize")
        return out
    S = F[:, :P][idx]                                           # [B, TH, N, P]
    m = mask.view(B, 1, N, 1)
    n = mask.sum(1).view(B, 1, 1, 1)
    mean = (S * m).sum(2, keepdim=True) / n
    mean[..., 0].fill_(0.0)
    S = (S - mean) * m
    norm = torch.sqrt(1.0 / (S * S).sum(2, keepdim=True))
    out.zero_()
    out[:, :, 0, :P] = mean[:, :, 0]
    out[:, :, 1, :P] = norm[:, :, 0]
    return out


def date_sums(F: torch.Tensor, urows: torch.Tensor, un: torch.Tensor, P: int, Pw: int,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """Per-date shifted column sums over the date's union universe U(d) (csrc/panel.hip
    date_sums_kernel): urows [nd, umax] panel rows (the first un[d] real), returns dsum
    [nd, 3, Pw] = (sum (x - K), sum (x - K)^2, K) with K the value of U(d)'s first row; the
    statistics of every (month, lag) reading date d follow by ``excl_stats``.  Device only."""
    nd, umax = urows.shape
    if out is None:
        out = torch.empty((nd, 3, Pw), dtype=F.dtype, device=F.device)
    if F.stride(-1) != 1 or not urows.is_contiguous() or not un.is_contiguous():
        raise ValueError("date_sums: unsupported layout")
    _work.add("date_sums", 3.0 * int(un.numel()) * umax * P, 8.0 * nd * umax * P)
    nat.check(nat.hip_lib().pfml_date_sums(F.data_ptr(), P, F.stride(0), urows.data_ptr(),
                                           un.data_ptr(), umax, nd, Pw, out.data_ptr(),
                                           nat.stream_of(F)), "pfml_date_sums")
    return out


def excl_stats(F: torch.Tensor, erows: torch.Tensor, en: torch.Tensor, dpos: torch.Tensor,
               dsum: torch.Tensor, n_real: torch.Tensor, P: int, out: torch.Tensor
               ) -> torch.Tensor:
    """``signal_stats`` of the [B, TH] (month, lag) tiles from their dates' union sums
    (``date_sums``) minus the rows of U(d) outside the month's universe: erows [B * TH, emax]
    (the first en[.] real), dpos [B * TH] date slot of each tile.  out as ``signal_stats``
    ([B, TH, 2, >= Pw] view).  Device only."""
    B, TH = out.shape[0], out.shape[1]
    Pw = dsum.shape[-1]
    emax = erows.shape[-1]
    if (out.stride(-1) != 1 or out.stride(-2) != out.stride(1) // 2 or
            out.stride(1) * TH != out.stride(0) or F.stride(-1) != 1):
        raise ValueError("excl_stats: unsupported output layout")
    _work.add("excl_stats", 3.0 * B * TH * emax * P, 8.0 * B * TH * emax * P)
    nat.check(nat.hip_lib().pfml_excl_stats(F.data_ptr(), P, F.stride(0), erows.data_ptr(),
                                            en.data_ptr(), emax, dpos.data_ptr(),
                                            dsum.data_ptr(), n_real.data_ptr(), B, TH, Pw,
                                            out.data_ptr(), out.stride(-2), nat.stream_of(F)),
              "pfml_excl_stats")
    return out
