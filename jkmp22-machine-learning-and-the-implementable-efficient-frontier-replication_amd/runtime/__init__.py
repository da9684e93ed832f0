"""Python face of the host C++ runtime (``runtime/panel.cpp`` -> ``lib/libpfml_rt.so``).

Group-wise sequential kernels over panels sorted by (group, time): universe state machine,
rolling sums, percentile ranks, EWMA volatility, group shifts.  Inputs are numpy arrays;
``groups`` is a CSR array of group starts (length ngroups + 1).
"""
from __future__ import annotations

import ctypes as C

import numpy as np


def declare(lib) -> None:
    P, L, I, D = C.c_void_p, C.c_int64, C.c_int, C.c_double
    lib.pfml_investment_universe.argtypes = [P, P, P, L, P]
    lib.pfml_investment_universe.restype = None
    lib.pfml_rolling_sum.argtypes = [P, P, L, I, P]
    lib.pfml_rolling_sum.restype = None
    lib.pfml_pct_rank.argtypes = [P, L, L, P, L, P]
    lib.pfml_pct_rank.restype = None
    lib.pfml_pct_rank_rows.argtypes = [P, L, L, L, L, P, P, L, I, D, P, L, L]
    lib.pfml_pct_rank_rows.restype = None
    lib.pfml_ewma_vol.argtypes = [P, P, L, D, I, P]
    lib.pfml_ewma_vol.restype = None
    lib.pfml_group_starts.argtypes = [P, L, P]
    lib.pfml_group_starts.restype = L
    lib.pfml_group_shift.argtypes = [P, P, L, L, P]
    lib.pfml_group_shift.restype = None
    # runtime/sqlite_io.cpp (columnar SQLite I/O)
    lib.pfml_sql_query.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_longlong),
                                   C.POINTER(C.c_int), C.c_char_p, I]
    lib.pfml_sql_query.restype = P
    lib.pfml_sql_col_name.argtypes = [P, I]
    lib.pfml_sql_col_name.restype = C.c_char_p
    lib.pfml_sql_col_kind.argtypes = [P, I]
    lib.pfml_sql_col_kind.restype = I
    lib.pfml_sql_col_f64.argtypes = [P, I, P]
    lib.pfml_sql_col_f64.restype = None
    lib.pfml_sql_col_i64.argtypes = [P, I, P]
    lib.pfml_sql_col_i64.restype = None
    lib.pfml_sql_col_text_bytes.argtypes = [P, I]
    lib.pfml_sql_col_text_bytes.restype = C.c_longlong
    lib.pfml_sql_col_text.argtypes = [P, I, P, P, P]
    lib.pfml_sql_col_text.restype = None
    lib.pfml_sql_free.argtypes = [P]
    lib.pfml_sql_free.restype = None
    lib.pfml_sql_write.argtypes = [C.c_char_p, C.c_char_p, I, I, P, P, P, P, P, P, C.c_longlong,
                                   C.c_char_p, I]
    lib.pfml_sql_write.restype = I


def _lib():
    from ..ops._native import rt_lib
    return rt_lib()


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def group_starts(key: np.ndarray) -> np.ndarray:
    key = _c(key, np.int64)
    gs = np.empty(len(key) + 1, dtype=np.int64)
    ng = _lib().pfml_group_starts(key.ctypes.data, len(key), gs.ctypes.data)
    return gs[: ng + 1].copy()


def investment_universe(add, delete, groups) -> np.ndarray:
    add, delete = _c(add, np.uint8), _c(delete, np.uint8)
    groups = _c(groups, np.int64)
    out = np.empty(len(add), dtype=np.uint8)
    _lib().pfml_investment_universe(add.ctypes.data, delete.ctypes.data, groups.ctypes.data,
                                    len(groups) - 1, out.ctypes.data)
    return out.astype(bool)


def rolling_sum(x, groups, window: int) -> np.ndarray:
    x = _c(x, np.float64)
    groups = _c(groups, np.int64)
    out = np.empty(len(x), dtype=np.float64)
    _lib().pfml_rolling_sum(x.ctypes.data, groups.ctypes.data, len(groups) - 1, int(window),
                            out.ctypes.data)
    return out


def pct_rank(x: np.ndarray, segments) -> np.ndarray:
    """x: [nrows] or [nrows, ncol] (rows sorted by segment) -> pct ranks, NaN preserved."""
    squeeze = x.ndim == 1
    X = x.reshape(len(x), -1)
    Xc = np.asfortranarray(X, dtype=np.float64)          # column-major for the kernel
    out = np.empty_like(Xc, order="F")
    seg = _c(segments, np.int64)
    _lib().pfml_pct_rank(Xc.ctypes.data, Xc.shape[0], Xc.shape[1], seg.ctypes.data,
                         len(seg) - 1, out.ctypes.data)
    return out[:, 0].copy() if squeeze else np.ascontiguousarray(out)


def pct_rank_rows(X: np.ndarray, perm, segments, zero_keep: bool = False,
                  impute: float | None = None) -> np.ndarray:
    """Percentile ranks of the row-major panel X [nrows, ncol] within the segments of the row
    permutation ``perm`` (segment s = rows perm[segments[s]:segments[s + 1]]), written in X's
    own row order; NaN preserved (or set to ``impute``), exact zeros ranked 0 with
    ``zero_keep``."""
    Xc = np.asarray(X, dtype=np.float64)
    if Xc.ndim != 2 or not (Xc.flags.c_contiguous or Xc.flags.f_contiguous):
        Xc = np.ascontiguousarray(Xc)
    pm = _c(perm, np.int64)
    seg = _c(segments, np.int64)
    out = np.empty_like(Xc)                  # same layout as X (C or Fortran order): no copies
    xs = [st // 8 for st in Xc.strides]
    os_ = [st // 8 for st in out.strides]
    _lib().pfml_pct_rank_rows(Xc.ctypes.data, Xc.shape[0], Xc.shape[1], xs[0], xs[1],
                              pm.ctypes.data, seg.ctypes.data, len(seg) - 1, int(zero_keep),
                              float("nan") if impute is None else float(impute), out.ctypes.data,
                              os_[0], os_[1])
    return out


def ewma_vol(x, groups, lam: float, start: int) -> np.ndarray:
    x = _c(x, np.float64)
    groups = _c(groups, np.int64)
    out = np.empty(len(x), dtype=np.float64)
    _lib().pfml_ewma_vol(x.ctypes.data, groups.ctypes.data, len(groups) - 1, float(lam),
                         int(start), out.ctypes.data)
    return out


def group_shift(x, groups, k: int) -> np.ndarray:
    x = _c(x, np.float64)
    groups = _c(groups, np.int64)
    out = np.empty(len(x), dtype=np.float64)
    _lib().pfml_group_shift(x.ctypes.data, groups.ctypes.data, len(groups) - 1, int(k),
                            out.ctypes.data)
    return out
