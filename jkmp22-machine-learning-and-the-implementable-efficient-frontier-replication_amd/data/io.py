"""Schema-faithful readers/writers for the reference's on-disk inputs and outputs.

Readers accept exactly the files the reference reads; the parity CSV writers
emit exactly the reference's column order.  ``Factor Details.xlsx`` is read when
an xlsx engine is importable, otherwise the CSV twin ``Factor Details.csv`` is used.
"""
from __future__ import annotations

import os
import sqlite3

import numpy as np
import pandas as pd

CSV_COLUMNS = {
    "wealth_processed.csv": ["eom", "wealth", "mu_ld1"],
    "cluster_labels_processed.csv": ["characteristic", "direction", "cluster"],
    "validation.csv": ["eom", "eom_ret", "obj", "l", "p", "hp_end", "cum_obj", "rank", "g"],
    "weights.csv": ["eom", "mu_ld1", "id", "tr_ld1", "w_start", "w"],
    "pf.csv": ["inv", "shorting", "turnover", "r", "tc", "eom_ret"],
    "pf_summary.csv": ["type", "n", "inv", "shorting", "turnover_notional", "r", "sd",
                       "sr_gross", "tc", "r_tc", "sr", "obj"],
}


def path(data_dir: str, name: str) -> str:
    return os.path.join(data_dir, name)


# wall seconds spent in this module's file I/O (SQLite, CSV); the stage runner reports the
# per-stage delta next to the stage time (pipeline.run -> metrics "io_seconds")
IO_SECONDS = [0.0]


def _io_timed(fn):
    import functools
    import time

    @functools.wraps(fn)
    def wrap(*a, **k):
        depth = _io_timed.depth
        _io_timed.depth += 1
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            _io_timed.depth -= 1
            if depth == 0:                       # outermost I/O call only
                IO_SECONDS[0] += time.perf_counter() - t0
    return wrap


_io_timed.depth = 0


@_io_timed
def read_risk_free(data_dir: str) -> pd.DataFrame:
    """FF monthly RF (percent) -> [eom, rf] (Prepare_Data.py:62-71)."""
    rf = pd.read_csv(path(data_dir, "FF_RF_monthly.csv"), usecols=["yyyymm", "RF"])
    eom = pd.to_datetime(rf["yyyymm"].astype(str) + "01", format="%Y%m%d") + pd.offsets.MonthEnd(0)
    return pd.DataFrame({"eom": eom, "rf": rf["RF"] / 100.0})


@_io_timed
def read_market(data_dir: str) -> pd.DataFrame:
    """US value-weighted market excess return -> [eom_ret, mkt_vw_exc] (Prepare_Data.py:82-89)."""
    m = pd.read_csv(path(data_dir, "market_returns.csv"), dtype={"eom": str})
    m = m[m["excntry"] == "USA"]
    return pd.DataFrame({"eom_ret": pd.to_datetime(m["eom"], format="%Y-%m-%d").values,
                         "mkt_vw_exc": m["mkt_vw_exc"].values})


@_io_timed
def read_factor_details(data_dir: str) -> pd.DataFrame:
    x = path(data_dir, "Factor Details.xlsx")
    if os.path.exists(x):
        try:
            return pd.read_excel(x)
        except ImportError:
            pass
    return pd.read_csv(path(data_dir, "Factor Details.csv"))


@_io_timed
def read_rff_w(data_dir: str) -> np.ndarray:
    """RFF weight matrix, k x p_max/2, stored with an unnamed index column."""
    w = pd.read_csv(path(data_dir, "rff_w.csv"))
    if "Unnamed: 0" in w.columns:
        w = w.drop(columns="Unnamed: 0")
    return w.to_numpy(dtype=np.float64)


def _rt():
    try:
        from ..ops._native import rt_lib
        return rt_lib()
    except Exception:                      # noqa: BLE001 - no native runtime: pandas path
        return None


def _native_read(db: str, query: str, parse_dates) -> pd.DataFrame | None:
    """Columnar read through runtime/sqlite_io.cpp: the query stepped once in C++, each
    column returned as one typed buffer.  The DataFrame equals pandas.read_sql_query's: int64
    for integer-only columns, float64 (NaN for NULL) for numeric ones, object strings (None
    for NULL) for text, datetime64 for ``parse_dates``.  None (-> pandas) when the library
    is missing or a column mixes text and numbers."""
    import ctypes as C
    lib = _rt()
    if lib is None or not hasattr(lib, "pfml_sql_query"):
        return None
    nrow, ncol = C.c_longlong(0), C.c_int(0)
    err = C.create_string_buffer(512)
    h = lib.pfml_sql_query(db.encode(), query.encode(), C.byref(nrow), C.byref(ncol), err, 512)
    if not h:
        raise RuntimeError(f"sqlite read failed: {err.value.decode(errors='replace')}")
    try:
        n = int(nrow.value)
        kinds = [lib.pfml_sql_col_kind(h, c) for c in range(ncol.value)]
        if any(k < 0 for k in kinds):
            return None
        names = [lib.pfml_sql_col_name(h, c).decode() for c in range(ncol.value)]
        # the float64 columns land in the rows of ONE [nf, n] array, which becomes the frame's
        # single float block without a copy (a dict of columns gives one block per column:
        # a "highly fragmented" frame whose every take / filter pays per column)
        fcols = [c for c, k in enumerate(kinds) if k == 2]
        F = np.empty((len(fcols), n), dtype=np.float64)
        for j, c in enumerate(fcols):
            lib.pfml_sql_col_f64(h, c, F[j].ctypes.data)
        cols = {}
        for c, k in enumerate(kinds):
            name = names[c]
            if k == 2:
                continue
            if k == 1:
                a = np.empty(n, dtype=np.int64)
                lib.pfml_sql_col_i64(h, c, a.ctypes.data)
            elif k == 3:
                nb = int(lib.pfml_sql_col_text_bytes(h, c))
                buf = np.empty(max(nb, 1), dtype=np.uint8)
                off = np.empty(n + 1, dtype=np.int64)
                nul = np.empty(max(n, 1), dtype=np.uint8)
                lib.pfml_sql_col_text(h, c, buf.ctypes.data, off.ctypes.data, nul.ctypes.data)
                raw = buf.tobytes()
                a = np.array([None if nul[i] else raw[off[i]:off[i + 1]].decode()
                              for i in range(n)], dtype=object)
            else:
                a = np.full(n, None, dtype=object)
            cols[name] = a
    finally:
        lib.pfml_sql_free(h)
    df = pd.DataFrame(F.T, columns=[names[c] for c in fcols], copy=False)
    import warnings
    with warnings.catch_warnings():                    # (blocks merged once, below)
        warnings.simplefilter("ignore", pd.errors.PerformanceWarning)
        for c, name in enumerate(names):               # the other columns at their positions
            if kinds[c] != 2:
                df.insert(c, name, cols[name])
    if len(names) - len(fcols) > 16:
        # many int / text columns: merge their one-column blocks (the float block is alone
        # in its dtype and stays as it is)
        df._consolidate_inplace()
    for c in (parse_dates or ()):
        if c in df.columns:
            df[c] = pd.to_datetime(df[c])
    return df


@_io_timed
def sql_read(db: str, query: str, **kw) -> pd.DataFrame:
    """pandas.read_sql_query semantics; the columnar native reader when available (about 20x
    faster on the 430k x 130 Factors tables), pandas otherwise / for other keywords."""
    if set(kw) <= {"parse_dates"} and os.environ.get("PFML_SQL_NATIVE", "1") != "0":
        if not os.path.exists(db):
            raise FileNotFoundError(db)
        df = _native_read(db, query, kw.get("parse_dates"))
        if df is not None:
            return df
    with sqlite3.connect(db) as con:
        return pd.read_sql_query(query, con, **kw)


def _native_write(db: str, table: str, df: pd.DataFrame, if_exists: str) -> bool:
    """DataFrame.to_sql(index=False) through runtime/sqlite_io.cpp (pandas' SQLite column
    types; datetimes as pandas writes them, 'YYYY-MM-DD HH:MM:SS' TIMESTAMP text)."""
    import ctypes as C
    lib = _rt()
    if lib is None or not hasattr(lib, "pfml_sql_write") or if_exists not in ("replace", "append"):
        return False
    n, nc = len(df), df.shape[1]
    names, decls, kinds, keep = [], [], [], []
    datas, offs, nulls = [], [], []
    for name in df.columns:
        s = df[name]
        dt = s.dtype
        if pd.api.types.is_bool_dtype(dt):
            a = np.ascontiguousarray(s.to_numpy(np.int64))
            kinds.append(4), decls.append("INTEGER")
            datas.append(a), offs.append(None), nulls.append(None)
        elif pd.api.types.is_integer_dtype(dt):
            a = np.ascontiguousarray(s.to_numpy(np.int64))
            kinds.append(1), decls.append("INTEGER")
            datas.append(a), offs.append(None), nulls.append(None)
        elif pd.api.types.is_float_dtype(dt):
            a = np.ascontiguousarray(s.to_numpy(np.float64))
            kinds.append(2), decls.append("REAL")
            datas.append(a), offs.append(None), nulls.append(None)
        else:
            if pd.api.types.is_datetime64_any_dtype(dt):
                decls.append("TIMESTAMP")
                v = s.dt.strftime("%Y-%m-%d %H:%M:%S").to_numpy(object)
            elif dt == object or pd.api.types.is_string_dtype(dt):
                vals = s.to_numpy(object)
                if any(x is not None and not isinstance(x, str) and not
                       (isinstance(x, float) and np.isnan(x)) for x in vals[: min(n, 1000)]):
                    return False                      # non-string objects: leave to pandas
                decls.append("TEXT")
                v = vals
            else:
                return False
            isnul = np.array([x is None or (isinstance(x, float) and np.isnan(x)) for x in v],
                             dtype=np.uint8)
            enc = [b"" if isnul[i] else str(v[i]).encode() for i in range(n)]
            o = np.zeros(n + 1, dtype=np.int64)
            if n:
                o[1:] = np.cumsum([len(e) for e in enc])
            buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
            kinds.append(3)
            datas.append(buf), offs.append(o), nulls.append(isnul)
        names.append(str(name).encode())
        keep.append(datas[-1])
    P = C.c_void_p
    arr_names = (C.c_char_p * nc)(*names)
    arr_decl = (C.c_char_p * nc)(*[d.encode() for d in decls])
    arr_kind = (C.c_int * nc)(*kinds)
    arr_data = (P * nc)(*[d.ctypes.data for d in datas])
    arr_off = (P * nc)(*[(o.ctypes.data if o is not None else None) for o in offs])
    arr_nul = (P * nc)(*[(u.ctypes.data if u is not None else None) for u in nulls])
    err = C.create_string_buffer(512)
    rc = lib.pfml_sql_write(db.encode(), table.encode(), 1 if if_exists == "replace" else 0, nc,
                            C.cast(arr_names, P), C.cast(arr_decl, P), C.cast(arr_kind, P),
                            C.cast(arr_data, P), C.cast(arr_off, P), C.cast(arr_nul, P), n, err,
                            512)
    if rc != 0:
        raise RuntimeError(f"sqlite write failed: {err.value.decode(errors='replace')}")
    return True


@_io_timed
def sql_write(db: str, table: str, df: pd.DataFrame, if_exists: str = "replace") -> None:
    """DataFrame.to_sql(index=False) semantics; the native column writer when available."""
    if os.environ.get("PFML_SQL_NATIVE", "1") != "0" and _native_write(db, table, df, if_exists):
        return
    with sqlite3.connect(db) as con:
        df.to_sql(table, con, if_exists=if_exists, index=False, chunksize=200_000)


PROCESSED_COLUMNS = ["id", "eom", "sic", "ff49", "size_grp", "me", "crsp_exchcd", "dolvol",
                     "lambda", "rvol_m", "tr_ld0", "eom_ret", "ret_ld1", "tr_ld1", "mu_ld0",
                     "ff12", "valid"]


@_io_timed
def read_processed_chars(data_dir: str, features: list[str]) -> pd.DataFrame:
    """Factors_processed as loaded by the later stages (e.g. PFML_Input_Data.py:53-79)."""
    q = "SELECT " + ", ".join(PROCESSED_COLUMNS + features) + " FROM Factors_processed"
    chars = sql_read(path(data_dir, "JKP_US_SP500.db"), q, parse_dates=["eom", "eom_ret"])
    chars["valid"] = chars["valid"].astype(bool)
    return chars


@_io_timed
def write_csv(df: pd.DataFrame, data_dir: str, name: str) -> str:
    cols = CSV_COLUMNS.get(name)
    if cols is not None:
        missing = [c for c in cols if c not in df.columns]
        if missing:
            raise ValueError(f"{name}: missing columns {missing}")
        df = df[cols]
    os.makedirs(data_dir, exist_ok=True)
    p = path(data_dir, name)
    df.to_csv(p, index=False)
    return p
