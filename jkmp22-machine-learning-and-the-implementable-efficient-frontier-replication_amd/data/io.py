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


def read_risk_free(data_dir: str) -> pd.DataFrame:
    """FF monthly RF (percent) -> [eom, rf] (Prepare_Data.py:62-71)."""
    rf = pd.read_csv(path(data_dir, "FF_RF_monthly.csv"), usecols=["yyyymm", "RF"])
    eom = pd.to_datetime(rf["yyyymm"].astype(str) + "01", format="%Y%m%d") + pd.offsets.MonthEnd(0)
    return pd.DataFrame({"eom": eom, "rf": rf["RF"] / 100.0})


def read_market(data_dir: str) -> pd.DataFrame:
    """US value-weighted market excess return -> [eom_ret, mkt_vw_exc] (Prepare_Data.py:82-89)."""
    m = pd.read_csv(path(data_dir, "market_returns.csv"), dtype={"eom": str})
    m = m[m["excntry"] == "USA"]
    return pd.DataFrame({"eom_ret": pd.to_datetime(m["eom"], format="%Y-%m-%d").values,
                         "mkt_vw_exc": m["mkt_vw_exc"].values})


def read_factor_details(data_dir: str) -> pd.DataFrame:
    x = path(data_dir, "Factor Details.xlsx")
    if os.path.exists(x):
        try:
            return pd.read_excel(x)
        except ImportError:
            pass
    return pd.read_csv(path(data_dir, "Factor Details.csv"))


def read_rff_w(data_dir: str) -> np.ndarray:
    """RFF weight matrix, k x p_max/2, stored with an unnamed index column."""
    w = pd.read_csv(path(data_dir, "rff_w.csv"))
    if "Unnamed: 0" in w.columns:
        w = w.drop(columns="Unnamed: 0")
    return w.to_numpy(dtype=np.float64)


def sql_read(db: str, query: str, **kw) -> pd.DataFrame:
    with sqlite3.connect(db) as con:
        return pd.read_sql_query(query, con, **kw)


def sql_write(db: str, table: str, df: pd.DataFrame, if_exists: str = "replace") -> None:
    with sqlite3.connect(db) as con:
        df.to_sql(table, con, if_exists=if_exists, index=False, chunksize=200_000)


PROCESSED_COLUMNS = ["id", "eom", "sic", "ff49", "size_grp", "me", "crsp_exchcd", "dolvol",
                     "lambda", "rvol_m", "tr_ld0", "eom_ret", "ret_ld1", "tr_ld1", "mu_ld0",
                     "ff12", "valid"]


def read_processed_chars(data_dir: str, features: list[str]) -> pd.DataFrame:
    """Factors_processed as loaded by the later stages (e.g. PFML_Input_Data.py:53-79)."""
    q = "SELECT " + ", ".join(PROCESSED_COLUMNS + features) + " FROM Factors_processed"
    chars = sql_read(path(data_dir, "JKP_US_SP500.db"), q, parse_dates=["eom", "eom_ret"])
    chars["valid"] = chars["valid"].astype(bool)
    return chars


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
