"""L0 data acquisition: excess-return ETL and the S&P 500 subset.

* ``get_additional_data``  - 0_Get_Additional_Data.py: daily CRSP returns + FF daily RF ->
  ``crsp_daily.db:d_ret_ex`` (permno, date, ret, primaryexch, ret_excess; float32 returns),
  processed in 5-year chunks.  The WRDS download itself (PostgreSQL, :30-79) needs network
  access and credentials; ``download_wrds`` documents the query and refuses offline.
* ``sp500_subset``         - 0_SP500_Subset.py: inner joins of the JKP ``Factors`` table and
  the daily returns with the historical constituents on (permno, eom).  The reference writes
  ``JKP_SP500.db`` / ``db_crsp_daily_SP500.db`` with table ``Factors`` while the later stages
  read ``JKP_US_SP500.db`` / ``crsp_daily_SP500.db:d_ret_ex`` (quirk Q11, a manual rename in
  the reference); this step writes the names the later stages read.
Both are idempotent (tables are replaced, not appended to).
"""
from __future__ import annotations

import os
import sqlite3

import numpy as np
import pandas as pd

from ..config import Config
from ..utils.log import get_logger
from . import io

log = get_logger("acquire")

WRDS_QUERY = (
    "SELECT dsf.permno, dsf.dlycaldt AS date, dsf.dlyret AS ret, dsf.primaryexch "
    "FROM crsp.dsf_v2 AS dsf WHERE dsf.dlycaldt BETWEEN '{start}' AND '{end}' "
    "AND sharetype = 'NS' AND securitytype = 'EQTY' AND securitysubtype = 'COM' "
    "AND usincflg = 'Y' AND issuertype in ('ACOR', 'CORP') AND primaryexch in ('N', 'A', 'Q') "
    "AND conditionaltype in ('RW', 'NW') AND tradingstatusflg = 'A'")


def download_wrds(*_a, **_k):
    raise RuntimeError("WRDS download needs network access and credentials (not available); "
                       "place crsp_daily.db:crsp_daily in the data directory instead. Query:\n"
                       + WRDS_QUERY)


def _chunks(start: pd.Timestamp, end: pd.Timestamp, years: int = 5):
    cur = start
    while cur < end:
        nxt = min(cur + pd.DateOffset(years=years), end)
        yield cur, nxt
        cur = nxt + pd.Timedelta(days=1)


def get_additional_data(cfg: Config, start="1952-01-01", end="2024-12-31") -> int:
    dd = cfg.run.data_dir
    rf = pd.read_csv(io.path(dd, "FF_RF_daily.csv"))[["date", "RF"]]
    rf["date"] = pd.to_datetime(rf["date"].astype(str), format="%Y%m%d")
    rf = rf[rf["date"] > "1951-12-31"]
    rf["RF"] = rf["RF"] / 100.0
    db = io.path(dd, "crsp_daily.db")
    n = 0
    with sqlite3.connect(db) as con:
        con.execute("DROP TABLE IF EXISTS crsp_daily_excess")
    # chunked as the reference (bounded memory); reads and appends through the columnar
    # SQLite I/O (data/io.py, runtime/sqlite_io.cpp)
    for a, b in _chunks(pd.Timestamp(start), pd.Timestamp(end)):
        log.info(f"Processing chunk: {a.date()} to {b.date()}")
        ch = io.sql_read(db, f"SELECT * FROM crsp_daily WHERE date BETWEEN '{a.date()}' AND "
                             f"'{b.date()}'", parse_dates=["date"]).dropna()
        if ch.empty:
            continue
        ch["ret"] = pd.to_numeric(ch["ret"], errors="coerce")
        ch = ch.dropna(subset=["ret"]).merge(rf, on="date", how="left").dropna(subset=["RF"])
        ch["permno"] = ch["permno"].astype(np.int64)
        ch["ret_excess"] = (ch["ret"] - ch["RF"]).astype(np.float32)
        ch["ret"] = ch["ret"].astype(np.float32)
        ch["date"] = ch["date"].dt.strftime("%Y-%m-%d")
        io.sql_write(db, "crsp_daily_excess",
                     ch[["permno", "date", "ret", "primaryexch", "ret_excess"]], if_exists="append")
        n += len(ch)
    with sqlite3.connect(db) as con:
        con.execute("DROP TABLE IF EXISTS d_ret_ex")
        con.execute("ALTER TABLE crsp_daily_excess RENAME TO d_ret_ex")
    log.info("Processing complete.")
    return n


def sp500_subset(cfg: Config, start="1952-01-01", end="2024-12-31") -> dict:
    dd = cfg.run.data_dir
    cons = pd.read_csv(io.path(dd, "SP500_Historical_Constituents.csv"),
                       parse_dates=["start", "ending", "date"])
    cons = cons.drop(columns=[c for c in cons.columns if c.startswith("Unnamed")])
    cons["eom"] = cons["date"] + pd.offsets.MonthEnd(0)
    outs = {"factors": io.path(dd, "JKP_US_SP500.db"), "daily": io.path(dd, "crsp_daily_SP500.db")}
    counts = {"factors": 0, "daily": 0}
    for p in outs.values():
        if os.path.exists(p):
            with sqlite3.connect(p) as con:
                con.execute("DROP TABLE IF EXISTS Factors")
                con.execute("DROP TABLE IF EXISTS d_ret_ex")
    src = io.path(dd, "JKP_US.db")
    for a, b in _chunks(pd.Timestamp(start), pd.Timestamp(end)):
        ch = io.sql_read(src, f"SELECT * FROM Factors WHERE eom BETWEEN '{a.date()}' AND "
                              f"'{b.date()}'", parse_dates=["eom"])
        if ch.empty:
            continue
        sub = cons[["permno", "eom"]].merge(ch, left_on=["permno", "eom"],
                                            right_on=["id", "eom"], how="inner")
        sub = sub.drop(columns=["permno"])
        sub["eom"] = sub["eom"].dt.strftime("%Y-%m-%d")
        io.sql_write(outs["factors"], "Factors", sub, if_exists="append")
        counts["factors"] += len(sub)
    log.info("Processing JKP_SP500 complete.")
    src = io.path(dd, "crsp_daily.db")
    for a, b in _chunks(pd.Timestamp(start), pd.Timestamp(end)):
        ch = io.sql_read(src, f"SELECT * FROM d_ret_ex WHERE date BETWEEN '{a.date()}' AND "
                              f"'{b.date()}'", parse_dates=["date"])
        if ch.empty:
            continue
        ch["eom"] = ch["date"] + pd.offsets.MonthEnd(0)
        sub = cons[["permno", "eom"]].merge(ch, on=["eom", "permno"], how="inner")
        sub = sub.drop(columns=["eom"])
        sub["date"] = sub["date"].dt.strftime("%Y-%m-%d")
        io.sql_write(outs["daily"], "d_ret_ex", sub, if_exists="append")
        counts["daily"] += len(sub)
    log.info("Processing crsp_daily_SP500 complete.")
    return counts
