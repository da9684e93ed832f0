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


def _between(a: pd.Timestamp, b: pd.Timestamp, compat: bool) -> str:
    """The chunk filter of the reference's chunked reads.  compat: its literal
    ``BETWEEN 'a' AND 'b'`` - on dates stored as pandas' TIMESTAMP text ('YYYY-MM-DD
    00:00:00', which sorts after 'YYYY-MM-DD') the rows of each chunk's END day match neither
    that chunk nor the next, so the reference loses them (quirk Q19); corrected: the end day
    taken whole."""
    if compat:
        return f"BETWEEN '{a.date()}' AND '{b.date()}'"
    return f"BETWEEN '{a.date()}' AND '{b.date()} 23:59:59'"


def get_additional_data(cfg: Config, start="1952-01-01", end="2024-12-31") -> int:
    """0_Get_Additional_Data.py:82-163: crsp_daily + FF daily RF -> d_ret_ex (permno, date,
    ret, primaryexch, ret_excess; float32 returns), in the reference's 5-year chunks.  The
    raw ``crsp_daily`` table is kept (the reference drops it, :155-157, so it cannot be re-run;
    this stage is idempotent - quirk Q20).  compat: dates written as pandas writes the
    reference's datetime column (TIMESTAMP text), so the S&P 500 subset's chunked reads see
    what the reference's see (Q19); corrected: date-only text."""
    dd = cfg.run.data_dir
    compat = bool(cfg.run.compat_mode)
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
        ch = io.sql_read(db, f"SELECT * FROM crsp_daily WHERE date {_between(a, b, compat)}",
                         parse_dates=["date"]).dropna()
        if ch.empty:
            continue
        ch["ret"] = pd.to_numeric(ch["ret"], errors="coerce")
        ch = ch.dropna(subset=["ret"]).merge(rf, on="date", how="left").dropna(subset=["RF"])
        ch["permno"] = ch["permno"].astype(np.int64)
        ch["ret_excess"] = (ch["ret"] - ch["RF"]).astype(np.float32)
        ch["ret"] = ch["ret"].astype(np.float32)
        if not compat:
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
    """0_SP500_Subset.py: inner joins of the JKP Factors table (chunks filtered on its `date`,
    :52-55) and of the daily excess returns with the historical constituents on (permno, eom),
    with the reference's columns: the constituents' permno kept, their start / ending / date
    dropped (`_drop` suffixes, :59-64, :111-112).  Written under the names the later stages
    read (Q11): JKP_US_SP500.db:Factors and crsp_daily_SP500.db:d_ret_ex."""
    dd = cfg.run.data_dir
    compat = bool(cfg.run.compat_mode)
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
    with sqlite3.connect(src) as con:
        jcols = [r[1] for r in con.execute("PRAGMA table_info(Factors)")]
    dcol = "date" if "date" in jcols else "eom"          # (a JKP extract without `date`)
    jdates = ["eom", "date"] if "date" in jcols else ["eom"]
    for a, b in _chunks(pd.Timestamp(start), pd.Timestamp(end)):
        ch = io.sql_read(src, f"SELECT * FROM Factors WHERE {dcol} {_between(a, b, compat)}",
                         parse_dates=jdates)
        if ch.empty:
            continue
        sub = cons.merge(ch, left_on=["permno", "eom"], right_on=["id", "eom"],
                         suffixes=("_drop", ""), how="inner")
        sub = sub.drop(columns=[c for c in sub.columns if c.endswith("_drop")] +
                       ["start", "ending"])
        io.sql_write(outs["factors"], "Factors", sub, if_exists="append")
        counts["factors"] += len(sub)
    log.info("Processing JKP_SP500 complete.")
    src = io.path(dd, "crsp_daily.db")
    for a, b in _chunks(pd.Timestamp(start), pd.Timestamp(end)):
        ch = io.sql_read(src, f"SELECT * FROM d_ret_ex WHERE date {_between(a, b, compat)}",
                         parse_dates=["date"])
        if ch.empty:
            continue
        ch["eom"] = ch["date"] + pd.offsets.MonthEnd(0)
        sub = cons.merge(ch, on=["eom", "permno"], how="inner", suffixes=("_drop", ""))
        sub = sub.drop(columns=["start", "ending", "date_drop", "eom"])
        if not compat:
            sub["date"] = sub["date"].dt.strftime("%Y-%m-%d")
        io.sql_write(outs["daily"], "d_ret_ex", sub, if_exists="append")
        counts["daily"] += len(sub)
    log.info("Processing crsp_daily_SP500 complete.")
    return counts
