"""Native columnar SQLite I/O (runtime/sqlite_io.cpp) == pandas read_sql_query / to_sql."""
import os
import sqlite3

import numpy as np
import pandas as pd
import pytest


def _frame(n=257, seed=0):
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({
        "id": np.arange(n, dtype=np.int64) + 10001,
        "eom": pd.date_range("1801-01-31", periods=n, freq="ME" if n < 2000 else "D").strftime("%Y-%m-%d"),
        "x": rng.normal(size=n),
        "y": np.where(rng.random(n) < 0.2, np.nan, rng.normal(size=n)),
        "whole": np.round(rng.normal(size=n) * 100),          # integral-valued floats
        "grp": np.where(rng.random(n) < 0.1, None, rng.choice(["mega", "small", "micro"], n)),
        "flag": rng.random(n) < 0.5,
        "nothing": [None] * n,
    })
    return df


@pytest.fixture
def native():
    from pfml.data import io
    if io._rt() is None or not hasattr(io._rt(), "pfml_sql_query"):
        pytest.skip("native runtime not built")
    return io


def test_native_read_equals_pandas(native, tmp_path, monkeypatch):
    db = str(tmp_path / "t.db")
    df = _frame()
    with sqlite3.connect(db) as con:
        df.to_sql("T", con, index=False)
        con.execute('CREATE TABLE U (a INTEGER, b REAL)')
        con.executemany("INSERT INTO U VALUES (?, ?)", [(1, 2.5), (None, None), (3, 4.0)])
    for q, pdt in (("SELECT * FROM T", ["eom"]), ("SELECT id, x, grp FROM T WHERE id > 10100", None),
                   ("SELECT * FROM U", None), ("SELECT * FROM T WHERE id < 0", None)):
        got = native.sql_read(db, q, **({"parse_dates": pdt} if pdt else {}))
        monkeypatch.setenv("PFML_SQL_NATIVE", "0")
        ref = native.sql_read(db, q, **({"parse_dates": pdt} if pdt else {}))
        monkeypatch.delenv("PFML_SQL_NATIVE")
        assert list(got.columns) == list(ref.columns)
        for c in ref.columns:
            if len(ref) == 0:
                continue
            assert got[c].dtype == ref[c].dtype, (q, c, got[c].dtype, ref[c].dtype)
        pd.testing.assert_frame_equal(got, ref, check_dtype=len(ref) > 0)


def test_native_write_roundtrip(native, tmp_path, monkeypatch):
    df = _frame(n=300, seed=1)
    df["when"] = pd.date_range("2001-01-31", periods=300, freq="ME")
    a, b = str(tmp_path / "a.db"), str(tmp_path / "b.db")
    native.sql_write(a, "T", df)                             # native
    native.sql_write(a, "T", df.iloc[:10], if_exists="append")
    monkeypatch.setenv("PFML_SQL_NATIVE", "0")
    native.sql_write(b, "T", df)                             # pandas
    native.sql_write(b, "T", df.iloc[:10], if_exists="append")
    ra, rb = native.sql_read(a, "SELECT * FROM T"), native.sql_read(b, "SELECT * FROM T")
    pd.testing.assert_frame_equal(ra, rb)
    with sqlite3.connect(a) as ca, sqlite3.connect(b) as cb:
        sa = ca.execute("PRAGMA table_info(T)").fetchall()
        sb = cb.execute("PRAGMA table_info(T)").fetchall()
    assert [(r[1], r[2]) for r in sa] == [(r[1], r[2]) for r in sb]


def test_native_parallel_scan_equals_pandas(native, tmp_path, monkeypatch):
    """A plain full-table scan above 64k rows is read in rowid ranges by several
    connections at once: same rows, same order, same dtypes as pandas (incl. deleted rowids)."""
    db = str(tmp_path / "big.db")
    df = _frame(n=90_001, seed=3)
    with sqlite3.connect(db) as con:
        df.to_sql("Big", con, index=False)
        con.execute("DELETE FROM Big WHERE id % 97 = 0")
    got = native.sql_read(db, "SELECT id, eom, x, y, grp, flag FROM Big", parse_dates=["eom"])
    monkeypatch.setenv("PFML_SQL_NATIVE", "0")
    ref = native.sql_read(db, "SELECT id, eom, x, y, grp, flag FROM Big", parse_dates=["eom"])
    pd.testing.assert_frame_equal(got, ref)


def test_native_aggregates_and_distinct_on_big_table(native, tmp_path, monkeypatch):
    """Queries over a > 64k-row table that are NOT plain column scans (DISTINCT, aggregates,
    expressions) run on one connection: one result, as pandas gives it."""
    db = str(tmp_path / "agg.db")
    df = _frame(n=70_001, seed=4)
    with sqlite3.connect(db) as con:
        df.to_sql("Big", con, index=False)
    for q in ("SELECT DISTINCT grp FROM Big", "SELECT count(*) FROM Big",
              "SELECT max(eom) FROM Big", "SELECT id + 1 AS k FROM Big",
              'SELECT "id", x FROM Big'):
        got = native.sql_read(db, q)
        monkeypatch.setenv("PFML_SQL_NATIVE", "0")
        ref = native.sql_read(db, q)
        monkeypatch.delenv("PFML_SQL_NATIVE")
        if "DISTINCT" in q:
            got = got.sort_values("grp", na_position="first").reset_index(drop=True)
            ref = ref.sort_values("grp", na_position="first").reset_index(drop=True)
        pd.testing.assert_frame_equal(got, ref, check_dtype=False)
        assert len(got) == len(ref), q
