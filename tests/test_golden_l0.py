"""L0 parity against the reference's own 0_Get_Additional_Data.py and 0_SP500_Subset.py.

tests/golden/ref_l0/l0_golden.json was frozen by tools/make_golden_l0.py (a manual dev-time
tool that exec()s the two reference scripts on the synthetic ``l0_spec`` raw files; nothing
from the reference runs here).  This test regenerates the same raw files, runs the engine's
L0 stages in compat mode and compares every output table value for value: the column list,
the row count and an md5 per column in table order (REAL as float64 bytes) - i.e. bitwise the
reference's tables, including its quirks:

* Q19: the reference's chunked ``BETWEEN`` reads compare pandas' TIMESTAMP text
  ('YYYY-MM-DD 00:00:00') with date-only bounds, so every 5-year chunk's end day is lost
  (1962-01-02, 1967-01-03, ... 2022-01-14, 2024-12-31);
* the subset Factors table keeps the constituents' ``permno`` and is filtered on JKP's
  ``date`` (0_SP500_Subset.py:52-64).

Deviations by design: Q11 (output databases / tables under the names the later stages read:
JKP_US_SP500.db:Factors, crsp_daily_SP500.db:d_ret_ex) and Q20 (the raw crsp_daily table is
kept, so the stage can be re-run; the reference drops it, 0_Get_Additional_Data.py:155-157).
"""
import hashlib
import json
import os
import sqlite3

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_l0",
                    "l0_golden.json")


def table_fingerprint(db: str, table: str) -> dict:
    with sqlite3.connect(db) as con:
        cols = [r[1] for r in con.execute(f"PRAGMA table_info({table})")]
        rows = con.execute(f"SELECT * FROM {table} ORDER BY rowid").fetchall()
    out = {"columns": cols, "rows": len(rows), "md5": {}}
    for k, c in enumerate(cols):
        h = hashlib.md5()
        for r in rows:
            v = r[k]
            if v is None:
                h.update(b"N")
            elif isinstance(v, float):
                h.update(b"f" + np.float64(v).tobytes())
            elif isinstance(v, int):
                h.update(b"i" + np.int64(v).tobytes())
            else:
                h.update(b"s" + str(v).encode())
        out["md5"][c] = h.hexdigest()
    if "date" in cols:
        k = cols.index("date")
        ds = sorted({str(r[k]) for r in rows})
        out["distinct_dates"] = len(ds)
        out["dates_md5"] = hashlib.md5("\n".join(ds).encode()).hexdigest()
    return out


@pytest.fixture(scope="module")
def engine_l0(tmp_path_factory):
    from pfml.config import Config
    from pfml.data import acquire
    from pfml.data import synthetic as syn
    d = str(tmp_path_factory.mktemp("l0"))
    syn.write_raw(syn.generate(syn.l0_spec()), d)
    cfg = Config.default().override([f"run.data_dir={d}"])
    assert cfg.run.compat_mode
    acquire.get_additional_data(cfg)
    acquire.sp500_subset(cfg)
    return d


@pytest.mark.parametrize("name,db,table", [
    ("d_ret_ex", "crsp_daily.db", "d_ret_ex"),
    ("jkp_sp500_factors", "JKP_US_SP500.db", "Factors"),        # reference: JKP_SP500.db (Q11)
    ("daily_sp500", "crsp_daily_SP500.db", "d_ret_ex"),         # reference: db_crsp_daily_SP500.db:Factors
])
def test_l0_tables_match_reference(engine_l0, name, db, table):
    gold = json.load(open(GOLD))[name]
    got = table_fingerprint(os.path.join(engine_l0, db), table)
    assert got["columns"] == gold["columns"]
    assert got["rows"] == gold["rows"]
    if "distinct_dates" in gold:
        assert got["distinct_dates"] == gold["distinct_dates"]
        assert got["dates_md5"] == gold["dates_md5"]
    bad = [c for c in gold["columns"] if got["md5"][c] != gold["md5"][c]]
    assert not bad, bad


def test_l0_chunk_end_days_lost_as_in_reference(engine_l0):
    """Q19 made visible: the chunk-end trading days are absent from d_ret_ex (compat)."""
    with sqlite3.connect(os.path.join(engine_l0, "crsp_daily.db")) as con:
        n_end = con.execute("SELECT count(*) FROM d_ret_ex WHERE date LIKE '1962-01-02%'").fetchone()[0]
        n_next = con.execute("SELECT count(*) FROM d_ret_ex WHERE date LIKE '1962-01-03%'").fetchone()[0]
        tables = {r[0] for r in con.execute("SELECT name FROM sqlite_master WHERE type='table'")}
    assert n_end == 0 and n_next > 0
    assert tables == {"crsp_daily", "d_ret_ex"}                 # Q20: raw table kept
    assert json.load(open(GOLD))["crsp_daily_tables"] == ["d_ret_ex"]


def test_l0_corrected_mode_keeps_chunk_end_days(tmp_path):
    from pfml.config import Config
    from pfml.data import acquire
    from pfml.data import synthetic as syn
    d = str(tmp_path)
    syn.write_raw(syn.generate(syn.l0_spec()), d)
    cfg = Config.default().override([f"run.data_dir={d}", "run.compat_mode=false"])
    acquire.get_additional_data(cfg)
    counts = acquire.sp500_subset(cfg)
    with sqlite3.connect(os.path.join(d, "crsp_daily_SP500.db")) as con:
        n_end = con.execute("SELECT count(*) FROM d_ret_ex WHERE date = '1962-01-02'").fetchone()[0]
    gold = json.load(open(GOLD))
    assert n_end > 0
    assert counts["daily"] > gold["daily_sp500"]["rows"]
