#!/usr/bin/env python3
"""Freeze L0 golden outputs by running the REFERENCE's own 0_Get_Additional_Data.py and
0_SP500_Subset.py on the tests' synthetic raw data.

OFFLINE, MANUAL, DEV-TIME TOOL: it exec()s the untrusted reference scripts in-process, so it
is never run by a test, by ``build()`` or on the GPU box; run it by hand in a scratch
container.  Harness-only edits:

* ``path`` (the scripts' hard-coded data root) points at a scratch copy of the raw files;
* ``dotenv.load_dotenv`` is a no-op and ``sqlalchemy.create_engine`` returns an inert object:
  the WRDS download (0_Get_Additional_Data.py:38-79) is inside a string literal in the
  reference, so the engine object is never used.

Inputs: data/synthetic.py ``l0_spec`` raw files (12 names over the reference's 1952-2024 L0
window) (crsp_daily with pandas' TIMESTAMP date
text, as read_sql_query(parse_dates) + to_sql of the WRDS pull leaves it; JKP Factors with
its `date` column).  Frozen under tests/golden/ref_l0/l0_golden.json, per output table
(d_ret_ex; the two subset tables the reference writes as JKP_SP500.db:Factors and
db_crsp_daily_SP500.db:Factors): the column list, the row count, and per column an md5 of the
values in table order (REAL as float64 bytes, INTEGER as int64, TEXT as utf-8), plus the
md5 of the sorted distinct dates.

    python tools/make_golden_l0.py [/root/reference]
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sqlite3
import sys
import tempfile
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden", "ref_l0")


def table_fingerprint(db: str, table: str) -> dict:
    """Column list, row count and per-column md5 of a SQLite table in rowid order."""
    with sqlite3.connect(db) as con:
        cols = [r[1] for r in con.execute(f"PRAGMA table_info({table})")]
        rows = con.execute(f"SELECT * FROM {table} ORDER BY rowid").fetchall()
    out = {"columns": cols, "rows": len(rows), "md5": {}}
    for k, c in enumerate(cols):
        vals = [r[k] for r in rows]
        h = hashlib.md5()
        for v in vals:
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


def write_raw(data_dir: str) -> None:
    from pfml.data import synthetic as syn
    syn.write_raw(syn.generate(syn.l0_spec()), data_dir)


def install_stubs() -> None:
    dotenv = types.ModuleType("dotenv")
    dotenv.load_dotenv = lambda *a, **k: True
    sa = types.ModuleType("sqlalchemy")
    sa.create_engine = lambda *a, **k: object()
    sys.modules["dotenv"] = dotenv
    sys.modules["sqlalchemy"] = sa


def run_reference(base: str) -> None:
    """base/JKMP_22_Replication/Data holds the raw files; both scripts exec'd verbatim but for
    their `path` line."""
    install_stubs()
    s1 = open(os.path.join(REF, "0_Get_Additional_Data.py")).read()
    s1 = s1.replace('path = "...Single Authored/"', f'path = "{base}/"')
    s2 = open(os.path.join(REF, "0_SP500_Subset.py")).read()
    s2 = s2.replace('path = "...JKMP_22_Replication/"', f'path = "{base}/JKMP_22_Replication/"')
    cwd = os.getcwd()
    try:
        exec(compile(s1, "0_Get_Additional_Data.py", "exec"), {"__name__": "__main__"})
        exec(compile(s2, "0_SP500_Subset.py", "exec"), {"__name__": "__main__"})
    finally:
        os.chdir(cwd)


def main() -> None:
    base = tempfile.mkdtemp(prefix="pfml_l0_")
    data = os.path.join(base, "JKMP_22_Replication", "Data")
    os.makedirs(data)
    try:
        write_raw(data)
        run_reference(base)
        gold = {
            "d_ret_ex": table_fingerprint(os.path.join(data, "crsp_daily.db"), "d_ret_ex"),
            "jkp_sp500_factors": table_fingerprint(os.path.join(data, "JKP_SP500.db"), "Factors"),
            "daily_sp500": table_fingerprint(os.path.join(data, "db_crsp_daily_SP500.db"),
                                             "Factors"),
        }
        with sqlite3.connect(os.path.join(data, "crsp_daily.db")) as con:
            gold["crsp_daily_tables"] = sorted(r[0] for r in con.execute(
                "SELECT name FROM sqlite_master WHERE type = 'table'"))
        os.makedirs(OUT, exist_ok=True)
        with open(os.path.join(OUT, "l0_golden.json"), "w") as f:
            json.dump(gold, f, indent=1, sort_keys=True)
        print(json.dumps({k: (v["rows"] if isinstance(v, dict) else v) for k, v in gold.items()}))
    finally:
        shutil.rmtree(base, ignore_errors=True)


if __name__ == "__main__":
    main()
