#!/usr/bin/env python3
"""Kernel timeline of the last N dispatches of a rocprofv3 run (rocpd SQLite output):
start/end relative to the first shown dispatch, queue id, duration.

usage: python tools/rocprof_timeline.py <run_results.db> [--last N] [--grep PATTERN]
"""
import argparse
import re
import sqlite3

import pandas as pd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--grep", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    q = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    k = pd.read_sql(f"select name, start, end{', ' + q if q else ''} from kernels order by start", con)
    if a.grep:
        k = k[k["name"].str.contains(a.grep)]
    k = k.tail(a.last).copy()
    t0 = k["start"].min()
    k["t0_us"] = (k["start"] - t0) / 1e3
    k["t1_us"] = (k["end"] - t0) / 1e3
    k["dur_us"] = (k["end"] - k["start"]) / 1e3
    k["name"] = k["name"].map(lambda n: re.sub(r"\(.*", "", re.sub(r"void |\(anonymous namespace\)::", "", n))[:60])
    pd.set_option("display.width", 200)
    print(k[["name"] + ([q] if q else []) + ["t0_us", "t1_us", "dur_us"]].to_string(index=False))


if __name__ == "__main__":
    main()
