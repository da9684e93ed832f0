#!/usr/bin/env python3
"""Compact per-kernel summary of a rocprofv3 run (rocpd SQLite output or kernel_stats.csv).

usage: python tools/rocprof_summary.py <run_results.db | kernel_stats.csv> [--top N] [--md]
"""
import argparse
import re
import sqlite3
import sys

import pandas as pd


def short(name: str, width: int = 70) -> str:
    n = re.sub(r"void |at::native::|\(anonymous namespace\)::", "", name)
    n = re.sub(r"\(.*", "", n)                    # drop argument lists
    return n if len(n) <= width else n[: width - 3] + "..."


def from_db(path: str) -> pd.DataFrame:
    con = sqlite3.connect(path)
    k = pd.read_sql("select name, start, end from kernels", con)
    k["dur_us"] = (k["end"] - k["start"]) / 1000.0
    g = k.groupby("name")["dur_us"].agg(["count", "sum", "mean", "max"]).reset_index()
    return g.rename(columns={"count": "calls", "sum": "total_us", "mean": "avg_us",
                             "max": "max_us"})


def from_csv(path: str) -> pd.DataFrame:
    d = pd.read_csv(path)
    return pd.DataFrame({"name": d["Name"], "calls": d["Calls"],
                         "total_us": d["TotalDurationNs"] / 1000.0,
                         "avg_us": d["AverageNs"] / 1000.0, "max_us": d["MaxNs"] / 1000.0})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    df = from_db(a.path) if a.path.endswith(".db") else from_csv(a.path)
    df = df.sort_values("total_us", ascending=False)
    tot = df["total_us"].sum()
    df["pct"] = 100.0 * df["total_us"] / tot
    df["name"] = df["name"].map(short)
    df = df.head(a.top)
    cols = ["name", "calls", "total_us", "avg_us", "max_us", "pct"]
    if a.md:
        print("| kernel | calls | total µs | avg µs | max µs | % |")
        print("|---|---:|---:|---:|---:|---:|")
        for _, r in df.iterrows():
            print(f"| `{r['name']}` | {r['calls']} | {r['total_us']:.1f} | {r['avg_us']:.1f} | "
                  f"{r['max_us']:.1f} | {r['pct']:.1f} |")
        print(f"\nTotal kernel time: {tot / 1000.0:.2f} ms")
    else:
        with pd.option_context("display.width", 200, "display.max_colwidth", 80):
            print(df[cols].to_string(index=False, float_format=lambda v: f"{v:.1f}"))
        print(f"total kernel time {tot / 1000.0:.2f} ms")


if __name__ == "__main__":
    sys.exit(main())
