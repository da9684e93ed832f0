#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 --pmc counters (counter_collection.csv or rocpd .db).

usage: python tools/pmc_summary.py <dir> [--top N]"""
import argparse
import glob
import os
import sqlite3

import pandas as pd


def load(d: str) -> pd.DataFrame:
    csvs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if csvs:
        df = pd.read_csv(csvs[0])
        name = "Kernel_Name" if "Kernel_Name" in df else "Kernel-Name"
        return df.rename(columns={name: "kernel", "Counter_Name": "counter",
                                  "Counter_Value": "value"})[["kernel", "counter", "value"]]
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    con = sqlite3.connect(dbs[0])
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    for t in ("counters_collection", "pmc_events", "counters"):
        if t in tabs:
            df = pd.read_sql(f"select * from {t}", con)
            break
    else:
        raise SystemExit(f"no counter table in {dbs[0]}: {tabs}")
    cols = {c.lower(): c for c in df.columns}
    k = cols.get("kernel_name") or cols.get("name")
    c = cols.get("counter_name") or cols.get("counter")
    v = cols.get("value") or cols.get("counter_value")
    return df.rename(columns={k: "kernel", c: "counter", v: "value"})[["kernel", "counter", "value"]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    df = load(a.dir)
    df["kernel"] = (df["kernel"].str.replace("(anonymous namespace)::", "", regex=False)
                    .str.replace(r"^void ", "", regex=True).str.replace(r"\(.*", "", regex=True)
                    .str.slice(0, 48))
    piv = df.pivot_table(index="kernel", columns="counter", values="value", aggfunc="sum")
    tr = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if tr:
        # per-kernel time from the trace of the same run; GRBM_GUI_ACTIVE is summed over the 8
        # XCDs (MI355X_MICROARCH.md, DVFS give-back): effective clock = it / 8 / time
        t = pd.read_csv(tr[0])
        t["kernel"] = (t["Kernel_Name"].str.replace("(anonymous namespace)::", "", regex=False)
                       .str.replace(r"^void ", "", regex=True)
                       .str.replace(r"\(.*", "", regex=True).str.slice(0, 48))
        t["ns"] = t["End_Timestamp"] - t["Start_Timestamp"]
        piv["time_us"] = t.groupby("kernel")["ns"].sum() / 1e3
        if "GRBM_GUI_ACTIVE" in piv:
            piv["clk_ghz"] = piv["GRBM_GUI_ACTIVE"] / 8.0 / (piv["time_us"] * 1e3)
    first = piv.columns[0]
    piv = piv.sort_values(first, ascending=False).head(a.top)
    pd.set_option("display.width", 250)
    pd.set_option("display.max_columns", 20)
    print(piv.to_string(float_format=lambda x: f"{x:.3e}"))


if __name__ == "__main__":
    main()
