#!/usr/bin/env python3
"""Freeze L2/L3 golden outputs by running the REFERENCE's own Prepare_Data.py and
"Estimate Covariance Matrix.py" on the tests' synthetic raw data.

OFFLINE, MANUAL, DEV-TIME TOOL: it exec()s the untrusted reference scripts
in-process, so it is never run by a test, by ``build()`` or on the GPU box; run it by hand in a
scratch container.  Nothing the reference writes is unpickled here: the Barra dict is taken
from the scripts' shared namespace (the reference's in-memory ``barra_cov``), the panel from
its SQLite table, the rest from its CSVs.

Inputs: the tests' 50-stock synthetic raw files (data/synthetic.py ``small_spec``) taken
through this engine's L0 stages (S0a/S0b: ETL + S&P 500 subset, the reference's file layout
``Data/JKP_US_SP500.db:Factors`` and ``Data/crsp_daily_SP500.db:d_ret_ex``), then the two
reference scripts exec'd verbatim in one namespace as Main.py does (Main.py:16-22), with
harness-only edits:

* ``get_settings`` wrapped to apply the small-panel settings the engine's tests use
  (data/synthetic.py ``settings_for_small``: screen window, test_end, cov_set obs / half-lives);
* ``pd.read_excel("Factor Details.xlsx")`` reads the CSV twin (openpyxl is not installed);
* ``numba.njit`` is the identity (numba is not installed: ewma_vol runs as plain Python,
  Estimate Covariance Matrix.py:345);
* matplotlib on the Agg backend (the universe plot of Prepare_Data.py:459-468 is not shown).

Frozen under tests/golden/ref_l2l3/:
* ``factors_meta.json``     row count, per-column fingerprints of Factors_processed (ALL rows:
                            count, NaN count, sum, sum |x|, sum x^2; bool / date columns as
                            integers), the sampled row keys;
* ``factors_sample.npz``    1500 sampled rows, every numeric column, exact;
* ``wealth_processed.csv``, ``cluster_labels_processed.csv``   full;
* ``barra.npz``             per Barra month: ids, fct_load, fct_cov, ivol_vec for 3 months,
                            and per-month fingerprints of all months.

    python tools/make_golden_l2l3.py [/root/reference]
"""
from __future__ import annotations

import json
import os
import shutil
import sqlite3
import sys
import tempfile
import types

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden", "ref_l2l3")
L2L3_SCRIPTS = ["Prepare_Data.py", "Estimate Covariance Matrix.py"]


def raw_inputs(data_dir: str):
    """Synthetic raw files + the engine's L0 (the tests' small_data fixture up to L0)."""
    from pfml.config import Config
    from pfml.data import acquire
    from pfml.data import synthetic as syn
    spec = syn.small_spec()
    syn.write_raw(syn.generate(spec), data_dir)
    cfg = syn.settings_for_small(Config.default().override([f"run.data_dir={data_dir}"]), spec)
    acquire.get_additional_data(cfg)
    acquire.sp500_subset(cfg)
    return cfg


def install_stubs() -> None:
    sm = types.ModuleType("statsmodels")
    smd = types.ModuleType("statsmodels.distributions")
    sme = types.ModuleType("statsmodels.distributions.empirical_distribution")

    class ECDF:                                        # only used by dead code (ecdf_transform)
        def __init__(self, x):
            self.x = np.sort(np.asarray(x))

        def __call__(self, v):
            return np.searchsorted(self.x, v, side="right") / len(self.x)

    sme.ECDF = ECDF
    nb = types.ModuleType("numba")
    nb.njit = lambda f=None, **kw: f if f is not None else (lambda g: g)
    sys.modules.update({"statsmodels": sm, "statsmodels.distributions": smd,
                        "statsmodels.distributions.empirical_distribution": sme, "numba": nb})
    import matplotlib
    matplotlib.use("Agg")
    orig_excel = pd.read_excel

    def read_excel(p, *a, **k):
        if str(p).endswith("Factor Details.xlsx"):
            return pd.read_csv(str(p)[:-len(".xlsx")] + ".csv")
        return orig_excel(p, *a, **k)

    pd.read_excel = read_excel


def patched_settings(gf, cfg) -> None:
    orig = gf.get_settings

    def get_settings():
        s, p = orig()
        for sec, keys in (("screens", ("start", "end")), ("split", ("test_end",))):
            for k in keys:
                s[sec][k] = pd.Timestamp(cfg.settings[sec][k])
        for k in ("obs", "hl_cor", "hl_var"):
            s["cov_set"][k] = cfg.settings["cov_set"][k]
        return s, p

    gf.get_settings = get_settings


def run_reference_l2l3(tmp: str, cfg, ref: str = REF) -> dict:
    """Exec the two reference scripts on ``tmp``/Data; returns the shared namespace."""
    install_stubs()
    sys.path.insert(0, ref)
    cwd = os.getcwd()
    os.chdir(ref)
    try:
        import General_functions as gf
        patched_settings(gf, cfg)
        ns = {"__name__": "__main__", "path": tmp + "/"}
        for s in L2L3_SCRIPTS:
            print(f"=== reference {s}", flush=True)
            src = open(os.path.join(ref, s), encoding="utf-8").read()
            exec(compile(src, os.path.join(ref, s), "exec"), ns)
    finally:
        os.chdir(cwd)
    return ns


def _num(col: pd.Series) -> np.ndarray | None:
    if col.dtype == bool or col.dtype.kind == "b":
        return col.to_numpy().astype(np.float64)
    if np.issubdtype(col.dtype, np.datetime64):
        return col.to_numpy().astype("datetime64[D]").astype(np.int64).astype(np.float64)
    if col.dtype.kind in "iuf":
        return col.to_numpy(np.float64)
    return None


def fingerprint(a: np.ndarray) -> list:
    a = np.asarray(a, np.float64).ravel()
    nan = np.isnan(a)
    v = a[~nan]
    return [float(a.size), float(nan.sum()), float(v.sum()), float(np.abs(v).sum()),
            float((v * v).sum())]


def read_factors_processed(data_dir: str) -> pd.DataFrame:
    with sqlite3.connect(os.path.join(data_dir, "JKP_US_SP500.db")) as con:
        df = pd.read_sql_query("SELECT * FROM Factors_processed", con, parse_dates=["eom", "eom_ret"])
    return df


def main():
    tmp = tempfile.mkdtemp(prefix="pfml_ref_l2l3_")
    data = os.path.join(tmp, "Data")
    os.makedirs(data)
    cfg = raw_inputs(data)
    ns = run_reference_l2l3(tmp, cfg)
    os.makedirs(OUT, exist_ok=True)
    fp = read_factors_processed(data).sort_values(["id", "eom"]).reset_index(drop=True)
    cols = [c for c in fp.columns if _num(fp[c]) is not None]
    meta = {"rows": int(len(fp)), "columns": list(fp.columns),
            "fingerprint": {c: fingerprint(_num(fp[c])) for c in cols},
            "ff12_counts": fp["ff12"].astype(str).value_counts().sort_index().to_dict(),
            "scripts": L2L3_SCRIPTS}
    rng = np.random.default_rng(0)
    samp = np.sort(rng.choice(len(fp), size=min(1500, len(fp)), replace=False))
    np.savez_compressed(os.path.join(OUT, "factors_sample.npz"), rows=samp,
                        cols=np.array(cols),
                        values=np.stack([_num(fp[c])[samp] for c in cols], axis=1),
                        ff12=fp["ff12"].astype(str).to_numpy()[samp].astype("U16"))
    with open(os.path.join(OUT, "factors_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    for n in ("wealth_processed.csv", "cluster_labels_processed.csv"):
        shutil.copy(os.path.join(data, n), os.path.join(OUT, n))
    barra = ns["barra_cov"]                      # the reference's in-memory dict, no unpickling
    dates = sorted(barra.keys())
    pick = [dates[0], dates[len(dates) // 2], dates[-1]]
    arr = {"months": np.array([str(pd.Timestamp(d).date()) for d in dates])}
    fps = []
    for d in dates:
        o = barra[d]
        fps.append(fingerprint(o["fct_load"].to_numpy()) + fingerprint(o["fct_cov"].to_numpy())
                   + fingerprint(o["ivol_vec"].to_numpy())
                   + [float(np.asarray(o["fct_load"].index, np.int64).sum())])
    arr["fingerprints"] = np.asarray(fps)
    arr["factors"] = np.array([str(c) for c in barra[dates[0]]["fct_cov"].columns])
    for i, d in enumerate(pick):
        o = barra[d]
        arr[f"pick{i}_month"] = np.array(str(pd.Timestamp(d).date()))
        arr[f"pick{i}_ids"] = np.asarray(o["fct_load"].index, np.int64)
        arr[f"pick{i}_load"] = o["fct_load"].to_numpy(np.float64)
        arr[f"pick{i}_cov"] = o["fct_cov"].to_numpy(np.float64)
        arr[f"pick{i}_ivol"] = o["ivol_vec"].to_numpy(np.float64)
    np.savez_compressed(os.path.join(OUT, "barra.npz"), **arr)
    print("golden written to", OUT, {"rows": meta["rows"], "barra_months": len(dates)})
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
