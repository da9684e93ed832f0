#!/usr/bin/env python3
"""S3 (Estimate Covariance Matrix.py) stage wall-clock at production shape: ~18.8k trading
days x ~500 stocks (9.4M daily rows), ~860 months of processed characteristics (115 ranked
features, 13 clusters + 12 FF12 industries = 25 factors), 2520-day EWMA windows.  Synthetic
in-memory frames of the reference's schema (no CRSP/JKP data).  Times the batched device form
(estimate_cov_frames) and the round-1 pandas-bound form (estimate_cov_frames_pandas) on the
same frames; prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.config import get_features, get_settings  # noqa: E402
from pfml.models import risk  # noqa: E402


def frames(n_stocks: int, start: str, end: str, seed: int = 0):
    rng = np.random.default_rng(seed)
    feats = get_features()
    eoms = pd.date_range(start, end, freq="ME")
    T = len(eoms)
    ids = np.arange(n_stocks) + 10001
    mi = np.repeat(np.arange(T), n_stocks)
    chars = pd.DataFrame({"id": np.tile(ids, T), "eom": np.repeat(eoms, n_stocks)})
    chars["size_grp"] = rng.choice(["mega", "large", "small", "micro", "nano"], len(chars))
    chars["ff12"] = rng.choice([f"ind{i}" for i in range(12)], len(chars))
    F = rng.random((len(chars), len(feats)))
    chars = pd.concat([chars, pd.DataFrame(F, columns=feats)], axis=1)
    days = pd.bdate_range(start, end)
    D = len(days)
    daily = pd.DataFrame({"id": np.tile(ids, D), "date": np.repeat(days, n_stocks),
                          "ret_exc": 0.02 * rng.standard_normal(D * n_stocks)})
    clusters = ["accruals", "debt_issuance", "investment", "low_leverage", "low_risk",
                "momentum", "profit_growth", "profitability", "quality", "seasonality",
                "short_term_reversal", "size", "value"]
    labels = pd.DataFrame({"characteristic": feats,
                           "cluster": [clusters[i % len(clusters)] for i in range(len(feats))],
                           "direction": rng.choice([-1, 1], len(feats))})
    del mi
    return chars, daily, labels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stocks", type=int, default=500)
    ap.add_argument("--start", default="1952-01-31")
    ap.add_argument("--end", default="2023-12-31")
    ap.add_argument("--no-pandas", action="store_true")
    args = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    t0 = time.perf_counter()
    chars, daily, labels = frames(args.stocks, args.start, args.end)
    t_data = time.perf_counter() - t0
    cs = get_settings()[0]["cov_set"]
    risk.estimate_cov_frames(chars.iloc[: 200 * args.stocks], daily.iloc[: 4000 * args.stocks],
                             labels, dict(cs, obs=500), dev)          # warm-up (kernels, JIT)
    if dev == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    b = risk.estimate_cov_frames(chars, daily, labels, cs, dev)
    if dev == "cuda":
        torch.cuda.synchronize()
    t_dev = time.perf_counter() - t0
    rec = {"metric": "S3 estimate-cov stage wall-clock (batched, device)", "s3_s": round(t_dev, 2),
           "days": int(daily["date"].nunique()), "daily_rows": len(daily),
           "months": int(chars["eom"].nunique()), "stocks": args.stocks,
           "barra_months": len(b.months), "factors": len(b.factors), "device": dev,
           "data_gen_s": round(t_data, 1),
           "data": "synthetic frames of the reference schema (no CRSP/JKP data)"}
    if not args.no_pandas:
        t0 = time.perf_counter()
        p = risk.estimate_cov_frames_pandas(chars, daily, labels, cs, dev)
        if dev == "cuda":
            torch.cuda.synchronize()
        rec["s3_pandas_form_s"] = round(time.perf_counter() - t0, 2)
        rec["speedup"] = round(rec["s3_pandas_form_s"] / t_dev, 1)
        rec["max_rel_F"] = float(np.abs(b.F - p.F).max() / np.abs(p.F).max())
        rec["max_rel_ivol"] = float(np.abs(b.ivol - p.ivol).max() / np.abs(p.ivol).max())
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
