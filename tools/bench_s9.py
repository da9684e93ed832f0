#!/usr/bin/env python3
"""S9 weight recursion (PFML_best_hps.py:168-218) at production shape: the synthetic
500-stock engine panel (bench.py's engine_inputs), the last ``--months`` Barra months as the
OOS period and random aim weights.  Times the whole ``pfml_weights`` call; run with
PFML_HOST_TIMING=sync for its sections (plan / m_t / chain / gather+frame)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stocks", type=int, default=500)
    ap.add_argument("--months", type=int, default=360)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args()
    from pfml.config import Config
    from pfml.data.synthetic import engine_inputs
    from pfml.models.portfolio import pfml_weights
    from pfml.utils.dates import month_index
    cfg = Config.default()
    t0 = time.perf_counter()
    chars, barra, wealth, rf = engine_inputs(n_stocks=a.stocks)
    mi = month_index(chars["eom"])
    cm = np.intersect1d(np.unique(mi[chars["valid"].to_numpy()]), barra.months)
    wm = month_index(wealth["eom"])
    cm = cm[np.isin(cm, wm) & np.isin(cm + 1, wm)]
    oos = cm[-a.months:]
    sub = chars[np.isin(mi, oos) & chars["valid"].to_numpy()][["eom", "id"]].copy()
    rng = np.random.default_rng(0)
    sub["w_aim"] = rng.normal(size=len(sub)) / a.stocks
    data_s = time.perf_counter() - t0
    ts = []
    for _ in range(a.steps):
        if a.device == "cuda":
            torch.cuda.synchronize()
        t = time.perf_counter()
        w = pfml_weights(cfg, chars, barra, wealth, rf, sub, oos, a.device)
        if a.device == "cuda":
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    print(json.dumps({"metric": "S9 pfml_weights wall-clock", "s9_ms": round(1000 * min(ts), 1),
                      "s9_ms_all": [round(1000 * x, 1) for x in ts], "oos_months": int(len(oos)),
                      "stocks": a.stocks, "rows": int(len(w)), "finite": bool(np.isfinite(
                          w["w"].to_numpy()).all()), "data_s": round(data_s, 2),
                      "device": a.device}))


if __name__ == "__main__":
    main()
