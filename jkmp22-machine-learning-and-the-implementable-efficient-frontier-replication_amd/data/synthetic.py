"""Synthetic raw inputs with the reference's external schema.

WRDS CRSP / JKP data are licensed and there is no network, so every test and benchmark runs
on synthetic panels that have exactly the columns the reference reads:

* ``JKP_US.db:Factors``             id, eom, sic, ff49, size_grp, me, crsp_exchcd, ret_exc, features
                                    (Prepare_Data.py:147-166; subset by 0_SP500_Subset.py)
* ``crsp_daily.db:crsp_daily``      permno, date, ret, primaryexch (0_Get_Additional_Data.py:104-149)
* ``FF_RF_monthly.csv``             yyyymm, RF (percent)            (Prepare_Data.py:62-71)
* ``FF_RF_daily.csv``               date, Mkt-RF, SMB, HML, RF      (0_Get_Additional_Data.py:82-91)
* ``market_returns.csv``            excntry, eom, mkt_vw_exc        (Prepare_Data.py:82-89)
* ``Cluster Labels.csv``            characteristic, cluster         (Prepare_Data.py:102-105)
* ``Factor Details.csv``            abr_jkp, direction              (Prepare_Data.py:108-117; .xlsx there)
* ``rff_w.csv``                     unnamed index + k x p_max/2 W   (PFML_Input_Data.py:245)
* ``SP500_Historical_Constituents.csv``  Unnamed: 0, permno, start, ending, date (0_SP500_Subset.py:18-23)

The generator is vectorised numpy (a 500-stock, 1952-2023 panel with ~9M daily rows builds
in tens of seconds); small panels for tests build in well under a second.
"""
from __future__ import annotations

import os
import sqlite3
from dataclasses import dataclass

import numpy as np
import pandas as pd

from ..config import get_features, get_settings
from ..utils.dates import month_end, month_index

# One representative SIC range per FF12 industry (General_functions.py:293-402) plus "Other".
_SIC_POOL = np.array([2000, 2080, 3711, 3714, 3560, 2650, 1311, 2911, 2810, 2860, 3570, 7372,
                      4813, 4911, 5311, 5812, 2834, 8062, 6021, 6311, 1000, 1540, 7011, 4011])
_CLUSTERS = ["Accruals", "Debt Issuance", "Investment", "Low Leverage", "Low Risk", "Momentum",
             "Profit Growth", "Profitability", "Quality", "Seasonality", "Short-Term Reversal",
             "Size", "Value"]


@dataclass
class SyntheticSpec:
    n_stocks: int = 500            # concurrent constituents (S&P 500 universe size)
    n_extra: int = 0               # non-constituent stocks in JKP_US (removed by the subset step)
    start: str = "1952-01-31"
    end: str = "2023-12-31"
    mean_life_months: int = 240
    feat_nan: float = 0.08
    feat_zero: float = 0.02
    missing_row: float = 0.002
    p_max: int = 512
    seed: int = 0
    daily: bool = True


def _firm_timelines(rng, n_slots, n_months, mean_life):
    """Each slot hosts a sequence of firms with geometric lifetimes; returns (slot, start, end)."""
    rows = []
    for s in range(n_slots):
        t = -int(rng.integers(0, mean_life))        # firms already alive at the start
        while t < n_months:
            life = max(24, int(rng.geometric(1.0 / mean_life)))
            a, b = max(t, 0), min(t + life, n_months) - 1
            if b >= a:
                rows.append((s, a, b))
            t += life
    return np.asarray(rows, dtype=np.int64)


def generate(spec: SyntheticSpec | None = None, features: list[str] | None = None) -> dict:
    """Return a dict of DataFrames (raw inputs, reference schema)."""
    spec = spec or SyntheticSpec()
    rng = np.random.default_rng(spec.seed)
    features = features or get_features()
    all_feats = get_features(exclude_poor_coverage=False)
    m0, m1 = int(month_index(spec.start)[0]), int(month_index(spec.end)[0])
    n_months = m1 - m0 + 1
    months = month_end(np.arange(m0, m1 + 1))

    # ---- market / rf -----------------------------------------------------------------
    rf_m = np.clip(rng.normal(0.30, 0.12, n_months), 0.0, None)            # percent
    mkt = rng.normal(0.006, 0.045, n_months + 1)                           # eom_ret aligned
    ff_rf = pd.DataFrame({"yyyymm": months.year * 100 + months.month, "RF": np.round(rf_m, 4)})
    market = pd.DataFrame({"excntry": "USA",
                           "eom": month_end(np.arange(m0, m1 + 2)).strftime("%Y-%m-%d"),
                           "mkt_vw_exc": mkt})

    # ---- firm timelines ----------------------------------------------------------------
    tl = _firm_timelines(rng, spec.n_stocks + spec.n_extra, n_months, spec.mean_life_months)
    n_firms = len(tl)
    ids = 10001 + np.arange(n_firms)
    is_const = tl[:, 0] < spec.n_stocks
    lens = tl[:, 2] - tl[:, 1] + 1
    firm_of_row = np.repeat(np.arange(n_firms), lens)
    t_of_row = np.concatenate([np.arange(a, b + 1) for _, a, b in tl])
    keep = rng.random(len(t_of_row)) >= spec.missing_row
    firm_of_row, t_of_row = firm_of_row[keep], t_of_row[keep]
    n_rows = len(t_of_row)

    beta = rng.normal(1.0, 0.3, n_firms)
    ivol = rng.uniform(0.04, 0.12, n_firms)
    ret = beta[firm_of_row] * mkt[t_of_row] + ivol[firm_of_row] * rng.standard_normal(n_rows)
    ret = np.clip(ret, -0.9, 3.0)
    # market equity: lognormal level, drifting with the firm's own returns
    me0 = np.exp(rng.normal(8.5, 1.3, n_firms))
    order = np.lexsort((t_of_row, firm_of_row))
    firm_of_row, t_of_row, ret = firm_of_row[order], t_of_row[order], ret[order]
    logg = np.log1p(ret)
    first = np.r_[True, firm_of_row[1:] != firm_of_row[:-1]]
    cum = np.cumsum(logg)
    base = np.maximum.accumulate(np.where(first, np.arange(n_rows), 0))
    me = me0[firm_of_row] * np.exp(cum - cum[base])

    # ---- characteristics: persistent AR(1) cross-sections --------------------------------
    k_all = len(all_feats)
    firm_fx = rng.standard_normal((n_firms, k_all)).astype(np.float32)
    noise = rng.standard_normal((n_rows, k_all)).astype(np.float32)
    X = 0.8 * firm_fx[firm_of_row] + 0.6 * noise
    X[rng.random(X.shape) < spec.feat_nan] = np.nan
    X[rng.random(X.shape) < spec.feat_zero] = 0.0
    chars = pd.DataFrame(X.astype(np.float64), columns=all_feats)
    # Raw-level features consumed before ranking (Prepare_Data.py:178-182)
    dolvol = np.exp(rng.normal(17.0, 1.5, n_firms))[firm_of_row] * np.exp(0.2 * noise[:, 0])
    chars["dolvol_126d"] = dolvol
    chars["rvol_252d"] = ivol[firm_of_row] / np.sqrt(21) * np.exp(0.1 * noise[:, 1])
    chars["market_equity"] = me
    nan_dv = rng.random(n_rows) < 0.001
    chars.loc[nan_dv, "dolvol_126d"] = np.nan

    sic = rng.choice(_SIC_POOL, n_firms)
    sic_row = sic[firm_of_row].astype(np.float64)
    sic_row[rng.random(n_rows) < 0.001] = np.nan
    size_q = pd.Series(me).groupby(t_of_row).rank(pct=True).to_numpy()
    size_grp = np.select([size_q > 0.8, size_q > 0.5, size_q > 0.2, size_q > 0.05],
                         ["mega", "large", "small", "micro"], "nano")
    # JKP's `date`: the month's last business day (the column 0_SP500_Subset.py:52-55 filters
    # the Factors chunks on)
    mdt = pd.DatetimeIndex(months[t_of_row])
    last_bday = mdt - pd.to_timedelta(np.maximum(mdt.weekday.to_numpy() - 4, 0), unit="D")
    head = pd.DataFrame({
        "id": ids[firm_of_row],
        "eom": months[t_of_row].strftime("%Y-%m-%d"),
        "date": last_bday.strftime("%Y-%m-%d"),
        "sic": sic_row,
        "ff49": rng.integers(1, 50, n_firms)[firm_of_row],
        "size_grp": size_grp,
        "me": np.where(rng.random(n_rows) < 0.001, np.nan, me),
        "crsp_exchcd": rng.choice([1, 2, 3], n_firms, p=[0.6, 0.1, 0.3])[firm_of_row],
        "ret_exc": np.where(rng.random(n_rows) < 0.002, np.nan, ret),
    })
    factors = pd.concat([head, chars], axis=1)

    # ---- constituents ------------------------------------------------------------------
    const_rows = np.isin(firm_of_row, np.nonzero(is_const)[0])
    cons = pd.DataFrame({
        "permno": ids[firm_of_row[const_rows]],
        "start": months[tl[firm_of_row[const_rows], 1]].strftime("%Y-%m-%d"),
        "ending": months[tl[firm_of_row[const_rows], 2]].strftime("%Y-%m-%d"),
        "date": months[t_of_row[const_rows]].strftime("%Y-%m-%d"),
    })

    # ---- cluster labels / directions ---------------------------------------------------
    labels = pd.DataFrame({"characteristic": all_feats,
                           "cluster": [_CLUSTERS[i % len(_CLUSTERS)] for i in range(k_all)]})
    labels = labels[labels["characteristic"] != "rvol_252d"]     # appended by Prepare_Data
    details = pd.DataFrame({"abr_jkp": all_feats,
                            "direction": rng.choice([-1, 1], k_all)})

    # ---- RFF weights (k x p_max/2), written with an unnamed index column -----------------
    g0 = float(np.exp(-3.0))
    rff_w = rng.normal(0.0, np.sqrt(g0), (len(features), spec.p_max // 2))

    out = {"factors": factors, "ff_rf_monthly": ff_rf, "market": market,
           "cluster_labels": labels, "factor_details": details, "rff_w": rff_w,
           "constituents": cons}

    # ---- daily returns -------------------------------------------------------------------
    if spec.daily:
        days = pd.bdate_range(months[0] - pd.offsets.MonthBegin(1), months[-1])
        day_mi = month_index(days) - m0
        rf_d = rf_m[np.clip(day_mi, 0, n_months - 1)] / 21.0
        mkt_d = rng.normal(0.0003, 0.010, len(days))
        ff_daily = pd.DataFrame({"date": days.strftime("%Y%m%d").astype(int),
                                 "Mkt-RF": mkt_d * 100, "SMB": rng.normal(0, 0.5, len(days)),
                                 "HML": rng.normal(0, 0.5, len(days)), "RF": np.round(rf_d, 5)})
        # days of each month as a contiguous range
        mstart = np.searchsorted(day_mi, np.arange(n_months))
        mstop = np.searchsorted(day_mi, np.arange(n_months), side="right")
        cnt = (mstop - mstart)[t_of_row]
        d_firm = np.repeat(firm_of_row, cnt)
        d_idx = np.repeat(mstart[t_of_row] - np.cumsum(np.r_[0, cnt[:-1]]), cnt) + np.arange(cnt.sum())
        dret = beta[d_firm] * mkt_d[d_idx] + ivol[d_firm] / np.sqrt(21) * rng.standard_normal(len(d_idx))
        dret = dret + rf_d[d_idx] / 100.0
        # dates as pandas holds them after read_sql_query(parse_dates) of the WRDS pull: to_sql
        # stores "YYYY-MM-DD 00:00:00" text (0_Get_Additional_Data.py:65-79), the form the
        # reference's chunked BETWEEN reads compare as strings
        crsp_daily = pd.DataFrame({"permno": ids[d_firm], "date": days[d_idx],
                                   "ret": dret.astype(np.float32),
                                   "primaryexch": np.array(["N", "A", "Q"])[d_firm % 3]})
        out["crsp_daily"] = crsp_daily
        out["ff_rf_daily"] = ff_daily
    return out


def write_raw(raw: dict, data_dir: str) -> None:
    """Write the raw inputs in the reference's on-disk layout (L0 inputs)."""
    os.makedirs(data_dir, exist_ok=True)
    j = os.path.join
    for name in ("JKP_US.db", "crsp_daily.db"):
        if os.path.exists(j(data_dir, name)):
            os.remove(j(data_dir, name))
    with sqlite3.connect(j(data_dir, "JKP_US.db")) as con:
        raw["factors"].to_sql("Factors", con, index=False, chunksize=200_000)
    if "crsp_daily" in raw:
        with sqlite3.connect(j(data_dir, "crsp_daily.db")) as con:
            raw["crsp_daily"].to_sql("crsp_daily", con, index=False, chunksize=500_000)
        raw["ff_rf_daily"].to_csv(j(data_dir, "FF_RF_daily.csv"), index=False)
    raw["ff_rf_monthly"].to_csv(j(data_dir, "FF_RF_monthly.csv"), index=False)
    raw["market"].to_csv(j(data_dir, "market_returns.csv"), index=False)
    raw["cluster_labels"].to_csv(j(data_dir, "Cluster Labels.csv"), index=False)
    raw["factor_details"].to_csv(j(data_dir, "Factor Details.csv"), index=False)
    pd.DataFrame(raw["rff_w"]).to_csv(j(data_dir, "rff_w.csv"))
    cons = raw["constituents"].reset_index(drop=True)
    cons.to_csv(j(data_dir, "SP500_Historical_Constituents.csv"))


def small_spec(**kw) -> SyntheticSpec:
    """A CPU-test sized panel (plumbing config: ~50 stocks)."""
    base = dict(n_stocks=50, start="1990-01-31", end="2012-12-31", mean_life_months=120,
                seed=0)
    base.update(kw)
    return SyntheticSpec(**base)


def l0_spec(**kw) -> SyntheticSpec:
    """The L0 golden's panel: few names but the reference's whole 1952-2024 window, so every
    5-year chunk of the reference's L0 loops holds rows (0_SP500_Subset.py:109-111 merges an
    empty chunk's object-typed keys with int64 ones and raises)."""
    base = dict(n_stocks=12, start="1952-01-31", end="2024-12-31", mean_life_months=240,
                seed=7)
    base.update(kw)
    return SyntheticSpec(**base)


def settings_for_small(cfg, spec: SyntheticSpec):
    """Shrink the date-dependent settings so a short synthetic panel exercises every stage."""
    s = cfg.settings
    s["screens"]["start"] = pd.Timestamp(spec.start)
    s["screens"]["end"] = pd.Timestamp(spec.end)
    s["split"]["test_end"] = pd.Timestamp(spec.end)
    s["cov_set"]["obs"] = 400
    s["cov_set"]["hl_cor"] = 126
    s["cov_set"]["hl_var"] = 63
    return cfg


__all__ = ["SyntheticSpec", "generate", "write_raw", "small_spec", "l0_spec", "settings_for_small",
           "get_settings"]


def engine_inputs(n_stocks: int = 500, start: str = "1962-01-31", end: str = "2023-12-31",
                  n_factors: int = 25, seed: int = 0, turnover: float = 0.005):
    """Post-prep inputs of the PFML engine at production shape, built directly in memory:
    (chars DataFrame with the Factors_processed columns, BarraCov, wealth, risk_free).

    Used by the benchmark and the scaling tests to skip the (one-shot, pandas-bound) L2/L3
    stages: a rolling universe of ``n_stocks`` names with ``turnover`` monthly replacement,
    ranked features in (0, 1), Barra loadings ~ N(0,1), F = sample covariance * 21e-4,
    idiosyncratic variance U(0.01, 0.03)^2 * 21, lambda = 0.2 / U(1e7, 1e9), wealth 1e10.
    Every name has its full 13-month lookback, so every row after the first 12 months of
    its life is valid."""
    from .. import config as _c
    from ..models.risk import BarraCov
    rng = np.random.default_rng(seed)
    feats = _c.get_features()
    m0, m1 = int(month_index(start)[0]), int(month_index(end)[0])
    T = m1 - m0 + 1
    # slot timelines: each slot replaced with probability `turnover` per month
    ids_grid = np.zeros((T, n_stocks), dtype=np.int64)
    born = np.zeros((T, n_stocks), dtype=np.int64)
    cur = np.arange(n_stocks) + 10001
    b = np.full(n_stocks, -24)
    nxt = 10001 + n_stocks
    for t in range(T):
        rep = rng.random(n_stocks) < turnover
        k = int(rep.sum())
        cur = cur.copy(); b = b.copy()
        cur[rep] = nxt + np.arange(k)
        b[rep] = t
        nxt += k
        ids_grid[t], born[t] = cur, b
    tt = np.repeat(np.arange(T), n_stocks)
    ids = ids_grid.ravel()
    age = tt - born.ravel()
    R = len(ids)
    months = month_end(m0 + tt)
    chars = pd.DataFrame({
        "id": ids, "eom": months, "size_grp": "large",
        "me": np.exp(rng.normal(9, 1, R)), "lambda": 0.2 / rng.uniform(1e7, 1e9, R),
        "ret_ld1": rng.normal(0.006, 0.08, R), "tr_ld0": rng.normal(0.009, 0.08, R),
        "mu_ld0": np.repeat(rng.normal(0.009, 0.04, T), n_stocks),
        "valid": age >= 12})
    chars["tr_ld1"] = chars["ret_ld1"] + 0.003
    chars["eom_ret"] = chars["eom"] + pd.offsets.MonthEnd(1)
    F = pd.DataFrame(rng.random((R, len(feats))), columns=feats)
    chars = pd.concat([chars, F], axis=1)
    # Barra objects for every month over the valid names
    Fm = np.stack([np.cov(rng.normal(size=(n_factors, 300))) * 1e-4 * 21 for _ in range(T)])
    val = chars["valid"].to_numpy()
    vm = (m0 + tt)[val]
    vid = ids[val]
    order = np.lexsort((vid, vm))
    vm, vid = vm[order], vid[order]
    cnt = np.bincount(vm - m0, minlength=T)
    barra = BarraCov(months=np.arange(m0, m1 + 1, dtype=np.int64),
                     offsets=np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64), ids=vid,
                     X=rng.normal(size=(len(vid), n_factors)),
                     ivol=rng.uniform(0.01, 0.03, len(vid)) ** 2 * 21, F=Fm,
                     factors=[f"f{i}" for i in range(n_factors)])
    allm = month_end(np.arange(m0 - 1, m1 + 1))
    wealth = pd.DataFrame({"eom": allm, "wealth": 1e10, "mu_ld1": rng.normal(0.009, 0.04, len(allm))})
    risk_free = pd.DataFrame({"eom": allm, "rf": 0.003})
    return chars, barra, wealth, risk_free
