"""L2 panel preparation (Prepare_Data.py, with the helpers of General_functions.py).

Outputs, identical in schema to the reference:
* ``JKP_US_SP500.db:Factors_processed`` (Prepare_Data.py:488),
* ``wealth_processed.csv`` (:482), ``cluster_labels_processed.csv`` (:485).

Vectorised rewrite: panels are handled as sorted (id, month-index) arrays; the per-id
sequential pieces (rolling add/delete counts, universe state machine) and the cross-sectional
percentile ranks run in the native host runtime (runtime/panel.cpp).
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd

from ..config import Config, get_features
from ..data import io
from .. import runtime as rt
from ..utils.dates import month_index
from ..utils.log import get_logger

log = get_logger("prep")

# Fama-French 12 industries (General_functions.py:293-402), evaluated in this priority order.
_FF12 = [
    ("NoDur", [(100, 999), (2000, 2399), (2700, 2749), (2770, 2799), (3100, 3199), (3940, 3989)], []),
    ("Durbl", [(2500, 2519), (3630, 3659), (3900, 3939), (3990, 3999)],
     [3710, 3711, 3714, 3716, 3750, 3751, 3792]),
    ("Manuf", [(2520, 2589), (2600, 2699), (2750, 2769), (3000, 3099), (3200, 3569), (3580, 3629),
               (3700, 3709), (3712, 3713), (3717, 3749), (3752, 3791), (3793, 3799), (3830, 3839),
               (3860, 3899)], [3715]),
    ("Enrgy", [(1200, 1399), (2900, 2999)], []),
    ("Chems", [(2800, 2829), (2840, 2899)], []),
    ("BusEq", [(3570, 3579), (3660, 3692), (3694, 3699), (3810, 3829), (7370, 7379)], []),
    ("Telcm", [(4800, 4899)], []),
    ("Utils", [(4900, 4949)], []),
    ("Shops", [(5000, 5999), (7200, 7299), (7600, 7699)], []),
    ("Hlth", [(2830, 2839), (3840, 3859), (8000, 8099)], [3693]),
    ("Money", [(6000, 6999)], []),
]


def categorize_sic(sic) -> np.ndarray:
    """Vectorised FF12 mapping; anything unmatched (incl. NaN) is "Other"."""
    s = np.asarray(sic, dtype=np.float64)
    out = np.full(s.shape, "Other", dtype=object)
    done = np.zeros(s.shape, dtype=bool)
    for name, ranges, singles in _FF12:
        m = np.zeros(s.shape, dtype=bool)
        for lo, hi in ranges:
            m |= (s >= lo) & (s <= hi)
        if singles:
            m |= np.isin(s, singles)
        m &= ~done
        out[m] = name
        done |= m
    return out


def wealth_func(wealth_end: float, end: pd.Timestamp, market: pd.DataFrame,
                risk_free: pd.DataFrame) -> pd.DataFrame:
    """Backward wealth path (General_functions.py:175-220; quirk Q4: cumprod(1 - tret))."""
    w = risk_free.rename(columns={"eom": "eom_ret"})[["eom_ret", "rf"]].merge(
        market, on="eom_ret", how="left")
    w["tret"] = w["mkt_vw_exc"] + w["rf"]
    w = w[w["eom_ret"] <= end].sort_values("eom_ret", ascending=False)
    w["wealth"] = (1.0 - w["tret"]).cumprod() * wealth_end
    w["eom"] = w["eom_ret"] + pd.offsets.MonthEnd(0) - pd.offsets.MonthEnd(1)
    res = pd.DataFrame({"eom": w["eom"].values, "wealth": w["wealth"].values,
                        "mu_ld1": w["tret"].values})
    res = pd.concat([res, pd.DataFrame({"eom": [pd.Timestamp(end)], "wealth": [wealth_end],
                                        "mu_ld1": [np.nan]})], ignore_index=True)
    return res.sort_values("eom", kind="stable").reset_index(drop=True)


def lead_returns(monthly: pd.DataFrame, h: int) -> pd.DataFrame:
    """ret_ld1 of long_horizon_ret (General_functions.py:222-288), zero-imputed."""
    return long_horizon_ret(monthly, h, "zero")[["id", "eom", "ret_ld1"]]


def long_horizon_ret(monthly: pd.DataFrame, h: int, impute: str = "zero") -> pd.DataFrame:
    """long_horizon_ret (General_functions.py:222-288): columns id, eom, ret_ld1..ret_ld{h}.

    Builds the dense (id, date) grid between each id's first and last valid return over the
    set of dates present in the data, forms leads 1..h, drops rows with all h leads missing,
    then fills the remaining gaps with zero or the per-eom mean / median of that lead (any
    other ``impute`` leaves them NaN, as the reference does).
    """
    m = monthly.dropna(subset=["ret_exc"])
    mi = month_index(m["eom"])
    ids = m["id"].to_numpy(np.int64)
    dates = np.unique(mi)
    order = np.lexsort((mi, ids))
    ids, mi, ret = ids[order], mi[order], m["ret_exc"].to_numpy(np.float64)[order]
    gs = rt.group_starts(ids)
    uid = ids[gs[:-1]]
    start = mi[gs[:-1]]
    end = mi[gs[1:] - 1]
    a = np.searchsorted(dates, start)
    b = np.searchsorted(dates, end, side="right")
    cnt = b - a
    gid = np.repeat(uid, cnt)
    gdate = dates[np.repeat(a - np.cumsum(np.r_[0, cnt[:-1]]), cnt) + np.arange(cnt.sum())]
    # returns on the grid
    key_data = ids * 100000 + mi
    key_grid = gid * 100000 + gdate
    pos = np.searchsorted(key_data, key_grid)
    pos = np.clip(pos, 0, len(key_data) - 1)
    gret = np.where(key_data[pos] == key_grid, ret[pos], np.nan)
    ggs = np.concatenate([[0], np.cumsum(cnt)])
    n = len(gret)
    leads = np.full((n, h), np.nan)
    idx = np.arange(n)
    grp_end = np.repeat(ggs[1:], cnt)
    for l in range(1, h + 1):
        ok = idx + l < grp_end
        leads[ok, l - 1] = gret[idx[ok] + l]
    all_missing = np.isnan(leads).all(axis=1)
    log.info(f"All missing excludes {all_missing.mean() * 100:.2f}% of the observations")
    keep = ~all_missing
    from ..utils.dates import month_end
    out = pd.DataFrame({"id": gid[keep], "eom": month_end(gdate[keep])})
    lead = pd.DataFrame(leads[keep], columns=[f"ret_ld{l}" for l in range(1, h + 1)])
    if impute == "zero":
        lead = lead.fillna(0.0)
    elif impute in ("mean", "median"):
        lead = lead.fillna(lead.groupby(out["eom"].to_numpy()).transform(impute))
    return pd.concat([out, lead], axis=1)


def size_screen(chars: pd.DataFrame, type_: str) -> None:
    """size_screen_fun (General_functions.py:404-504): adds ``valid_size`` in place."""
    vd = chars["valid_data"].to_numpy(bool)
    if type_ == "all":
        log.info("No size screen")
        chars["valid_size"] = vd
    elif type_.startswith("top") or type_.startswith("bottom"):
        top = type_.startswith("top")
        k = int(type_.replace("top", "").replace("bottom", ""))
        r = chars.loc[vd].groupby("eom")["me"].rank(method="first", ascending=not top)
        rk = pd.Series(np.nan, index=chars.index)
        rk.loc[r.index] = r
        chars["valid_size"] = (rk <= k).to_numpy()
    elif type_.startswith("size_grp_"):
        chars["valid_size"] = (chars["size_grp"] == type_.replace("size_grp_", "")).to_numpy() & vd
    elif "perc" in type_:
        import re
        lo = int(re.search(r"(?<=low)\d+", type_).group(0))
        hi = int(re.search(r"(?<=high)\d+", type_).group(0))
        mn = int(re.search(r"(?<=min)\d+", type_).group(0))
        log.info(f"Percentile-based screening: Range {lo}% - {hi}%, min_n: {mn} stocks")
        pc = chars.loc[vd].groupby("eom")["me"].rank(method="min", pct=True)
        perc = pd.Series(np.nan, index=chars.index)
        perc.loc[pc.index] = pc
        g = chars.assign(_p=perc, _vd=vd).groupby("eom")
        n_tot = g["_vd"].transform("sum")
        base = (perc > lo / 100) & (perc <= hi / 100)
        n_size = base.groupby(chars["eom"]).transform("sum")
        n_less = (chars.assign(_x=vd & (perc <= lo / 100)).groupby("eom")["_x"].transform("sum"))
        n_more = (chars.assign(_x=vd & (perc > hi / 100)).groupby("eom")["_x"].transform("sum"))
        n_miss = (mn - n_size).clip(lower=0)
        n_below = np.ceil(np.minimum(n_miss / 2, n_less)).astype(int)
        n_above = np.ceil(np.minimum(n_miss / 2, n_more)).astype(int)
        adj = (n_below + n_above) < n_miss
        extra = n_miss - n_below - n_above
        n_above = np.where(adj & (n_above > n_below), n_above + extra, n_above)
        n_below = np.where(adj & (n_above < n_below), n_below + extra, n_below)
        chars["valid_size"] = ((perc > lo / 100 - n_below / n_tot) &
                               (perc <= hi / 100 + n_above / n_tot)).to_numpy()
    else:
        raise ValueError(f"Size screen type not recognized: {type_}")


def addition_deletion(chars: pd.DataFrame, addition_n: int, deletion_n: int) -> pd.DataFrame:
    """addition_deletion_fun (General_functions.py:550-699) with native per-id kernels."""
    ids = chars["id"].to_numpy(np.int64)
    o = np.lexsort((month_index(chars["eom"]), ids))
    if (np.diff(o) > 0).all():                         # already (id, eom) ordered (prepare_data)
        chars = chars.copy(deep=False)
    else:
        chars = chars.take(o)
    chars.index = pd.RangeIndex(len(chars))
    vt = (chars["valid_data"].to_numpy(bool) & chars["valid_size"].fillna(False).to_numpy(bool))
    gs = rt.group_starts(chars["id"].to_numpy(np.int64))
    add_cnt = rt.rolling_sum(vt.astype(np.float64), gs, addition_n)
    del_cnt = rt.rolling_sum(vt.astype(np.float64), gs, deletion_n)
    add = add_cnt == addition_n
    delete = del_cnt == 0
    valid = rt.investment_universe(add, delete, gs)
    valid &= chars["valid_data"].to_numpy(bool)
    # turnover diagnostics, raw (valid_temp) vs adjusted (valid)
    first = np.zeros(len(chars), dtype=bool)
    first[gs[:-1]] = True
    prev_vt = np.r_[False, vt[:-1]]
    prev_v = np.r_[False, valid[:-1]]
    chg_raw = np.where(first, 0.0, (vt != prev_vt).astype(float))
    chg_adj = np.where(first, 0.0, (valid != prev_v).astype(float))
    vt_c = np.where(first, 0.0, vt.astype(float))
    v_c = np.where(first, 0.0, valid.astype(float))
    agg = pd.DataFrame({"eom": chars["eom"], "chg_raw": chg_raw, "chg_adj": chg_adj,
                        "vt": vt_c, "v": v_c}).groupby("eom", sort=False).sum()
    agg["raw"] = agg["chg_raw"] / agg["vt"]
    agg["adj"] = agg["chg_adj"] / agg["v"]
    agg = agg[agg["adj"].notna() & (agg["adj"] != 0)]
    log.info(f"Turnover wo addition/deletion rule: {round(agg['raw'].mean() * 100, 2)}%")
    log.info(f"Turnover w  addition/deletion rule: {round(agg['adj'].mean() * 100, 2)}%")
    chars["valid"] = valid
    del chars["valid_data"], chars["valid_size"]
    return chars


def prepare_data(cfg: Config, write: bool = True) -> dict:
    """Run L2 end to end; returns {'chars', 'wealth', 'cluster_labels'}."""
    s, pf = cfg.settings, cfg.pf_set
    dd = cfg.run.data_dir
    features = get_features()
    risk_free = io.read_risk_free(dd)
    log.info("Risk-free Rate Data Complete.")
    market = io.read_market(dd)
    log.info("Market Data Complete.")

    labels = pd.read_csv(io.path(dd, "Cluster Labels.csv"))
    labels["cluster"] = labels["cluster"].str.lower().str.replace(r"[\s-]", "_", regex=True)
    signs = io.read_factor_details(dd)[["abr_jkp", "direction"]].dropna(subset=["abr_jkp"])
    signs = signs.rename(columns={"abr_jkp": "characteristic"})
    signs["direction"] = pd.to_numeric(signs["direction"], errors="coerce")
    labels = signs.merge(labels, on="characteristic", how="right")
    labels = pd.concat([labels, pd.DataFrame({"characteristic": ["rvol_252d"], "direction": [-1],
                                              "cluster": ["low_risk"]})], ignore_index=True)
    log.info("Factor Labels Complete.")

    q = ("SELECT id, eom, sic, ff49, size_grp, me, crsp_exchcd, ret_exc, " + ", ".join(features)
         + " FROM Factors")
    chars = io.sql_read(io.path(dd, "JKP_US_SP500.db"), q, parse_dates={"eom"})
    # only columns that need a conversion are replaced, and all of them in one go: replacing
    # ~130 columns one by one leaves one pandas block per column (PerformanceWarning: highly
    # fragmented) and every later take / filter pays per block
    conv = {f: pd.to_numeric(chars[f], errors="coerce") for f in features + ["sic"]
            if chars[f].dtype != np.float64}
    if chars["id"].dtype != np.int64:
        conv["id"] = chars["id"].astype("int64")
    if len(conv) > 8:
        chars = pd.concat([chars.drop(columns=list(conv)), pd.DataFrame(conv)],
                          axis=1)[list(chars.columns)]
    else:                                   # a few new blocks (sic, id): no full-panel copy
        for c, v in conv.items():
            chars[c] = v
    chars["dolvol"] = chars["dolvol_126d"]
    chars["lambda"] = 2.0 / chars["dolvol"] * s["pi"]
    chars["rvol_m"] = chars["rvol_252d"] * (21 ** 0.5)
    log.info("Chars Data Complete")

    # ---- lead / total returns (Prepare_Data.py:194-233) -------------------------------
    monthly = chars[["id", "eom", "ret_exc"]].copy()
    monthly["ret_exc"] = pd.to_numeric(monthly["ret_exc"], errors="coerce")
    ld = lead_returns(monthly.dropna(), h=s["pf"]["hps"]["m1"]["K"])
    ld["eom_ret"] = ld["eom"] + pd.offsets.MonthEnd(1)
    ld = risk_free.merge(ld, on="eom", how="right")
    ld["tr_ld1"] = ld["ret_ld1"] + ld["rf"]
    ld = ld.drop(columns=["rf"])
    lag = ld[["id", "eom", "tr_ld1"]].rename(columns={"tr_ld1": "tr_ld0"})
    lag["eom"] = lag["eom"] + pd.offsets.MonthEnd(1)
    ld = ld.merge(lag, on=["id", "eom"], how="left")[["id", "eom", "tr_ld0", "eom_ret",
                                                      "ret_ld1", "tr_ld1"]]
    # left merges onto the ~130-column panel as key lookups + column assignments (a merge
    # would copy the whole panel; the left-join semantics - every chars row kept, in order,
    # NaN where (id, eom) has no lead row - are the same; (id, eom) is unique in ld)
    key_c = chars["id"].to_numpy(np.int64) * 100000 + month_index(chars["eom"]).astype(np.int64)
    key_l = ld["id"].to_numpy(np.int64) * 100000 + month_index(ld["eom"]).astype(np.int64)
    pos = pd.Index(key_l).get_indexer(key_c)
    hit = pos >= 0
    add = {}
    for c in ("tr_ld0", "eom_ret", "ret_ld1", "tr_ld1"):
        v = ld[c].to_numpy()[np.where(hit, pos, 0)]
        if c == "eom_ret":
            add[c] = pd.Series(v, index=chars.index).where(hit)
        else:
            add[c] = np.where(hit, v, np.nan)
    log.info("Leading Returns Complete")

    wealth = wealth_func(pf["wealth"], s["split"]["test_end"], market, risk_free)
    ws = wealth[["eom", "mu_ld1"]].rename(columns={"mu_ld1": "mu_ld0"}).copy()
    ws["eom"] = ws["eom"] + pd.offsets.MonthEnd(1)
    wpos = pd.Index(ws["eom"]).get_indexer(chars["eom"])
    add["mu_ld0"] = np.where(wpos >= 0, ws["mu_ld0"].to_numpy()[np.where(wpos >= 0, wpos, 0)],
                             np.nan)
    for c, v in add.items():                # (five new columns: a few blocks, no panel copy)
        chars[c] = v
    log.info("Wealth Evolution Complete.")

    # ---- screens (Prepare_Data.py:268-309): one keep-mask, the panel filtered once --------
    sc = s["screens"]
    keep = np.ones(len(chars), dtype=bool)

    def screen(mask_keep, label):
        m = np.asarray(mask_keep, dtype=bool)
        log.info(f"   {label} excludes {(~m[keep]).mean() * 100:.2f}% of the observations")
        keep[:] = keep & m

    if sc["nyse_stocks"]:
        screen(chars["crsp_exchcd"].to_numpy() == 1, "NYSE stock screen")
    n_start = int(keep.sum())
    me = chars["me"].to_numpy(np.float64)
    me_start = np.nansum(me[keep])
    screen((chars["eom"] >= sc["start"]) & (chars["eom"] <= sc["end"]), "Date screen")
    screen(chars["me"].notna(), "Non-missing me")
    screen(chars["tr_ld1"].notna() & chars["tr_ld0"].notna(), "Valid return req")
    screen(chars["dolvol"].notna() & (chars["dolvol"] > 0), "Non-missing/non-zero dolvol")
    screen(chars["sic"].notna(), "Valid SIC code")
    avail = np.zeros(len(chars), dtype=np.int64)       # column views: no panel copy
    for f in features:
        avail += ~np.isnan(chars[f].to_numpy(np.float64))
    min_feat = np.floor(len(features) * sc["feat_pct"])
    screen(avail >= min_feat, f"At least {sc['feat_pct'] * 100}% of feature")
    log.info(f"In total, the final dataset has {round(int(keep.sum()) / n_start * 100, 2)}% of the "
             f"observations and {round(np.nansum(me[keep]) / me_start * 100, 2)}% of the market cap "
             f"in the post {sc['start']} data")
    # the panel in (id, eom) order, filtered: ONE reorder copy (the reference sorts by
    # (eom, id) for the ranks and back by (id, eom) for the lookback; the ranks below are
    # computed through a permutation instead)
    idx = np.nonzero(keep)[0]
    o = np.lexsort((month_index(chars["eom"].iloc[idx]), chars["id"].to_numpy(np.int64)[idx]))
    chars = chars.take(idx[o])
    chars.index = pd.RangeIndex(len(chars))            # (reset_index would copy the panel again)

    # ---- percentile ranks + imputation (Prepare_Data.py:324-374) ----------------------
    if s["feat_prank"]:
        mi_rows = month_index(chars["eom"]).astype(np.int64)
        pe = np.lexsort((chars["id"].to_numpy(np.int64), mi_rows))      # (eom, id) order
        seg = rt.group_starts(mi_rows[pe])
        # ranks within each month through the permutation, written back in panel order;
        # quirk Q15: exact zeros stay 0; imputation: NaN ranks -> 0.5
        Rb = rt.pct_rank_rows(chars[features].to_numpy(np.float64), pe, seg, zero_keep=True,
                              impute=0.5 if s["feat_impute"] else None)
        chars.loc[:, features] = Rb                    # in place: no per-column blocks
        log.info("Feature Rank Complete.")
        if s["feat_impute"]:
            log.info("Feature Imputation Complete.")
    elif s["feat_impute"]:
        chars[features] = chars.groupby("eom")[features].transform(lambda x: x.fillna(x.median()))
        log.info("Feature Imputation Complete.")
    chars["ff12"] = categorize_sic(chars["sic"].to_numpy()).astype(str)

    # ---- lookback validity, size screen, addition/deletion (Prepare_Data.py:412-453) ---
    lb = pf["lb_hor"] + 1
    gs = rt.group_starts(chars["id"].to_numpy(np.int64))
    mi = month_index(chars["eom"]).astype(np.float64)
    lagged = rt.group_shift(mi, gs, lb)
    diff = mi - lagged
    ok = diff == lb
    log.info(f"   Valid lookback observation screen excludes {round((~ok).mean() * 100, 2)}% of the observations")
    chars["valid_data"] = ok
    size_screen(chars, sc.get("size_screen", "all"))
    chars = addition_deletion(chars, s["addition_n"], s["deletion_n"])
    vpct = round(chars["valid"].mean() * 100, 2)
    mpct = round(chars.loc[chars["valid"], "me"].sum() / chars["me"].sum() * 100, 2)
    log.info(f"   The valid_data subset has {vpct}% of the observations and {mpct}% of the market cap")
    if cfg.run.plots and write:
        universe_plot(chars, os.path.join(dd, "plots"))

    if write:
        io.write_csv(wealth, dd, "wealth_processed.csv")
        io.write_csv(labels, dd, "cluster_labels_processed.csv")
        out = chars.copy(deep=False)                   # (column replacement only)
        out["eom"] = out["eom"].dt.strftime("%Y-%m-%d")
        out["eom_ret"] = out["eom_ret"].dt.strftime("%Y-%m-%d")
        io.sql_write(io.path(dd, "JKP_US_SP500.db"), "Factors_processed", out)
    return {"chars": chars, "wealth": wealth, "cluster_labels": labels}


def universe_counts(chars: pd.DataFrame) -> pd.DataFrame:
    """Valid stocks per month (Prepare_Data.py:459-462)."""
    v = chars.loc[chars["valid"].astype(bool)]
    return v.groupby("eom").size().reset_index(name="N")


@io._io_timed                                             # (figure files: stage I/O time)
def universe_plot(chars: pd.DataFrame, out_dir: str) -> list[str]:
    """The investable-universe figure of Prepare_Data.py:464-471 (valid stocks per eom, a
    scatter with a zero line) as a PNG, plus its data as universe_counts.csv."""
    os.makedirs(out_dir, exist_ok=True)
    vc = universe_counts(chars)
    f0 = os.path.join(out_dir, "universe_counts.csv")
    vc.assign(eom=pd.to_datetime(vc["eom"]).dt.strftime("%Y-%m-%d")).to_csv(f0, index=False)
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        log.info("matplotlib not available: universe plot skipped")
        return [f0]
    fig = plt.figure(figsize=(10, 6))
    plt.scatter(pd.to_datetime(vc["eom"]), vc["N"])
    plt.xlabel("eom")
    plt.ylabel("Valid stocks")
    plt.axhline(y=0, color="grey", linestyle="--")
    plt.title("Investable Universe Over Time")
    f1 = os.path.join(out_dir, "investable_universe.png")
    fig.savefig(f1, dpi=100)
    plt.close(fig)
    return [f0, f1]
