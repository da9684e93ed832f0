"""L6/L7 portfolio construction and reporting.

* ``aim_portfolios``   - PFML_aim_fun.py:130-163: December rank-1 hyper-parameters per g,
                         w_aim = s_t beta (K18), coefficients of year oos_year (quirk Q13);
* ``hps_bundle``       - PFML_hps.py: {g: {aim_pfs_list, validation, rff_w}};
* ``best_hps``         - PFML_best_hps.py:263-308: cross-g rank-first selection;
* ``pfml_weights``     - PFML_best_hps.py:137-218: value-weighted start, weight recursion (17)
                         w_t = m_t w_start + (I - m_t) w_aim with all m_t computed as ONE batched
                         device m_func (K19) and the sequential part reduced to GEMVs;
* ``pf_ts`` / ``pf_summary`` - :220-259, :326-358 (quirks Q3, Q18);
* ``plots``            - cumulative-performance / hyper-parameter figures (matplotlib).
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd
import torch

from ..config import Config
from ..ops import linalg as la
from ..ops.gemm import gemm
from ..utils.dates import month_end, month_index
from ..utils.log import get_logger
from .risk import BarraCov

log = get_logger("portfolio")


def _opt_hps(validation: pd.DataFrame, g: int) -> pd.DataFrame:
    v = validation[validation["g"] == g]
    er = pd.to_datetime(v["eom_ret"])
    sel = v[(er.dt.month == 12).to_numpy() & (v["rank"] == 1).to_numpy()]
    return pd.DataFrame({"hp_end": pd.to_datetime(sel["eom_ret"]).dt.year.to_numpy(),
                         "l": sel["l"].to_numpy(), "p": sel["p"].to_numpy()})


def aim_portfolios(cfg: Config, validation: pd.DataFrame, beta_years: np.ndarray,
                   beta: torch.Tensor, signal_months: np.ndarray, signal_t: list,
                   signal_ids: list, oos_months: np.ndarray) -> dict:
    """{g: {d: {'aim_pf': DataFrame(id, eom, w_aim), 'coef': ndarray}}} (internal order)."""
    G = beta.shape[0]
    p_vec = cfg.p_vec
    out = {}
    mpos = {int(m): i for i, m in enumerate(signal_months)}
    for g in range(G):
        opt = _opt_hps(validation, g)
        res = {}
        for d in oos_months:
            oos_year = int(month_end(int(d) + 1).year[0])
            row = opt[opt["hp_end"] == oos_year - 1]
            if row.empty:
                raise KeyError(f"no December rank-1 hyper-parameters for {oos_year - 1}")
            p, l = int(row["p"].iloc[0]), int(row["l"].iloc[0])
            yi = int(np.nonzero(beta_years == oos_year)[0][0])
            coef = beta[g, yi, p_vec.index(p), l, : p + 1]
            i = mpos[int(d)]
            s = signal_t[g][i][:, : p + 1]
            w_aim = (s @ coef.to(s.device)).cpu().numpy()
            res[int(d)] = {"aim_pf": pd.DataFrame({"id": signal_ids[i],
                                                   "eom": month_end(int(d))[0],
                                                   "w_aim": w_aim}),
                           "coef": coef.cpu().numpy(), "p": p, "l": l}
        out[g] = res
    return out


def hps_bundle(aims: dict, validation: pd.DataFrame, rff_w: np.ndarray) -> dict:
    return {g: {"aim_pfs_list": aims[g], "validation": validation[validation["g"] == g],
                "rff_w": rff_w[g]} for g in aims}


def best_hps(hps: dict, oos_months: np.ndarray):
    """Cross-g selection: rank 'first' by cum_obj within eom_ret, December rank 1."""
    bh = pd.concat([h["validation"] for h in hps.values()], ignore_index=True).drop(columns="rank")
    bh["eom"] = pd.to_datetime(bh["eom"])
    bh["eom_ret"] = pd.to_datetime(bh["eom_ret"])
    bh["rank"] = bh.groupby("eom_ret")["cum_obj"].rank(ascending=False, method="first")
    bh = bh[(bh["rank"] == 1) & (bh["eom_ret"].dt.month == 12)]
    chosen, aims = {}, []
    for d in oos_months:
        oos_year = int(month_end(int(d) + 1).year[0])
        sel = bh[bh["eom_ret"].dt.year == oos_year - 1]
        g = int(sel["g"].iloc[0])
        a = hps[g]["aim_pfs_list"][int(d)]
        chosen[int(d)] = {"g": g, "p": int(sel["p"].iloc[0]), "aim": a["aim_pf"], "coef": a["coef"]}
        aims.append(a["aim_pf"])
    return bh, chosen, pd.concat(aims, ignore_index=True)


def pfml_weights(cfg: Config, chars: pd.DataFrame, barra: BarraCov, wealth: pd.DataFrame,
                 risk_free: pd.DataFrame, aims: pd.DataFrame, oos_months: np.ndarray,
                 device) -> pd.DataFrame:
    """Weight recursion (17) (PFML_best_hps.py:168-218) -> weights.csv frame."""
    dev = torch.device(device)
    pf = cfg.pf_set
    gamma, mu = float(pf["gamma_rel"]), float(pf["mu"])
    tc_on = bool(cfg.settings["Transaction_Costs"])
    mi_all = month_index(chars["eom"])
    data = chars[np.isin(mi_all, oos_months) & chars["valid"].to_numpy()].copy()
    data["mi"] = month_index(data["eom"])
    data = data.sort_values(["mi", "id"], kind="stable").reset_index(drop=True)
    wmap = dict(zip(month_index(wealth["eom"]), wealth["wealth"].to_numpy(np.float64)))
    mumap = dict(zip(month_index(wealth["eom"]), wealth["mu_ld1"].to_numpy(np.float64)))
    rfmap = dict(zip(month_index(risk_free["eom"]), risk_free["rf"].to_numpy(np.float64)))
    aim_key = month_index(aims["eom"]) * 10_000_000 + aims["id"].to_numpy(np.int64)
    aim_val = dict(zip(aim_key, aims["w_aim"].to_numpy(np.float64)))

    months = np.asarray(oos_months, np.int64)
    groups = [data.index[data["mi"] == d].to_numpy() for d in months]
    ns = np.array([len(g) for g in groups])
    N = int(ns.max())
    B = len(months)
    K = barra.X.shape[1]
    # ---- batched m_t for every OOS month (K19) --------------------------------------
    ms = []
    chunk = int(cfg.run.month_batch)
    if chunk <= 0:
        from .pfml_inputs import auto_month_batch
        chunk = auto_month_batch(N, 0, dev)
    for c0 in range(0, B, chunk):
        cm = months[c0:c0 + chunk]
        Bc = len(cm)
        Xl = torch.zeros((Bc, N, K), dtype=torch.float64, device=dev)
        Fb = torch.zeros((Bc, K, K), dtype=torch.float64, device=dev)
        iv = torch.ones((Bc, N), dtype=torch.float64, device=dev)
        lam = torch.empty((Bc, N), dtype=torch.float64, device=dev)
        mask = torch.zeros((Bc, N), dtype=torch.float64, device=dev)
        for bi, d in enumerate(cm):
            rows = groups[c0 + bi]
            ids = data["id"].to_numpy(np.int64)[rows]
            bids, X, F, ivol = barra.slice(int(d))
            pos = np.searchsorted(bids, ids)
            n = len(ids)
            Xl[bi, :n] = torch.as_tensor(X[pos], device=dev)
            Fb[bi] = torch.as_tensor(F, device=dev)
            iv[bi, :n] = torch.as_tensor(ivol[pos], device=dev)
            lam[bi] = gamma / wmap[int(d)]
            lam_d = data["lambda"].to_numpy(np.float64)[rows] if tc_on else np.full(n, 1e-16)
            lam[bi, :n] = torch.as_tensor(lam_d, device=dev)
            mask[bi, :n] = 1.0
        Sig = gemm(gemm(Xl, Fb), Xl, trans_b=True)
        Sig.diagonal(dim1=1, dim2=2).add_(iv)
        wv = torch.as_tensor([wmap[int(d)] for d in cm], dtype=torch.float64, device=dev)
        rfv = torch.as_tensor([rfmap[int(d)] for d in cm], dtype=torch.float64, device=dev)
        ms.append(la.m_func(Sig, lam, wv, rfv, mu, gamma, cfg.run.iterations, mask=mask))
    m_all = torch.cat(ms)

    # ---- sequential recursion -------------------------------------------------------
    ids_all = data["id"].to_numpy(np.int64)
    me = data["me"].to_numpy(np.float64)
    tr1 = data["tr_ld1"].to_numpy(np.float64)
    w_start = np.full(len(data), np.nan)
    w = np.full(len(data), np.nan)
    g0 = groups[0]
    w_start[g0] = me[g0] / me[g0].sum()                   # value-weighted initial portfolio
    for t, d in enumerate(months):
        rows = groups[t]
        n = len(rows)
        key = int(d) * 10_000_000 + ids_all[rows]
        w_aim = np.array([aim_val.get(int(k), np.nan) for k in key])
        mt = m_all[t, :n, :n]
        ws = torch.as_tensor(w_start[rows], dtype=torch.float64, device=dev)
        wa = torch.as_tensor(w_aim, dtype=torch.float64, device=dev)
        w_opt = (wa + mt @ (ws - wa)).cpu().numpy()
        w[rows] = w_opt
        if t + 1 < B:
            nxt = groups[t + 1]
            nxt_ids = ids_all[nxt]
            drift = w_opt * (1.0 + tr1[rows]) / (1.0 + mumap[int(d)])
            pos = np.searchsorted(ids_all[rows], nxt_ids)
            pos = np.clip(pos, 0, n - 1)
            hit = ids_all[rows][pos] == nxt_ids
            w_start[nxt] = np.where(hit, drift[pos], 0.0)   # new names start at 0
    out = pd.DataFrame({"eom": month_end(data["mi"].to_numpy()),
                        "mu_ld1": [mumap[int(x)] for x in data["mi"]],
                        "id": ids_all, "tr_ld1": tr1, "w_start": w_start, "w": w})
    return out


def pf_ts(weights: pd.DataFrame, chars: pd.DataFrame, wealth: pd.DataFrame,
          compat: bool = True) -> pd.DataFrame:
    """Per-month portfolio statistics (PFML_best_hps.py:220-259)."""
    comb = chars[["id", "eom", "ret_ld1", "lambda"]].merge(weights, on=["id", "eom"], how="inner")
    comb = comb.merge(wealth[["eom", "wealth"]], on="eom", how="left")
    dw = comb["w"] - comb["w_start"]
    comb = comb.assign(absw=comb["w"].abs(), shortw=comb["w"].clip(upper=0).abs(),
                       to=dw.abs(), rr=comb["w"] * comb["ret_ld1"],
                       lam_dw2=comb["lambda"] * dw * dw)
    g = comb.groupby("eom")
    res = pd.DataFrame({"inv": g["absw"].sum(), "shorting": g["shortw"].sum(),
                        "turnover": g["to"].sum(), "r": g["rr"].sum(),
                        "tc": g["wealth"].first() / 2.0 * g["lam_dw2"].sum()}).reset_index()
    if compat:
        # quirk Q3: (eom + 1M).to_period('M').to_timestamp('M') - MonthEnd(1) == eom
        res["eom_ret"] = res["eom"]
    else:
        res["eom_ret"] = res["eom"] + pd.offsets.MonthEnd(1)
    return res.drop(columns=["eom"])


def pf_summary(pf: pd.DataFrame, gamma: float) -> pd.DataFrame:
    """Annualised summary (PFML_best_hps.py:326-358; ddof = 1, quirk Q18)."""
    r, tc = pf["r"], pf["tc"]
    sd = r.std(ddof=1)
    return pd.DataFrame([{
        "type": "Portfolio-ML", "n": int(r.count()), "inv": pf["inv"].mean(),
        "shorting": pf["shorting"].mean(), "turnover_notional": pf["turnover"].mean(),
        "r": r.mean() * 12, "sd": sd * np.sqrt(12), "sr_gross": r.mean() / sd * np.sqrt(12),
        "tc": tc.mean() * 12, "r_tc": (r - tc).mean() * 12,
        "sr": (r - tc).mean() / sd * np.sqrt(12),
        "obj": (r.mean() - 0.5 * r.var(ddof=1) * gamma - tc.mean()) * 12}])


def plots(pf: pd.DataFrame, best: pd.DataFrame, gamma: float, out_dir: str) -> list[str]:
    """Cumulative performance and chosen hyper-parameters (PFML_best_hps.py:281-291,361-422)."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        log.info("matplotlib not available: plots skipped")
        return []
    os.makedirs(out_dir, exist_ok=True)
    p = pf.sort_values("eom_ret").copy()
    p["e_var_adj"] = (p["r"] - p["r"].mean()) ** 2
    p["utility_t"] = p["r"] - p["tc"] - 0.5 * p["e_var_adj"] * gamma
    fig, ax = plt.subplots(1, 3, figsize=(14, 4))
    for a, (col, title) in zip(ax, [(p["r"].cumsum(), "Gross return"),
                                    ((p["r"] - p["tc"]).cumsum(), "Return net of TC"),
                                    (p["utility_t"].cumsum(), "Return net of TC and Risk")]):
        a.plot(pd.to_datetime(p["eom_ret"]), col)
        a.set_title(title)
    f1 = os.path.join(out_dir, "cumulative_performance.png")
    fig.savefig(f1, dpi=100)
    plt.close(fig)
    fig, ax = plt.subplots(3, 1, figsize=(8, 7), sharex=True)
    for a, c in zip(ax, ["p", "l", "g"]):
        a.plot(best["eom_ret"], best[c], "o-", alpha=0.6)
        a.set_ylabel(c)
    f2 = os.path.join(out_dir, "top_hyperparameters.png")
    fig.savefig(f2, dpi=100)
    plt.close(fig)
    return [f1, f2]
