"""L3 Barra risk model (Estimate Covariance Matrix.py + General_functions.py:715-835).

Pipeline, batched instead of per-day / per-month Python loops:

1. cluster ranks (K25): a masked GEMM of the ranked characteristics with a signed membership
   matrix (direction -1 columns enter as 1 - x), then a per-month z-score;
2. daily cross-sectional OLS (K21): rows sorted by trading day into CSR day segments, one
   workgroup per day on the device (csrc/risk.hip: [X|y]'[X|y] on MFMA, pivoted LU, residuals),
   pinv fallback for exactly singular days (:224-229) - instead of a full-array mask scan per day (the reference's ~182 s hot spot);
3. EWMA factor covariance (K22): one workgroup per month-end over its trailing window of
   daily factor returns (csrc/risk.hip): the weighted, unbiased cov.wt / cor.wt of
   General_functions.py:745-835 and F = sd cor sd * 21 fused;
4. EWMA idiosyncratic vol (K23): csrc/risk.hip wave-per-stock affine scan on the device
   (runtime/panel.cpp sequential scan on the CPU path), then the >= 200-of-252-days filter and the last observation per month;
5. Barra assembly (:453-494): size-group median imputation, F * 21, ivol = res_vol^2 * 21.

Output: ``BarraCov`` - per month-end the sorted ids, loadings X (N x K), factor cov F (K x K,
monthly) and idiosyncratic variances; ``create_cov`` (K1) builds Sigma = X F X' + diag(ivol).
"""
from __future__ import annotations

import os
import warnings
from dataclasses import dataclass

import numpy as np
import pandas as pd
import torch

from ..config import Config, get_features
from ..data import io
from .. import runtime as rt
from ..utils.dates import month_end, month_index
from ..utils.log import COUNTERS, get_logger

log = get_logger("risk")
warnings.simplefilter("ignore", category=pd.errors.PerformanceWarning)


@dataclass
class BarraCov:
    months: np.ndarray          # [M] month indices (calc dates), ascending
    offsets: np.ndarray         # [M+1] CSR offsets into the row arrays
    ids: np.ndarray             # [R] stock ids, sorted within each month
    X: np.ndarray               # [R, K] factor loadings
    ivol: np.ndarray            # [R] idiosyncratic variance (monthly)
    F: np.ndarray               # [M, K, K] factor covariance (monthly)
    factors: list               # factor names (industries, then clusters)

    def month_pos(self, mi: int) -> int:
        p = int(np.searchsorted(self.months, mi))
        if p >= len(self.months) or self.months[p] != mi:
            raise KeyError(f"no Barra covariance for month {month_end(mi)[0].date()}")
        return p

    def slice(self, mi: int):
        p = self.month_pos(mi)
        a, b = self.offsets[p], self.offsets[p + 1]
        return self.ids[a:b], self.X[a:b], self.F[p], self.ivol[a:b]

    def save(self, path: str) -> None:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        np.savez(path, months=self.months, offsets=self.offsets, ids=self.ids, X=self.X,
                 ivol=self.ivol, F=self.F, factors=np.asarray(self.factors, dtype="U64"))

    @classmethod
    def load(cls, path: str) -> "BarraCov":
        z = np.load(path, allow_pickle=False)
        return cls(z["months"], z["offsets"], z["ids"], z["X"], z["ivol"], z["F"],
                   [str(f) for f in z["factors"]])


def create_cov(barra: BarraCov, mi: int, ids=None) -> tuple[np.ndarray, np.ndarray]:
    """Sigma = X F X' + diag(ivol) for month ``mi`` (General_functions.py:847-897), optionally
    restricted to ``ids`` (in the given order).  Returns (ids, Sigma)."""
    mids, X, F, iv = barra.slice(mi)
    if ids is not None:
        pos = np.searchsorted(mids, ids)
        if np.any(pos >= len(mids)) or np.any(mids[np.clip(pos, 0, len(mids) - 1)] != ids):
            raise KeyError("create_cov: ids not in the Barra universe of this month")
        X, iv, mids = X[pos], iv[pos], np.asarray(ids)
    sigma = X @ F @ X.T + np.diag(iv)
    if np.min(np.diag(sigma)) < 0:                       # quirk Q7: warn, no repair
        log.warning("Warning: Negative Variances")
        COUNTERS.add("risk.negative_variance")
    return mids, sigma


# ---------------------------------------------------------------------------------------
def cluster_ranks(chars: pd.DataFrame, labels: pd.DataFrame, features: list[str]):
    """Row-mean of each cluster's member ranks, direction -1 flipped as 1 - x."""
    clusters = labels["cluster"].unique().tolist()
    feats = [f for f in features]
    fidx = {f: i for i, f in enumerate(feats)}
    K = len(clusters)
    M = np.zeros((len(feats), K))
    flip = np.zeros(len(feats), dtype=bool)
    for ci, cl in enumerate(clusters):
        sub = labels[(labels["cluster"] == cl) & labels["characteristic"].isin(feats)]
        members = sub["characteristic"].tolist()
        if not members:
            continue
        for c, dirv in zip(sub["characteristic"], sub["direction"]):
            M[fidx[c], ci] = 1.0 / len(members)
            if dirv == -1:
                flip[fidx[c]] = True
    X = chars[feats].to_numpy(np.float64)
    X = np.where(flip[None, :], 1.0 - X, X)
    R = X @ M
    empty = M.sum(0) == 0
    R[:, empty] = np.nan
    return clusters, R


def weighted_cov(X: torch.Tensor, w: torch.Tensor, cor: bool) -> torch.Tensor:
    """Batched R cov.wt(..., method='unbiased') [and cor=TRUE] (General_functions.py:745-835).

    X: [B, T, K], w: [B, T] (zero weight = padding)."""
    wn = w / w.sum(1, keepdim=True)
    mu = (wn.unsqueeze(-1) * X).sum(1, keepdim=True)
    Xw = (X - mu) * wn.sqrt().unsqueeze(-1)
    cov = Xw.transpose(1, 2) @ Xw / (1.0 - (wn * wn).sum(1)).view(-1, 1, 1)
    if not cor:
        return cov
    sd = torch.sqrt(torch.diagonal(cov, dim1=1, dim2=2))
    c = cov / (sd.unsqueeze(-1) * sd.unsqueeze(-2))
    idx = torch.arange(c.shape[-1])
    c[:, idx, idx] = 1.0
    return c


def daily_ols(X: np.ndarray, y: np.ndarray, day: np.ndarray, device) -> tuple:
    """Per-day OLS without intercept (Estimate Covariance Matrix.py:193-264).

    Rows must be sorted by ``day``; each day is a CSR segment (no full-array mask scan per
    day).  Device: csrc/risk.hip daily_ols_kernel (Z'Z on MFMA + pivoted LU per day, pinv
    fallback for exactly singular days).  Returns (unique days, coef [D, K], residuals [R],
    number of pinv fallbacks)."""
    from ..ops.risk_kernels import daily_ols as _ols
    gs = rt.group_starts(day.astype(np.int64))
    dev = torch.device(device)
    Xt = torch.as_tensor(np.ascontiguousarray(X, np.float64), device=dev)
    yt = torch.as_tensor(np.ascontiguousarray(y, np.float64), device=dev)
    coef, resid, nbad = _ols(Xt, yt, torch.as_tensor(gs))
    return day[gs[:-1]], coef.cpu().numpy(), resid.cpu().numpy(), nbad


def estimate_cov(cfg: Config, device: str = "cpu", write: bool = True) -> BarraCov:
    s = cfg.settings
    cs = s["cov_set"]
    dd = cfg.run.data_dir
    features = get_features()
    chars = io.read_processed_chars(dd, features)
    chars = chars.loc[chars["valid"], ["id", "eom", "size_grp", "ff12"] + features]
    chars = chars.sort_values(["eom", "id"], kind="stable").reset_index(drop=True)
    daily = io.sql_read(io.path(dd, "crsp_daily_SP500.db"),
                        "SELECT permno as id, date, ret_excess as ret_exc FROM d_ret_ex",
                        parse_dates={"date"})
    valid_ids = chars["id"].unique()
    daily = daily[daily["ret_exc"].notna() & daily["id"].isin(valid_ids)].copy()
    labels = pd.read_csv(io.path(dd, "cluster_labels_processed.csv"))

    clusters, R = cluster_ranks(chars, labels, features)
    log.info(f"Cluster Labels are the following {clusters}")
    cm = chars[["id", "eom", "size_grp", "ff12"]].copy()
    cm["eom_ret"] = cm["eom"] + pd.offsets.MonthEnd(1)
    industries = sorted(cm["ff12"].dropna().unique())
    for ind in industries:
        cm[str(ind)] = (cm["ff12"] == ind).astype(np.int64)
    # z-score clusters per month (ddof = 1)
    Rdf = pd.DataFrame(R, columns=clusters)
    Rz = Rdf.groupby(cm["eom"].values).transform(lambda x: (x - x.mean()) / x.std())
    for c in clusters:
        cm[c] = Rz[c].to_numpy()
    factor_cols = [str(i) for i in industries] + clusters
    log.info("Cluster Ranks Completed.")

    # ---- daily merge with previous month's exposures (:168-183) ----------------------
    daily = daily[daily["date"] >= cm["eom"].min()]
    daily["eom_ret"] = daily["date"] + pd.offsets.MonthEnd(0)
    dm = cm.merge(daily[["id", "date", "ret_exc", "eom_ret"]], how="inner", on=["id", "eom_ret"])
    dm = dm.dropna()
    dm = dm.sort_values(["date", "id"], kind="stable").reset_index(drop=True)
    dnum = dm["date"].values.astype("datetime64[D]").astype(np.int64)
    days, coef, resid, nbad = daily_ols(dm[factor_cols].to_numpy(np.float64),
                                        dm["ret_exc"].to_numpy(np.float64), dnum, device)
    log.info(f"Factor Returns Completed ({len(days)} days, {nbad} pinv fallbacks).")

    # ---- EWMA factor covariance per calc month (:275-338) --------------------------
    obs = int(cs["obs"])
    tr = np.arange(obs, 0, -1, dtype=np.float64)
    w_cor = (0.5 ** (1.0 / cs["hl_cor"])) ** tr
    w_var = (0.5 ** (1.0 / cs["hl_var"])) ** tr
    if len(days) <= obs:
        raise ValueError(f"need more than {obs} factor-return days, have {len(days)}")
    day_dt = days.astype("datetime64[D]")
    ref = pd.Timestamp(day_dt[obs])
    min_date = ref.to_period("M").to_timestamp() - pd.offsets.MonthEnd(1)
    calc = np.sort(cm.loc[cm["eom"] >= min_date, "eom"].unique())
    calc_mi = month_index(calc)
    end_idx = np.searchsorted(day_dt, np.asarray(calc, dtype="datetime64[D]"), side="right")
    dev = torch.device(device)
    from ..ops.risk_kernels import ewma_factor_cov, ewma_vol as _ewma_vol
    fr = torch.as_tensor(coef, dtype=torch.float64, device=dev)
    Fm = ewma_factor_cov(fr, end_idx, obs, w_cor, w_var, scale=21.0).cpu().numpy()

    # ---- idiosyncratic EWMA vol (:345-442) -----------------------------------------
    sr = pd.DataFrame({"id": dm["id"].to_numpy(np.int64), "date": dnum, "residual": resid})
    sr = sr.sort_values(["id", "date"], kind="stable").reset_index(drop=True)
    gs = rt.group_starts(sr["id"].to_numpy())
    lam = 0.5 ** (1.0 / cs["hl_stock_var"])
    rv = _ewma_vol(torch.as_tensor(sr["residual"].to_numpy(), device=dev), gs, lam,
                   int(cs["initial_var_obs"]))
    sr["res_vol"] = rv.cpu().numpy()
    td = pd.Series(days)
    td252 = pd.DataFrame({"date": days, "td_252d": td.shift(252).to_numpy()})
    sr = sr.merge(td252, on="date", how="left")
    sr["date_200d"] = rt.group_shift(sr["date"].to_numpy(np.float64), gs, 200)
    sr = sr[(sr["date_200d"] >= sr["td_252d"]) & sr["res_vol"].notna()]
    d_eom = month_index(sr["date"].to_numpy().astype("datetime64[D]"))
    sr = sr.assign(mi=d_eom)
    last = sr.groupby(["id", "mi"])["date"].transform("max")
    srm = sr[sr["date"] == last][["id", "mi", "res_vol"]]

    # ---- Barra assembly (:453-494) ---------------------------------------------------
    cm["mi"] = month_index(cm["eom"])
    ids_l, X_l, iv_l, off = [], [], [], [0]
    for mi in calc_mi:
        cd = cm[cm["mi"] == mi].merge(srm, on=["id", "mi"], how="left")
        med = cd.groupby("size_grp")["res_vol"].transform(lambda x: x.median(skipna=True))
        if med.isna().any():
            med = med.fillna(cd["res_vol"].median(skipna=True))
        cd["res_vol"] = cd["res_vol"].fillna(med)
        cd = cd.sort_values("id", kind="stable")
        ids_l.append(cd["id"].to_numpy(np.int64))
        X_l.append(cd[factor_cols].to_numpy(np.float64))
        iv_l.append(cd["res_vol"].to_numpy(np.float64) ** 2 * 21.0)
        off.append(off[-1] + len(cd))
    barra = BarraCov(months=calc_mi.astype(np.int64), offsets=np.asarray(off, np.int64),
                     ids=np.concatenate(ids_l), X=np.concatenate(X_l), ivol=np.concatenate(iv_l),
                     F=Fm, factors=factor_cols)
    log.info(f"Barra covariance for {len(calc_mi)} months, K = {len(factor_cols)} factors.")
    if write:
        barra.save(os.path.join(dd, "Barra_Cov.npz"))
    return barra
