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

    @io._io_timed                                         # (file output: stage I/O time)
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
    # direction -1 members enter as 1 - x: folded into the weights, (1 - x) m = m - x m, so
    # the panel is not copied ( R = X (s o M) + sum_flipped M, s = -1 on flipped rows )
    sgn = np.where(flip, -1.0, 1.0)[:, None]
    R = X @ (sgn * M) + M[flip].sum(0)[None, :]
    empty = M.sum(0) == 0
    R[:, empty] = np.nan
    return clusters, R


def weighted_cov(X: torch.Tensor, w: torch.Tensor, cor: bool,
                 nan_cor: bool = False) -> torch.Tensor:
    """Batched R cov.wt(..., method='unbiased') [and cor=TRUE] (General_functions.py:745-835).

    X: [B, T, K], w: [B, T] (zero weight = padding).  A zero-variance column's correlations:
    0 (default) or, with ``nan_cor`` (compat mode), 0 / 0 = NaN as weighted_cor_wt divides."""
    wn = w / w.sum(1, keepdim=True)
    mu = (wn.unsqueeze(-1) * X).sum(1, keepdim=True)
    Xw = (X - mu) * wn.sqrt().unsqueeze(-1)
    cov = Xw.transpose(1, 2) @ Xw / (1.0 - (wn * wn).sum(1)).view(-1, 1, 1)
    if not cor:
        return cov
    sd = torch.sqrt(torch.diagonal(cov, dim1=1, dim2=2))
    den = sd.unsqueeze(-1) * sd.unsqueeze(-2)
    if nan_cor:
        c = cov / den
    else:
        # zero-variance factor (no exposure in the window): correlations 0, as csrc/risk.hip
        c = torch.where(den > 0, cov / torch.where(den > 0, den, 1.0), torch.zeros_like(cov))
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


def _load_risk_inputs(cfg: Config):
    """Factors_processed (valid rows), the daily excess returns of those ids and the cluster
    labels (Estimate Covariance Matrix.py:50-100)."""
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
    return chars, daily, labels


def estimate_cov(cfg: Config, device: str = "cpu", write: bool = True) -> BarraCov:
    """S3 (Estimate Covariance Matrix.py): load, ``estimate_cov_frames``, write Barra_Cov."""
    chars, daily, labels = _load_risk_inputs(cfg)
    # compat mode: a zero-variance factor's NaN correlations as the reference computes them
    barra = estimate_cov_frames(chars, daily, labels, cfg.settings["cov_set"], device,
                                nan_cor=bool(cfg.run.compat_mode))
    log.info(f"Barra covariance for {len(barra.months)} months, K = {len(barra.factors)} "
             f"factors.")
    if write:
        barra.save(os.path.join(cfg.run.data_dir, "Barra_Cov.npz"))
    return barra


def _seg_zscore(X: torch.Tensor, g: torch.Tensor, G: int) -> torch.Tensor:
    """(x - mean) / std per group g of the rows, column-wise, NaN skipped, ddof = 1 (pandas
    groupby transform of ``(x - x.mean()) / x.std()``; two-pass like nanops.nanvar)."""
    ok = torch.isfinite(X)
    Xz = torch.where(ok, X, torch.zeros_like(X))
    okf = ok.to(X.dtype)
    cnt = torch.zeros((G, X.shape[1]), dtype=X.dtype, device=X.device).index_add_(0, g, okf)
    sm = torch.zeros_like(cnt).index_add_(0, g, Xz)
    mean = sm / cnt
    dev = (X - mean[g])
    ss = torch.zeros_like(cnt).index_add_(0, g, torch.where(ok, dev * dev, torch.zeros_like(X)))
    std = torch.sqrt(ss / (cnt - 1.0))
    std = torch.where(cnt > 1.0, std, torch.full_like(std, float("nan")))
    return dev / std[g]


def _seg_median(v: torch.Tensor, g: torch.Tensor, G: int) -> torch.Tensor:
    """Median of the non-NaN values of each group (pandas median: mean of the two middle
    values; NaN for an all-NaN / empty group) via two stable sorts on the device."""
    key = torch.where(torch.isnan(v), torch.full_like(v, float("inf")), v)
    o1 = torch.sort(key, stable=True).indices
    o2 = torch.sort(g[o1], stable=True).indices
    order = o1[o2]
    sv = v[order]
    size = torch.zeros(G, dtype=torch.int64, device=v.device).index_add_(
        0, g, torch.ones_like(g))
    cnt = torch.zeros(G, dtype=torch.int64, device=v.device).index_add_(
        0, g, (~torch.isnan(v)).to(torch.int64))
    start = torch.cumsum(size, 0) - size
    lo = start + torch.clamp(cnt - 1, min=0) // 2
    hi = start + cnt // 2
    last = max(len(v) - 1, 0)
    med = 0.5 * (sv[lo.clamp(max=last)] + sv[hi.clamp(max=last)])
    return torch.where(cnt > 0, med, torch.full_like(med, float("nan")))


def _zero_exposureless(Fm: np.ndarray, coef: torch.Tensor, end_idx, obs: int) -> None:
    """Compat NaN correlations only where the reference has them.

    A factor without exposure on every day of a window comes out of the pinv fallback
    (Estimate Covariance Matrix.py:228-229) as exactly 0 in the device Jacobi pinv, but as
    LAPACK rounding noise (|c| ~ 1e-17) in the reference's numpy.linalg.pinv, so the
    reference's weighted_cor_wt divides noise by noise: finite correlations and F entries
    ~1e-34.  Such a factor's F row / column is set to 0 here (equal to the reference's to any
    tolerance); a factor with exposure and exactly constant returns keeps its NaN."""
    nz = (coef != 0).to(torch.int64).cumsum(0).cpu().numpy()
    nz = np.vstack([np.zeros((1, nz.shape[1]), np.int64), nz])
    e = np.asarray(end_idx, np.int64)
    cnt = nz[e] - nz[np.maximum(e - obs, 0)]                  # nonzero coefficient days
    for b, k in zip(*np.nonzero(cnt == 0)):
        Fm[b, k, :] = 0.0
        Fm[b, :, k] = 0.0


def estimate_cov_frames(chars: pd.DataFrame, daily: pd.DataFrame, labels: pd.DataFrame,
                        cs: dict, device: str = "cpu", nan_cor: bool = True) -> BarraCov:
    """The Barra model from in-memory frames, batched end to end (no per-day / per-month
    Python loop, no groupby lambda, no frame merges over the daily panel):

    * cluster ranks (K25): one GEMM; the per-month z-score of the clusters (:155-158) as a
      segmented two-pass mean / std on the device (``_seg_zscore``);
    * the daily <- previous-month exposure merge (:168-183) by integer (id, month) keys and a
      sorted search, exposures gathered on the device;
    * daily OLS (K21), EWMA factor cov (K22), EWMA idio vol (K23): csrc/risk.hip;
    * the >= 200-of-252-days filter and last observation per month (:409-439) on index arrays;
    * Barra assembly (:453-494) for all calc months at once: size-group medians and the
      month-median fallback as segmented device medians (``_seg_median``, K27).
    ``estimate_cov_frames_pandas`` is the previous, pandas-bound form (test oracle)."""
    from ..ops.risk_kernels import daily_ols as _ols, ewma_factor_cov, ewma_vol as _ewma_vol
    from ..ops.ridge import _HostClock
    th = _HostClock()                                   # PFML_HOST_TIMING=1: section times
    dev = torch.device(device)
    f64 = dict(dtype=torch.float64, device=dev)
    features = get_features()
    ids_m = chars["id"].to_numpy(np.int64)
    mi_m = month_index(chars["eom"])
    srt = (mi_m * (1 << 32) + ids_m) if len(ids_m) else mi_m
    if not (np.all(srt[1:] >= srt[:-1]) and isinstance(chars.index, pd.RangeIndex)
            and chars.index.start == 0 and chars.index.step == 1):
        chars = chars.sort_values(["eom", "id"], kind="stable").reset_index(drop=True)
        ids_m = chars["id"].to_numpy(np.int64)
        mi_m = month_index(chars["eom"])
    clusters, R = cluster_ranks(chars, labels, features)
    log.info(f"Cluster Labels are the following {clusters}")
    industries = sorted(chars["ff12"].dropna().unique())
    icode = pd.Categorical(chars["ff12"], categories=industries).codes.astype(np.int64)
    D = np.zeros((len(chars), len(industries)))
    hasi = icode >= 0
    D[np.nonzero(hasi)[0], icode[hasi]] = 1.0                          # one-hot, NaN row: 0
    mcode = np.searchsorted(np.unique(mi_m), mi_m)
    Z = _seg_zscore(torch.as_tensor(R, **f64), torch.as_tensor(mcode, device=dev),
                    int(mcode.max()) + 1 if len(mcode) else 0)
    Fexp = torch.cat([torch.as_tensor(D, **f64), Z], dim=1)          # [rows, K] exposures
    factor_cols = [str(i) for i in industries] + clusters
    sg = chars["size_grp"]
    row_ok = torch.isfinite(Fexp).all(1) & torch.as_tensor(
        (sg.notna().to_numpy() & hasi), device=dev)
    log.info("Cluster Ranks Completed.")
    th("s3.cluster_ranks+zscore")

    # ---- daily <- exposures of the PREVIOUS month (eom_ret = eom + 1M), inner + dropna ------
    # The daily panel (~9.4M rows at S&P 500 scale) is handled on the device: integer
    # (id, month) keys, one sorted search into the monthly rows, compaction, and the (date, id)
    # order as ONE sort of a dense int64 key; only per-day / per-month results come back.
    i64 = dict(dtype=torch.int64, device=dev)
    t_dn = torch.as_tensor(daily["date"].to_numpy().astype("datetime64[D]").astype(np.int64),
                           **i64)
    t_id = torch.as_tensor(daily["id"].to_numpy(np.int64), **i64)
    t_ret = torch.as_tensor(daily["ret_exc"].to_numpy(np.float64), **f64)
    keep = t_dn >= int(np.datetime64(chars["eom"].min().date(), "D").astype(np.int64))
    ud, uinv = torch.unique(t_dn, return_inverse=True)
    ud_mi = torch.as_tensor(month_index(ud.cpu().numpy().astype("datetime64[D]")), **i64)
    SH = np.int64(1 << 20)
    mkey = ids_m * SH + (mi_m + 1)                                   # key of (id, eom_ret)
    mo = np.argsort(mkey, kind="stable")
    mkey_s = torch.as_tensor(mkey[mo], **i64)
    dkey = t_id * int(SH) + ud_mi[uinv]
    pos = torch.searchsorted(mkey_s, dkey).clamp_(max=max(len(mkey) - 1, 0))
    hit = (mkey_s[pos] == dkey) if len(mkey) else torch.zeros_like(keep)
    mrow = torch.as_tensor(mo, **i64)[pos]
    sel = keep & hit & row_ok[mrow] & torch.isfinite(t_ret)
    idx = torch.nonzero(sel).squeeze(1)
    t_id, t_dn, t_ret, mrow = t_id[idx], t_dn[idx], t_ret[idx], mrow[idx]
    ids_u = torch.unique(t_id)
    code = torch.searchsorted(ids_u, t_id)
    dmin = int(t_dn.min()) if len(t_dn) else 0
    span = (int(t_dn.max()) - dmin + 1) if len(t_dn) else 1
    order = torch.sort((t_dn - dmin) * len(ids_u) + code, stable=True).indices   # (date, id)
    t_id, t_dn, t_ret, mrow, code = t_id[order], t_dn[order], t_ret[order], mrow[order], code[order]
    udays, dcnt = torch.unique_consecutive(t_dn, return_counts=True)
    gs_day = torch.cat([torch.zeros(1, **i64), torch.cumsum(dcnt, 0)])
    th("s3.daily_merge")
    Xd = Fexp[mrow].contiguous()
    coef, resid_t, nbad = _ols(Xd, t_ret, gs_day)
    days = udays.cpu().numpy()
    log.info(f"Factor Returns Completed ({len(days)} days, {nbad} pinv fallbacks).")
    th("s3.daily_ols")

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
    eoms = chars["eom"].to_numpy().astype("datetime64[D]")
    calc = np.unique(eoms[eoms >= np.datetime64(min_date.date())])
    calc_mi = month_index(calc)
    end_idx = np.searchsorted(day_dt, calc, side="right")
    Fm = ewma_factor_cov(coef, end_idx, obs, w_cor, w_var, scale=21.0,
                         nan_cor=nan_cor).cpu().numpy()
    if nan_cor:
        _zero_exposureless(Fm, coef, end_idx, obs)
    th("s3.ewma_factor_cov")

    # ---- idiosyncratic EWMA vol (:345-442), on the device ---------------------------------
    o2 = torch.sort(code * span + (t_dn - dmin), stable=True).indices   # (id, date)
    s_id, s_dn = t_id[o2], t_dn[o2]
    resid_s = resid_t[o2]
    _, icnt = torch.unique_consecutive(s_id, return_counts=True)
    gs_id = torch.cat([torch.zeros(1, **i64), torch.cumsum(icnt, 0)])
    lam = 0.5 ** (1.0 / cs["hl_stock_var"])
    res_vol = _ewma_vol(resid_s, gs_id, lam, int(cs["initial_var_obs"]))
    days_t = torch.as_tensor(days, **i64)
    dpos = torch.searchsorted(days_t, s_dn)
    nanv = torch.full(s_dn.shape, float("nan"), **f64)
    td_252 = torch.where(dpos >= 252, days_t[(dpos - 252).clamp(min=0)].to(torch.float64), nanv)
    row = torch.arange(len(s_dn), **i64)
    src = row - 200                                                    # group_shift(., 200)
    gstart = torch.repeat_interleave(gs_id[:-1], icnt)
    d200 = torch.where(src >= gstart, s_dn[src.clamp(min=0)].to(torch.float64), nanv)
    ok = (d200 >= td_252) & ~torch.isnan(res_vol)
    day_mi = torch.as_tensor(month_index(days.astype("datetime64[D]")), **i64)
    s_mi = day_mi[dpos]
    # the last observation per (id, month) among the rows that pass the filter
    kidx = torch.nonzero(ok).squeeze(1)
    f_id, f_mi, f_vol = s_id[kidx], s_mi[kidx], res_vol[kidx]
    if len(f_id):
        flast = torch.cat([(f_id[1:] != f_id[:-1]) | (f_mi[1:] != f_mi[:-1]),
                           torch.ones(1, dtype=torch.bool, device=dev)])
    else:
        flast = torch.zeros(0, dtype=torch.bool, device=dev)
    vkey = (f_id[flast] * int(SH) + f_mi[flast]).cpu().numpy()
    vval = f_vol[flast].cpu().numpy()
    th("s3.idio_vol")

    # ---- Barra assembly (:453-494), every calc month at once -----------------------------
    in_calc = np.isin(mi_m, calc_mi)
    rows = np.nonzero(in_calc)[0]                                     # (eom, id) order
    rkey = ids_m[rows] * SH + mi_m[rows]
    vo = np.argsort(vkey, kind="stable")
    vp = np.clip(np.searchsorted(vkey[vo], rkey), 0, max(len(vkey) - 1, 0))
    vhit = (vkey[vo][vp] == rkey) if len(vkey) else np.zeros(len(rkey), bool)
    rv = np.where(vhit, vval[vo][vp], np.nan)
    rv_t = torch.as_tensor(rv, **f64)
    # (month, size group) groups as integer codes: month position x (size-group code + 1),
    # a NaN size group gets its own slot and is masked below
    mcode2 = np.searchsorted(calc_mi, mi_m[rows])
    sgc = pd.Categorical(sg.to_numpy(object)[rows]).codes.astype(np.int64)
    nsg = int(sgc.max()) + 2 if len(sgc) else 1
    gcode = mcode2 * nsg + (sgc + 1)
    sg_nan = sgc < 0
    G1 = len(calc_mi) * nsg
    gct = torch.as_tensor(gcode, device=dev)
    med_g = _seg_median(rv_t, gct, G1)[gct]
    med_g = torch.where(torch.as_tensor(sg_nan, device=dev), torch.full_like(med_g, float("nan")),
                        med_g)                                        # NaN size_grp: no group
    med_m = _seg_median(rv_t, torch.as_tensor(mcode2, device=dev), len(calc_mi))[
        torch.as_tensor(mcode2, device=dev)]
    med = torch.where(torch.isnan(med_g), med_m, med_g)
    rv_f = torch.where(torch.isnan(rv_t), med, rv_t)
    ivol = (rv_f * rv_f * 21.0).cpu().numpy()
    off = np.concatenate([[0], np.cumsum(np.bincount(np.searchsorted(calc_mi, mi_m[rows]),
                                                     minlength=len(calc_mi)))])
    th("s3.barra_assembly")
    return BarraCov(months=calc_mi.astype(np.int64), offsets=off.astype(np.int64),
                    ids=ids_m[rows], X=Fexp[torch.as_tensor(rows, device=dev)].cpu().numpy(),
                    ivol=ivol, F=Fm, factors=factor_cols)


def estimate_cov_frames_pandas(chars: pd.DataFrame, daily: pd.DataFrame, labels: pd.DataFrame,
                               cs: dict, device: str = "cpu", nan_cor: bool = True) -> BarraCov:
    """The round-1 pandas-bound form of ``estimate_cov_frames`` (groupby-lambda z-score,
    frame merges over the daily panel, one loop iteration per calc month): the test oracle
    and the host baseline of tools/bench_s3.py."""
    features = get_features()
    chars = chars.sort_values(["eom", "id"], kind="stable").reset_index(drop=True)
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
    daily = daily.assign(eom_ret=daily["date"] + pd.offsets.MonthEnd(0))
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
    Fm = ewma_factor_cov(fr, end_idx, obs, w_cor, w_var, scale=21.0,
                         nan_cor=nan_cor).cpu().numpy()
    if nan_cor:
        _zero_exposureless(Fm, fr, end_idx, obs)

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
        # (an all-NaN size group has no median: NaN, filled by the overall median below -
        # groupby's own median gives it without numpy's empty-slice warning)
        med = cd.groupby("size_grp")["res_vol"].transform("median")
        if med.isna().any() and cd["res_vol"].notna().any():
            med = med.fillna(cd["res_vol"].median(skipna=True))
        cd["res_vol"] = cd["res_vol"].fillna(med)
        cd = cd.sort_values("id", kind="stable")
        ids_l.append(cd["id"].to_numpy(np.int64))
        X_l.append(cd[factor_cols].to_numpy(np.float64))
        iv_l.append(cd["res_vol"].to_numpy(np.float64) ** 2 * 21.0)
        off.append(off[-1] + len(cd))
    return BarraCov(months=calc_mi.astype(np.int64), offsets=np.asarray(off, np.int64),
                    ids=np.concatenate(ids_l), X=np.concatenate(X_l), ivol=np.concatenate(iv_l),
                    F=Fm, factors=factor_cols)
