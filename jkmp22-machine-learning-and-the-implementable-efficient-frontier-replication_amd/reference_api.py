"""Reference-compatible function surface.

A user of the Python replication calls its helpers by name (General_functions.py,
PFML_Input_Data.py, PFML_Search_Coef.py, Estimate Covariance Matrix.py, PFML_best_hps.py).
Every function here keeps the reference's name, signature and pandas / numpy types and runs
the engine's implementation underneath (the vectorised host code, the native runtime, or -
with ``device="cuda"`` where offered - the gfx950 kernels), so scripts written against the
reference port by changing one import:

    from pfml.reference_api import *          # instead of: from General_functions import *

Citations are file:line in the reference.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import runtime as _rt
from .config import get_features, get_settings, pfml_feat_fun  # noqa: F401  (re-exported)
from .models import portfolio as _pf
from .models import prep as _prep
from .ops import linalg as _la
from .ops.risk_kernels import weighted_cov_torch as _wcov
from .utils.log import get_logger

log = get_logger("reference_api")

__all__ = ["get_settings", "get_features", "wealth_func", "long_horizon_ret", "categorize_sic",
           "size_screen_fun", "investment_universe", "addition_deletion_fun", "ecdf_transform",
           "build_cluster_ranks", "weighted_cov_wt", "weighted_cor_wt", "pfml_feat_fun",
           "create_cov", "create_lambda", "m_func", "rff", "denom_sum_fun", "ewma_vol",
           "initial_weights_new", "compute_stats", "pf_ts_fun"]


# ---- General_functions.py --------------------------------------------------------------
def wealth_func(wealth_end, end, market, risk_free) -> pd.DataFrame:
    """General_functions.py:175-220 (quirk Q4: cumprod(1 - tret))."""
    return _prep.wealth_func(wealth_end, pd.Timestamp(end), market, risk_free)


def long_horizon_ret(data, h, impute="zero") -> pd.DataFrame:
    """General_functions.py:222-288: leads ret_ld1..ret_ld{h}, zero / mean / median imputed."""
    d = data.copy()
    d["eom"] = pd.to_datetime(d["eom"])
    return _prep.long_horizon_ret(d, int(h), impute)


def categorize_sic(sic):
    """General_functions.py:293-402: FF12 industry of a SIC code (scalar or array)."""
    out = _prep.categorize_sic(np.atleast_1d(np.asarray(sic, dtype=np.float64)))
    return str(out[0]) if np.ndim(sic) == 0 else out


def size_screen_fun(chars, type_) -> None:
    """General_functions.py:404-504: sets ``chars['valid_size']`` in place; ValueError on an
    unknown screen type."""
    _prep.size_screen(chars, type_)


def investment_universe(add, delete) -> np.ndarray:
    """General_functions.py:507-548: universe state machine of ONE id's rows."""
    add = np.asarray(add, dtype=bool)
    return _rt.investment_universe(add, np.asarray(delete, dtype=bool),
                                   np.array([0, len(add)], dtype=np.int64))


def addition_deletion_fun(chars, addition_n, deletion_n) -> pd.DataFrame:
    """General_functions.py:550-699 (native rolling counts + state machine per id)."""
    return _prep.addition_deletion(chars, int(addition_n), int(deletion_n))


def ecdf_transform(group: pd.Series) -> pd.Series:
    """General_functions.py:702-711 (dead code in the reference): ECDF of the non-NaN values,
    evaluated at every element (NaN stays NaN)."""
    vals = group.dropna().to_numpy(np.float64)
    if vals.size == 0:
        return group
    srt = np.sort(vals)
    x = group.to_numpy(np.float64)
    out = np.searchsorted(srt, x, side="right") / srt.size
    return pd.Series(np.where(np.isnan(x), np.nan, out), index=group.index)


def build_cluster_ranks(cluster_data_m, cluster_labels, clusters, features) -> pd.DataFrame:
    """General_functions.py:715-740: per cluster, the row mean (NaN-skipping) of its members'
    ranks with direction -1 members flipped to 1 - x."""
    out = pd.DataFrame(index=cluster_data_m.index)
    for cl in clusters:
        sub = cluster_labels[(cluster_labels["cluster"] == cl)
                             & cluster_labels["characteristic"].isin(features)]
        X = cluster_data_m[sub["characteristic"].tolist()].to_numpy(np.float64, copy=True)
        flip = sub["direction"].to_numpy() == -1
        X[:, flip] = 1.0 - X[:, flip]
        out[cl] = pd.DataFrame(X, index=cluster_data_m.index).mean(axis=1)
    return out


def weighted_cov_wt(df, weights) -> pd.DataFrame:
    """General_functions.py:745-784: R cov.wt(center=TRUE, method='unbiased')."""
    X = torch.as_tensor(np.asarray(df, dtype=np.float64))
    c = _wcov(X, torch.as_tensor(np.asarray(weights, dtype=np.float64)), cor=False).numpy()
    cols = getattr(df, "columns", None)
    return pd.DataFrame(c, index=cols, columns=cols)


def weighted_cor_wt(df, weights) -> pd.DataFrame:
    """General_functions.py:786-835: the correlation form (unit diagonal)."""
    X = torch.as_tensor(np.asarray(df, dtype=np.float64))
    c = _wcov(X, torch.as_tensor(np.asarray(weights, dtype=np.float64)), cor=True).numpy()
    cols = getattr(df, "columns", None)
    return pd.DataFrame(c, index=cols, columns=cols)


def create_cov(x: dict, ids=None):
    """General_functions.py:847-897: Barra Sigma = X F X' + diag(ivol) from the month's
    {'fct_load', 'fct_cov', 'ivol_vec'}; warns on a negative variance (quirk Q7, no repair)."""
    load, ivol = x["fct_load"], x["ivol_vec"]
    if ids is not None:
        if isinstance(load, pd.DataFrame):
            load, ivol = load.loc[list(ids)], pd.Series(ivol).loc[list(ids)]
        else:
            sel = np.asarray(ids)
            load, ivol = np.asarray(load)[sel], np.asarray(ivol)[sel]
    L = np.asarray(load, dtype=np.float64)
    S = L @ np.asarray(x["fct_cov"], dtype=np.float64) @ L.T + np.diag(np.asarray(ivol, float))
    if np.min(np.diag(S)) < 0:
        log.warning("Warning: Negative Variances")
    if isinstance(load, pd.DataFrame):
        return pd.DataFrame(S, index=load.index, columns=load.index)
    return S


def create_lambda(x, ids) -> np.ndarray:
    """General_functions.py:900-916: diag(lambda_i for i in ids)."""
    if isinstance(x, dict):
        return np.diag([x[i] for i in ids])
    return np.diag(np.asarray(x)[np.asarray(ids)])


def m_func(w, mu, rf, sigma_gam, gam, K_Lambda, iterations, device: str = "cpu") -> np.ndarray:
    """General_functions.py:919-963: trading-speed matrix m of Lemma 1 (sigma_gam = gamma
    Sigma, K_Lambda = diag(lambda)).  The Schur sqrtm is replaced by the cancellation-free
    symmetric form, the inversions are the batched SPD inverse (a HIP kernel
    on ``device="cuda"``)."""
    sig = torch.as_tensor(np.asarray(sigma_gam, dtype=np.float64) / float(gam), device=device)
    lam = torch.as_tensor(np.diag(np.asarray(K_Lambda, dtype=np.float64)).copy(), device=device)
    one = lambda v: torch.tensor([float(v)], dtype=torch.float64, device=device)  # noqa: E731
    m = _la.m_func(sig[None], lam[None], one(w), one(rf), float(mu), float(gam), int(iterations))
    return m[0].cpu().numpy()


# ---- PFML_Search_Coef.py -------------------------------------------------------------------
def denom_sum_fun(train):
    """PFML_Search_Coef.py:37-46: element-wise sum of the 'denom' of every month of ``train``
    ({eom: {'denom': matrix, ...}}); a plain list of matrices is accepted too."""
    items = train.values() if isinstance(train, dict) else train
    mats = [e["denom"] if isinstance(e, dict) else e for e in items]
    total = mats[0].copy()
    for d in mats[1:]:
        total = total + d
    return total


# ---- PFML_Input_Data.py ------------------------------------------------------------------
def rff(X, p=None, g=None, W=None, seed=None) -> dict:
    """PFML_Input_Data.py:159-185: {'W', 'X_cos', 'X_sin'}; W ~ N(0, g I_k) of shape
    (k, p/2) when not given (quirk Q1: g is ignored when W is passed)."""
    X = np.asarray(X, dtype=np.float64)
    if W is None:
        rng = np.random.default_rng(seed)
        W = rng.standard_normal((X.shape[1], int(p) // 2)) * np.sqrt(float(g))
    Z = X @ np.asarray(W, dtype=np.float64)
    return {"W": W, "X_cos": np.cos(Z), "X_sin": np.sin(Z)}


# ---- Estimate Covariance Matrix.py ---------------------------------------------------------
def ewma_vol(x, lam, start) -> np.ndarray:
    """Estimate Covariance Matrix.py:345-386 (the numba kernel): zero-mean EWMA volatility."""
    x = np.asarray(x, dtype=np.float64)
    return _rt.ewma_vol(x, np.array([0, len(x)], dtype=np.int64), float(lam), int(start))


# ---- PFML_best_hps.py -------------------------------------------------------------------------
def initial_weights_new(data, w_type, udf_weights=None) -> pd.DataFrame:
    """PFML_best_hps.py:137-166: value- ("vw") or equal-weighted ("ew") starting weights at
    the first eom only (NaN elsewhere), plus an empty ``w`` column."""
    if w_type not in ("vw", "ew"):
        raise ValueError(f"Unknown w_type: {w_type}")
    d = data[["id", "eom"] + (["me"] if w_type == "vw" else [])].copy()
    if w_type == "vw":
        d["w_start"] = d["me"] / d.groupby("eom")["me"].transform("sum")
    else:
        d["w_start"] = 1.0 / d.groupby("eom")["id"].transform("size")
    d = d.sort_values("eom", kind="stable").reset_index(drop=True)[["id", "eom", "w_start"]]
    d.loc[d["eom"] != d["eom"].min(), "w_start"] = np.nan
    d["w"] = np.nan
    return d


def compute_stats(group: pd.DataFrame) -> pd.Series:
    """PFML_best_hps.py:220-239: inv, shorting, turnover, r, tc of one month's portfolio."""
    w, ws = group["w"].to_numpy(), group["w_start"].to_numpy()
    dw = w - ws
    lam = group["lambda"].to_numpy()
    return pd.Series({"inv": np.abs(w).sum(), "shorting": np.abs(w[w < 0]).sum(),
                      "turnover": np.abs(dw).sum(),
                      "r": (w * group["ret_ld1"].to_numpy()).sum(),
                      "tc": group["wealth"].iloc[0] / 2 * (lam * dw ** 2).sum()})


def pf_ts_fun(weights, data, wealth, gam=None, compat: bool = True) -> pd.DataFrame:
    """PFML_best_hps.py:241-259: per-month statistics (columns inv, shorting, turnover, r, tc,
    eom_ret; quirk Q3: eom_ret equals eom in compat mode)."""
    return _pf.pf_ts(weights, data, wealth, compat=compat)
