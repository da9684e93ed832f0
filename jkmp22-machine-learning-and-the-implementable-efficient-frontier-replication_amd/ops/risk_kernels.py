"""Device ops of the Barra risk model (csrc/risk.hip).

* ``daily_ols``       - per-day OLS without intercept on CSR day segments; exactly singular
                        days take pinv(X'X) X'y (Estimate Covariance Matrix.py:214-233) inside
                        the same kernel (cyclic Jacobi, numpy's rcond = 1e-15);
* ``ewma_factor_cov`` - monthly factor covariance F = sd cor sd * 21 from EWMA-weighted
                        cov.wt / cor.wt over the trailing ``obs`` days (:297-335,
                        General_functions.py:745-835);
* ``ewma_vol``        - per-stock zero-mean EWMA volatility (numba ``ewma_vol``, :345-386).

Every op takes device tensors and runs the gfx950 kernel on the caller's current stream; CPU
tensors take the fp64 torch/numpy oracle path (no silent fallback on a GPU box: the native
library is mandatory there).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as nat
from ..utils.log import COUNTERS

_P, _I, _L, _D = C.c_void_p, C.c_int, C.c_int64, C.c_double
nat.register_hip("pfml_daily_ols", [_P, _P, _P, _I, _I, _P, _P, _P, _P])
nat.register_hip("pfml_ewma_factor_cov", [_P, _I, _P, _I, _I, _P, _P, _D, _P, _P, _P, _I, _P])
nat.register_hip("pfml_ewma_vol", [_P, _P, _L, _D, _I, _P, _P])
nat.register_hip("pfml_risk_max_factors", [])


def daily_ols(X: torch.Tensor, y: torch.Tensor, offsets: torch.Tensor):
    """OLS per segment [offsets[d], offsets[d+1]) of the rows of X [R, K], y [R].

    Returns (coef [D, K], resid [R], n_pinv)."""
    D = offsets.numel() - 1
    R, K = X.shape
    if not nat.is_device(X) or K > int(nat.hip_lib().pfml_risk_max_factors()):
        return _daily_ols_torch(X, y, offsets)
    X = X.to(torch.float64).contiguous()
    y = y.to(torch.float64).contiguous()
    off = offsets.to(device=X.device, dtype=torch.int64).contiguous()
    coef = torch.empty((D, K), dtype=torch.float64, device=X.device)
    resid = torch.empty(R, dtype=torch.float64, device=X.device)
    status = torch.zeros(D, dtype=torch.int32, device=X.device)
    nat.check(nat.hip_lib().pfml_daily_ols(X.data_ptr(), y.data_ptr(), off.data_ptr(), D, K,
                                           coef.data_ptr(), resid.data_ptr(), status.data_ptr(),
                                           nat.stream_of(X)), "pfml_daily_ols")
    # status 2: the day met an exact zero pivot (LinAlgError) and the kernel applied
    # pinv(X'X) X'y itself (reference :228-229); one count read, no host recompute
    nbad = int((status == 2).sum().item())
    if nbad:
        COUNTERS.add("risk.ols_pinv_fallback", nbad)
    return coef, resid, nbad


def _daily_ols_torch(X, y, offsets):
    off = [int(v) for v in offsets.tolist()]
    D = len(off) - 1
    K = X.shape[1]
    coef = torch.empty((D, K), dtype=torch.float64, device=X.device)
    resid = torch.empty_like(y, dtype=torch.float64)
    nbad = 0
    for d in range(D):
        Xd, yd = X[off[d]:off[d + 1]].double(), y[off[d]:off[d + 1]].double()
        XtX, Xty = Xd.T @ Xd, Xd.T @ yd
        c, info = torch.linalg.solve_ex(XtX, Xty)
        if int(info) != 0:
            nbad += 1
            c = torch.linalg.pinv(XtX, rtol=1e-15) @ Xty      # numpy's default rcond
        coef[d] = c
        resid[off[d]:off[d + 1]] = yd - Xd @ c
    if nbad:
        COUNTERS.add("risk.ols_pinv_fallback", nbad)
    return coef, resid, nbad


def ewma_factor_cov(fr: torch.Tensor, ends, obs: int, w_cor, w_var, scale: float = 21.0,
                    return_parts: bool = False, nan_cor: bool = True):
    """F[b] = sd_b cor_b sd_b * scale for the window fr[ends[b]-t_b : ends[b]], t_b = min(obs,
    ends[b]), with weights w_*[obs - t_b:] (cor: hl_cor, sd: hl_var).  fr: [days, K].
    ``nan_cor`` (compat mode): a zero-variance factor's correlations are 0 / 0 = NaN, as the
    reference's weighted_cor_wt gives them (General_functions.py:827); else 0."""
    dev = fr.device
    ends_np = np.asarray(ends, dtype=np.int64)
    B, K = len(ends_np), fr.shape[1]
    wc = torch.as_tensor(np.asarray(w_cor, np.float64), device=dev)
    wv = torch.as_tensor(np.asarray(w_var, np.float64), device=dev)
    if nat.is_device(fr):
        frc = fr.to(torch.float64).contiguous()
        e = torch.as_tensor(ends_np, device=dev)
        F = torch.empty((B, K, K), dtype=torch.float64, device=dev)
        cor = torch.empty_like(F) if return_parts else None
        var = torch.empty_like(F) if return_parts else None
        nat.check(nat.hip_lib().pfml_ewma_factor_cov(
            frc.data_ptr(), K, e.data_ptr(), B, int(obs), wc.data_ptr(), wv.data_ptr(),
            float(scale), F.data_ptr(), nat.ptr(cor), nat.ptr(var), int(bool(nan_cor)),
            nat.stream_of(frc)),
            "pfml_ewma_factor_cov")
        return (F, cor, var) if return_parts else F
    Fs, cs, vs = [], [], []
    for b in range(B):
        t = min(int(obs), int(ends_np[b]))
        Xw = fr[ends_np[b] - t: ends_np[b]].double()
        c = weighted_cov_torch(Xw, wc[obs - t:], cor=True, nan_cor=nan_cor)
        v = weighted_cov_torch(Xw, wv[obs - t:], cor=False)
        sd = torch.sqrt(torch.diagonal(v))
        Fs.append(sd.unsqueeze(-1) * c * sd.unsqueeze(0) * scale)
        cs.append(c)
        vs.append(v)
    F = torch.stack(Fs) if Fs else torch.zeros((0, K, K), dtype=torch.float64)
    if return_parts:
        return F, torch.stack(cs), torch.stack(vs)
    return F


def weighted_cov_torch(X: torch.Tensor, w: torch.Tensor, cor: bool,
                       nan_cor: bool = True) -> torch.Tensor:
    """R cov.wt(center=TRUE, method='unbiased'[, cor=TRUE]) of X [T, K] (oracle).  cor with a
    zero-variance column: NaN off the diagonal (``nan_cor``, the reference's division) or 0."""
    wn = w / w.sum()
    mu = (wn.unsqueeze(-1) * X).sum(0, keepdim=True)
    Xw = (X - mu) * wn.sqrt().unsqueeze(-1)
    cov = Xw.T @ Xw / (1.0 - (wn * wn).sum())
    if not cor:
        return cov
    sd = torch.sqrt(torch.diagonal(cov))
    den = sd.unsqueeze(-1) * sd.unsqueeze(0)
    if nan_cor:
        c = cov / den
    else:
        c = torch.where(den > 0, cov / torch.where(den > 0, den, 1.0), torch.zeros_like(cov))
    c.fill_diagonal_(1.0)
    return c


def ewma_vol(x: torch.Tensor, groups, lam: float, start: int) -> torch.Tensor:
    """EWMA vol per group of rows (sorted by (group, time)); groups = CSR starts."""
    if not nat.is_device(x):
        from .. import runtime as rt
        g = groups.cpu().numpy() if isinstance(groups, torch.Tensor) else np.asarray(groups)
        return torch.as_tensor(rt.ewma_vol(x.numpy(), g, lam, start))
    xc = x.to(torch.float64).contiguous()
    gs = (groups.to(device=x.device, dtype=torch.int64) if isinstance(groups, torch.Tensor)
          else torch.as_tensor(np.asarray(groups, np.int64), device=x.device))
    out = torch.empty_like(xc)
    nat.check(nat.hip_lib().pfml_ewma_vol(xc.data_ptr(), gs.data_ptr(), gs.numel() - 1,
                                          float(lam), int(start), out.data_ptr(),
                                          nat.stream_of(xc)), "pfml_ewma_vol")
    return out
