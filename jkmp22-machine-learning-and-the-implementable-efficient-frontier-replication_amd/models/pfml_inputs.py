"""L4 PFML inputs (PFML_Input_Data.py): r_tilde_t, risk_t, tc_t, denom_t of (25) per month.

The reference's hot loop (:318-491, 1.6-2.6 s per month on 8 CPU cores, pandas-bound) becomes
a batched device pipeline over MONTHS (dates are independent given m_t, Sigma_t and the
13-month signal window) and over g (the g-dependent part is only the signal block):

1. RFF features for the whole panel: one fp64 MFMA GEMM X W + cos/sin (K13, once per g),
   stored in the interleaved order [constant, cos1, sin1, ...];
2. vol scales sqrt(diag(Sigma_t)) = sqrt(rowsum((X F) o X) + ivol) without forming Sigma
   (K1 diag epilogue, :274-307), cross-sectional median fill;
3. per batch of months (ragged universes padded block-diagonally):
   * signals: gather the 13 x N x P window, demean RFF columns, unit-norm every column, scale
     rows by 1/vol (K11/K12, :357-391);
   * Sigma_t = X F X' + diag(ivol) (K1) and m_t = m_func(...) (K2/K3, Lemma 1);
   * the aggregation (24) in Horner form over the augmented [S_{t-theta} | I] (K5/K6):
       T_11 = [S_11 | I],  T_theta = [S_theta | I] + (m D_theta) T_{theta+1}
     gives both sum_theta agg_theta S_{t-theta} and sum_theta agg_theta in 11 GEMMs per chain
     (the reference forms 22 N x N products plus 24 N x P products), with both g stacked in
     the column dimension so m and the agg products are shared;
   * omega = const^-1 Omega (pivoted LU solve, K7), omega_chg = omega - D_0 omega_l1;
   * r_tilde = omega' r, risk = gamma omega' Sigma omega (Sigma applied in low-rank form),
     tc = w omega_chg' Lambda omega_chg, denom = risk + tc (K8-K10).

Output: ``PfmlReals`` (search.py) + per-month signals signal_t (all in internal feature
order; ``config.interleaved_order`` maps to the reference's feat_all).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import pandas as pd
import torch

from ..config import Config, get_features, interleaved_order
from ..data import io
from ..ops import linalg as la
from ..ops.gemm import gemm, gemm_prec
from ..ops.panel import rff_features, standardize_signals
from ..utils.dates import month_index, pfml_date_grids
from ..utils.log import get_logger
from ..utils.trace import range_pop, range_push
from .risk import BarraCov
from .search import PfmlReals

log = get_logger("pfml_inputs")


@dataclass
class Panel:
    """Monthly characteristics panel sorted by (month, id)."""
    mi: np.ndarray
    ids: np.ndarray
    key: np.ndarray           # mi * 10^7 + id, sorted
    valid: np.ndarray
    cols: dict                # name -> float64 array [R]
    feats: np.ndarray         # [R, k] ranked characteristics

    @classmethod
    def from_chars(cls, chars: pd.DataFrame, features: list[str]) -> "Panel":
        mi = month_index(chars["eom"])
        ids = chars["id"].to_numpy(np.int64)
        order = np.lexsort((ids, mi))
        mi, ids = mi[order], ids[order]
        cols = {}
        for c in ("ret_ld1", "tr_ld0", "mu_ld0", "tr_ld1", "lambda", "me"):
            if c in chars:
                cols[c] = chars[c].to_numpy(np.float64)[order]
        feats = np.ascontiguousarray(chars[features].to_numpy(np.float64)[order])
        return cls(mi=mi, ids=ids, key=mi * 10_000_000 + ids,
                   valid=chars["valid"].to_numpy(bool)[order], cols=cols, feats=feats)

    def rows(self, mi: int, ids: np.ndarray) -> np.ndarray:
        k = mi * 10_000_000 + np.asarray(ids, np.int64)
        p = np.searchsorted(self.key, k)
        p = np.clip(p, 0, len(self.key) - 1)
        ok = self.key[p] == k
        return np.where(ok, p, -1)

    def valid_rows(self, mi: int) -> np.ndarray:
        a = np.searchsorted(self.mi, mi, side="left")
        b = np.searchsorted(self.mi, mi, side="right")
        r = np.arange(a, b)
        return r[self.valid[a:b]]


@dataclass
class PfmlInputs:
    reals: PfmlReals
    months: np.ndarray                   # [T] month indices (dates_m2 handled here)
    signal_rows: list                    # per month: panel rows (valid ids at d, id order)
    signal_t: list                       # per g: per month [n_d, P] tensors (device)
    rff_w: np.ndarray                    # [G, k, P/2]
    ids: list                            # per month: ids


def _rff_weights(cfg: Config, k: int) -> np.ndarray:
    """W per g.  compat (quirk Q1): the supplied rff_w.csv for every g (g ignored);
    corrected: W_g ~ N(0, g I_k) drawn from seed_no."""
    G, half = len(cfg.g_vec), cfg.p_max // 2
    if cfg.run.compat_mode:
        W = io.read_rff_w(cfg.run.data_dir)
        if W.shape != (k, half):
            raise ValueError(f"rff_w.csv has shape {W.shape}, expected {(k, half)}")
        return np.stack([W] * G)
    rng = np.random.default_rng(cfg.settings["seed_no"])
    Z = rng.standard_normal((k, half))
    return np.stack([Z * np.sqrt(g) for g in cfg.g_vec])


def vol_scales(panel: Panel, barra: BarraCov, months: np.ndarray) -> np.ndarray:
    """sqrt(diag Sigma_t) merged on (id, month), NaN -> cross-sectional median (:274-307)."""
    vol = np.full(len(panel.mi), np.nan)
    for mi in months:
        ids, X, F, iv = barra.slice(mi)
        d = np.einsum("ik,kl,il->i", X, F, X) + iv
        r = panel.rows(mi, ids)
        ok = r >= 0
        vol[r[ok]] = np.sqrt(d[ok])
    # median fill per month over all panel rows of that month
    s = pd.Series(vol)
    med = s.groupby(panel.mi).transform("median")
    return s.fillna(med).to_numpy()


def auto_month_batch(n_stocks: int, gp: int, device, cap: int = 256) -> int:
    """Months per S4 batch from the memory one month's working set needs (fp64): the
    13-month signal window (13 N GP), the Horner chains and solves (~6 N (GP + N)) and ~14
    N x N matrices of m_func / Sigma.  A device batch takes up to 60 % of free HBM (288 GB on
    MI355X: ~256 months at N = 500, ~75 at N = 3000), a host batch 25 % of available RAM."""
    per = 8.0 * (13.0 * n_stocks * gp + 6.0 * n_stocks * (gp + n_stocks) + 14.0 * n_stocks ** 2)
    dev = torch.device(device)
    if dev.type == "cuda":
        free, _ = torch.cuda.mem_get_info(dev)
        budget = 0.6 * free
    else:
        try:
            import psutil
            budget = 0.25 * psutil.virtual_memory().available
        except Exception:                                   # pragma: no cover
            budget = 4e9
    return int(max(1, min(cap, budget // per)))


def build_inputs(cfg: Config, chars: pd.DataFrame, barra: BarraCov, wealth: pd.DataFrame,
                 risk_free: pd.DataFrame, device, months: np.ndarray | None = None,
                 keep_risk_tc: bool = False, batch: int | None = None) -> PfmlInputs:
    features = get_features()
    pf = cfg.pf_set
    gamma, mu = float(pf["gamma_rel"]), float(pf["mu"])
    lb = int(pf["lb_hor"])
    G, Pm = len(cfg.g_vec), cfg.p_max
    P = Pm + 1
    dev = torch.device(device)
    prec = cfg.run.precision         # fp64 | fp32 | bf16 | fp8: covariance / RFF / risk GEMMs
    panel = Panel.from_chars(chars, features)
    grids = pfml_date_grids(int(barra.months.min()), lb, cfg.settings["split"]["test_end"],
                            cfg.settings["pf"]["dates"]["start_year"],
                            cfg.settings["pf"]["dates"]["split_years"])
    if months is None:
        months = grids["m2"]
    months = np.asarray(months, np.int64)

    # ---- 1. RFF features (K13) and 2. vol scales ------------------------------------
    range_push("pfml_inputs.rff")
    W = _rff_weights(cfg, len(features))
    same_w = all(np.array_equal(W[0], W[g]) for g in range(G))
    Xf = torch.as_tensor(panel.feats, dtype=torch.float64, device=dev)
    rffs = []
    for g in range(G):
        if g > 0 and same_w:
            rffs.append(rffs[0])          # quirk Q1: identical inputs for every g
            continue
        R = rff_features(Xf, torch.as_tensor(W[g], dtype=torch.float64, device=dev), prec)
        rffs.append(torch.cat([R, torch.zeros((1, P), dtype=R.dtype, device=dev)]))  # pad row
    del Xf
    range_pop()
    lbm = grids["lb"]
    lbm = lbm[(lbm >= months.min() - (lb + 1)) & (lbm <= months.max())]
    vol = vol_scales(panel, barra, lbm)
    vol_t = torch.as_tensor(np.r_[vol, 1.0], dtype=torch.float64, device=dev)
    gt_all = (1.0 + panel.cols["tr_ld0"]) / (1.0 + panel.cols["mu_ld0"])
    gt_all = np.nan_to_num(gt_all, nan=1.0)
    gt_t = torch.as_tensor(np.r_[gt_all, 1.0], dtype=torch.float64, device=dev)
    wmap = dict(zip(month_index(wealth["eom"]), wealth["wealth"].to_numpy(np.float64)))
    rfmap = dict(zip(month_index(risk_free["eom"]), risk_free["rf"].to_numpy(np.float64)))
    tc_on = bool(cfg.settings["Transaction_Costs"])

    T = len(months)
    r_out = torch.zeros((G, T, P), dtype=torch.float64, device=dev)
    d_out = torch.zeros((G, T, P, P), dtype=torch.float64, device=dev)
    risk_out = torch.zeros_like(d_out) if keep_risk_tc else None
    tc_out = torch.zeros_like(d_out) if keep_risk_tc else None
    sig_rows, sig_ids = [], []
    signal_t = [[None] * T for _ in range(G)]
    Rpad = len(panel.mi)
    bsz = batch or cfg.run.month_batch
    if not bsz or bsz <= 0:
        nmax = max(len(panel.valid_rows(int(d))) for d in months) if T else 1
        bsz = auto_month_batch(nmax, G * P, dev)
        log.info(f"PFML inputs: {bsz} months per batch (N <= {nmax})")

    for b0 in range(0, T, bsz):
        bm = months[b0: b0 + bsz]
        B = len(bm)
        range_push("pfml_inputs.batch")
        rows_d = [panel.valid_rows(int(d)) for d in bm]
        ns = np.array([len(r) for r in rows_d])
        N = int(ns.max())
        idx = np.full((B, lb + 2, N), Rpad, dtype=np.int64)
        for bi, d in enumerate(bm):
            ids = panel.ids[rows_d[bi]]
            for th in range(lb + 2):
                r = panel.rows(int(d) - th, ids)
                if np.any(r < 0):
                    raise ValueError(f"month {d}: universe lacks the {th}-month lookback rows")
                idx[bi, th, : len(r)] = r
            sig_rows.append(rows_d[bi])
            sig_ids.append(ids)
        idx_t = torch.as_tensor(idx, device=dev)
        mask = torch.as_tensor((np.arange(N)[None, :] < ns[:, None]).astype(np.float64), device=dev)
        wv = torch.as_tensor([wmap[int(d)] for d in bm], dtype=torch.float64, device=dev)
        rfv = torch.as_tensor([rfmap[int(d)] for d in bm], dtype=torch.float64, device=dev)

        # signals for every g: [G, B, 13, N, P]
        S_all = []
        for g in range(G):
            if g > 0 and rffs[g] is rffs[0]:
                S_all.append(S_all[0])
                continue
            S_all.append(standardize_signals(rffs[g], idx_t, mask, vol_t))
        # Barra Sigma (padded: identity block), Lambda, returns
        K = barra.X.shape[1]
        Xl_h = np.zeros((B, N, K))
        Fb_h = np.zeros((B, K, K))
        iv_h = np.ones((B, N))
        lam_h = np.empty((B, N))
        r_h = np.zeros((B, N))
        for bi, d in enumerate(bm):
            ids = sig_ids[b0 + bi]
            bids, X, F, ivol = barra.slice(int(d))
            pos = np.searchsorted(bids, ids)
            if np.any(pos >= len(bids)) or np.any(bids[np.minimum(pos, len(bids) - 1)] != ids):
                raise KeyError(f"month {d}: valid ids missing from the Barra universe")
            n = len(ids)
            Xl_h[bi, :n] = X[pos]
            Fb_h[bi] = F
            iv_h[bi, :n] = ivol[pos]
            lam_h[bi] = gamma / float(wmap[int(d)])
            lam_h[bi, :n] = panel.cols["lambda"][rows_d[bi]] if tc_on else 1e-16
            r_h[bi, :n] = panel.cols["ret_ld1"][rows_d[bi]]
        Xl = torch.as_tensor(Xl_h, device=dev)
        Fb = torch.as_tensor(Fb_h, device=dev)
        iv = torch.as_tensor(iv_h, device=dev)
        lam = torch.as_tensor(lam_h, device=dev)
        r = torch.as_tensor(r_h, device=dev)
        XF = gemm(Xl, Fb)
        Sigma = gemm_prec(XF, Xl, prec, trans_b=True)            # K1: Barra covariance
        Sigma.diagonal(dim1=1, dim2=2).add_(iv)
        m = la.m_func(Sigma, lam, wv, rfv, mu, gamma, cfg.run.iterations, mask=mask)

        # (24): Horner chains over [S^{g=0} | ... | S^{g=G-1} | I]; with identical signals for
        # every g (quirk Q1, compat mode) one block is carried and shared
        Dg = gt_t[idx_t]                                           # [B, 13, N]
        Gc = 1 if same_w else G
        GP = Gc * P
        Wd = GP + N
        eye = torch.eye(N, dtype=torch.float64, device=dev).expand(B, N, N)

        def aug(th):
            Tm = torch.empty((B, N, Wd), dtype=torch.float64, device=dev)
            for g in range(Gc):
                Tm[:, :, g * P:(g + 1) * P] = S_all[g][:, th]
            Tm[:, :, GP:] = eye
            return Tm

        Tc = aug(lb)
        Ul = aug(lb + 1)
        for th in range(lb - 1, -1, -1):
            Mg = m * Dg[:, th].unsqueeze(1)                         # m diag(g_theta)
            Tn = aug(th)
            gemm(Mg, Tc, beta=1.0, out=Tn)
            Tc = Tn
            Mg1 = m * Dg[:, th + 1].unsqueeze(1)
            Un = aug(th + 1)
            gemm(Mg1, Ul, beta=1.0, out=Un)
            Ul = Un
        # omega = const^-1 Omega, solved in place on the augmented [Omega | const] rows
        omega = la.solve_augmented(Tc, N, GP, a0=GP, b0=0)          # [B, N, GP]
        omega_l1 = la.solve_augmented(Ul, N, GP, a0=GP, b0=0)
        omega_chg = omega - Dg[:, 0].unsqueeze(-1) * omega_l1

        # (25): r_tilde, risk, tc
        rt_ = gemm(omega, r.unsqueeze(-1), trans_a=True).squeeze(-1)        # [B, GP]
        XtO = gemm(Xl, omega, trans_a=True)                                  # [B, K, GP]
        SO = gemm(Xl, gemm(Fb, XtO)) + iv.unsqueeze(-1) * omega               # Sigma omega
        lw = lam * wv.view(B, 1)
        for g in range(G):
            if g >= Gc:                                  # shared block (quirk Q1)
                d_out[g, b0:b0 + B] = d_out[0, b0:b0 + B]
                r_out[g, b0:b0 + B] = r_out[0, b0:b0 + B]
                if keep_risk_tc:
                    risk_out[g, b0:b0 + B] = risk_out[0, b0:b0 + B]
                    tc_out[g, b0:b0 + B] = tc_out[0, b0:b0 + B]
                for bi in range(B):
                    signal_t[g][b0 + bi] = signal_t[0][b0 + bi]
                continue
            sl = slice(g * P, (g + 1) * P)
            og, cg = omega[:, :, sl].contiguous(), omega_chg[:, :, sl].contiguous()
            risk = gemm_prec(og, SO[:, :, sl].contiguous(), prec, trans_a=True, alpha=gamma)
            tc = gemm(cg, lw.unsqueeze(-1) * cg, trans_a=True)
            d_out[g, b0:b0 + B] = risk + tc
            r_out[g, b0:b0 + B] = rt_[:, sl]
            if keep_risk_tc:
                risk_out[g, b0:b0 + B] = risk
                tc_out[g, b0:b0 + B] = tc
            for bi in range(B):
                signal_t[g][b0 + bi] = S_all[g][bi, 0, : ns[bi]].clone()
        range_pop()
        log.info(f"PFML inputs: months {b0 + B}/{T}")
    reals = PfmlReals(months=months, r_tilde=r_out, denom=d_out, risk=risk_out, tc=tc_out)
    return PfmlInputs(reals=reals, months=months, signal_rows=sig_rows, signal_t=signal_t,
                      rff_w=W, ids=sig_ids)


def to_reference_order(x: torch.Tensor, p_max: int, dims: tuple = (-1,)) -> torch.Tensor:
    """Permute internal [const, cos1, sin1, ...] axes to the reference feat_all order."""
    inv = np.argsort(interleaved_order(p_max))
    idx = torch.as_tensor(inv, device=x.device)
    for d in dims:
        x = x.index_select(d, idx)
    return x
