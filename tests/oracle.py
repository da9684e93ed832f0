"""Straight-line fp64 NumPy oracle of one PFML month, in the reference's own operation order
(PFML_Input_Data.py:318-491; General_functions.py:919-963): explicit cumulative products,
np.linalg.solve, scipy.linalg.sqrtm.  Independent of the batched engine."""
import numpy as np
import scipy.linalg as sla


def m_func_ref(w, mu, rf, sigma_gam, gam, lam, iterations):
    n = len(lam)
    c = 1 + rf + mu
    mbar = np.full(n, c)
    sgr = (np.outer(mbar, mbar) + sigma_gam / gam) / c ** 2
    a = np.diag(lam ** -0.5)
    x = (1.0 / w) * a @ sigma_gam @ a
    y = np.diag(1 + np.diag(sgr))
    sh = x + 2 * np.eye(n)
    mt = 0.5 * (sh - np.real(sla.sqrtm(sh @ sh - 4 * np.eye(n))))
    for _ in range(iterations):
        mt = np.linalg.inv(x + y - mt * sgr)
    return a @ mt @ np.diag(lam ** 0.5)


def month_ref(S_win, gt_win, r, Sigma, lam, w, rf, mu, gamma, iterations=10):
    """S_win: [13, n, P] standardised signals for lags 0..12; gt_win: [13, n]."""
    n = Sigma.shape[0]
    m = m_func_ref(w, mu, rf, Sigma * gamma, gamma, lam, iterations)
    gtm = [m @ np.diag(gt_win[t]) for t in range(13)]
    agg = [np.eye(n)]
    agg_l1 = [np.eye(n)]
    for t in range(11):
        agg.append(agg[t] @ gtm[t])
        agg_l1.append(agg_l1[t] @ gtm[t + 1])
    om = sum(agg[t] @ S_win[t] for t in range(12))
    const = sum(agg[t] for t in range(12))
    om1 = sum(agg_l1[t] @ S_win[t + 1] for t in range(12))
    const1 = sum(agg_l1[t] for t in range(12))
    omega = np.linalg.solve(const, om)
    omega_l1 = np.linalg.solve(const1, om1)
    chg = omega - np.diag(gt_win[0]) @ omega_l1
    r_tilde = omega.T @ r
    risk = gamma * omega.T @ Sigma @ omega
    tc = w * chg.T @ np.diag(lam) @ chg
    return r_tilde, risk, tc, m
