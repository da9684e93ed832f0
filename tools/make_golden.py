#!/usr/bin/env python3
"""Freeze golden fixtures from the REFERENCE's own functions on synthetic inputs.

Dev-time only (needs /root/reference): each function is extracted from the reference source
with ``ast`` and executed in an isolated namespace (numba's @njit decorator is stripped: the
kernel then runs as plain Python with identical semantics).  Inputs and outputs are written
to tests/golden/*.npz (numeric, allow_pickle=False) and tests/golden/*.csv, so the parity
tests run anywhere without the reference checkout.

    python tools/make_golden.py [/root/reference]
"""
import ast
import os
import sys

import numpy as np
import pandas as pd
from scipy.linalg import sqrtm

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def extract(path, names):
    src = open(path, encoding="utf-8").read()
    tree = ast.parse(src)
    ns = {"np": np, "pd": pd, "sqrtm": sqrtm, "re": __import__("re")}
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in names:
            node.decorator_list = []
            code = compile(ast.Module(body=[node], type_ignores=[]), path, "exec")
            exec(code, ns)
    missing = [n for n in names if n not in ns]
    if missing:
        raise KeyError(f"{missing} not found in {path}")
    return ns


def main():
    os.makedirs(OUT, exist_ok=True)
    gf = extract(os.path.join(REF, "General_functions.py"),
                 ["m_func", "create_cov", "weighted_cov_wt", "weighted_cor_wt",
                  "investment_universe", "wealth_func", "categorize_sic", "pfml_feat_fun",
                  "build_cluster_ranks", "long_horizon_ret"])
    ec = extract(os.path.join(REF, "Estimate Covariance Matrix.py"), ["ewma_vol"])
    rng = np.random.default_rng(2024)

    # m_func (General_functions.py:919-963) at two sizes, TC on / off
    for tag, N, lam_kind in [("n40", 40, "tc"), ("n25_notc", 25, "notc")]:
        K = 6
        X = rng.normal(size=(N, K))
        F = np.cov(rng.normal(size=(K, 300))) * 1e-4 * 21
        S = X @ F @ X.T + np.diag(rng.uniform(0.01, 0.03, N) ** 2 * 21)
        lam = 0.2 / rng.uniform(1e7, 1e9, N) if lam_kind == "tc" else np.full(N, 1e-16)
        w, mu, rf, g = 3e9, 0.007, 0.002, 10.0
        m = gf["m_func"](w=w, mu=mu, rf=rf, sigma_gam=S * g, gam=g, K_Lambda=np.diag(lam),
                         iterations=10)
        np.savez(os.path.join(OUT, f"m_func_{tag}.npz"), sigma=S, lam=lam,
                 scal=np.array([w, mu, rf, g]), m=np.asarray(m))

    # m_func on production-like spectra: a Barra Sigma of the engine's synthetic universe
    # (25 factors, F = sample cov * 21e-4, ivol = U(.01,.03)^2 * 21), N = 120, wealth 1e10,
    # TC on (lambda = 0.2 / U(1e7, 1e9): cond(x^2 + 4x) ~ 1e4) and off (lambda = 1e-16:
    # x ~ 1e4..1e7, where the scipy sqrtm form cancels)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pfml.data.synthetic import engine_inputs
    _, barra, _, _ = engine_inputs(n_stocks=120)
    ids, X, F, iv = barra.slice(int(barra.months[-3]))
    S = X @ F @ X.T + np.diag(iv)
    rng2 = np.random.default_rng(77)                  # own stream: other fixtures unchanged
    for tag, lam in [("prod_tc", 0.2 / rng2.uniform(1e7, 1e9, len(ids))),
                     ("prod_notc", np.full(len(ids), 1e-16))]:
        w, mu, rf, g = 1e10, 0.007, 0.003, 10.0
        m = gf["m_func"](w=w, mu=mu, rf=rf, sigma_gam=S * g, gam=g, K_Lambda=np.diag(lam),
                         iterations=10)
        np.savez_compressed(os.path.join(OUT, f"m_func_{tag}.npz"), sigma=S, lam=lam,
                            scal=np.array([w, mu, rf, g]), m=np.real(np.asarray(m)))

    # create_cov (Barra (37)) with an id subset
    N, K = 30, 5
    ids = np.arange(100, 100 + N)
    load = pd.DataFrame(rng.normal(size=(N, K)), index=ids)
    fcov = pd.DataFrame(np.cov(rng.normal(size=(K, 200))) * 1e-3)
    ivol = pd.Series(rng.uniform(0.01, 0.02, N), index=ids)
    sub = ids[::3]
    sig = gf["create_cov"]({"fct_load": load, "fct_cov": fcov, "ivol_vec": ivol}, ids=sub)
    np.savez(os.path.join(OUT, "create_cov.npz"), X=load.to_numpy(), F=fcov.to_numpy(),
             ivol=ivol.to_numpy(), ids=ids, sub=sub, sigma=np.asarray(sig))

    # weighted cov / cor (R cov.wt)
    Xw = rng.normal(size=(120, 7))
    ww = 0.5 ** (np.arange(120, 0, -1) / 40.0)
    cov = gf["weighted_cov_wt"](pd.DataFrame(Xw), ww).to_numpy()
    cor = gf["weighted_cor_wt"](pd.DataFrame(Xw), ww).to_numpy()
    np.savez(os.path.join(OUT, "weighted_cov.npz"), X=Xw, w=ww, cov=cov, cor=cor)

    # EWMA vol (numba kernel, run as Python) incl. NaNs and a short series
    x = rng.normal(scale=0.01, size=400)
    x[rng.random(400) < 0.05] = np.nan
    v1 = ec["ewma_vol"](x, 0.5 ** (1 / 126), 63)
    v2 = ec["ewma_vol"](x[:50], 0.5 ** (1 / 126), 63)
    np.savez(os.path.join(OUT, "ewma_vol.npz"), x=x, vol=v1, vol_short=v2)

    # investment universe state machine
    add = rng.random(200) < 0.3
    dele = rng.random(200) < 0.2
    inc = gf["investment_universe"](add, dele)
    np.savez(os.path.join(OUT, "universe.npz"), add=add, delete=dele, included=inc)

    # wealth path
    months = pd.date_range("1990-01-31", periods=60, freq="ME")
    rf = pd.DataFrame({"eom": months, "rf": rng.uniform(0, 0.004, 60)})
    mk = pd.DataFrame({"eom_ret": months, "mkt_vw_exc": rng.normal(0.006, 0.04, 60)})
    wl = gf["wealth_func"](1e10, pd.Timestamp("1994-12-31"), mk, rf)
    rf.to_csv(os.path.join(OUT, "wealth_rf.csv"), index=False)
    mk.to_csv(os.path.join(OUT, "wealth_market.csv"), index=False)
    wl.to_csv(os.path.join(OUT, "wealth_out.csv"), index=False)

    # FF12 mapping on every SIC 0..9999
    sic = np.arange(0, 10000)
    ff = np.array([gf["categorize_sic"](int(s)) for s in sic])
    pd.DataFrame({"sic": sic, "ff12": ff}).to_csv(os.path.join(OUT, "ff12.csv"), index=False)

    # lead returns (long_horizon_ret, h = 12) on a ragged panel with gaps
    rows = []
    for i in range(6):
        start = rng.integers(0, 10)
        for t in range(start, start + rng.integers(15, 40)):
            if rng.random() < 0.1:
                continue
            rows.append((1000 + i, pd.Timestamp("2000-01-31") + pd.offsets.MonthEnd(t),
                         rng.normal(0, 0.1)))
    panel = pd.DataFrame(rows, columns=["id", "eom", "ret_exc"])
    lh = gf["long_horizon_ret"](panel, h=12)[["id", "eom", "ret_ld1"]]
    panel.to_csv(os.path.join(OUT, "lead_in.csv"), index=False)
    lh.to_csv(os.path.join(OUT, "lead_out.csv"), index=False)

    # cluster ranks
    feats = [f"f{i}" for i in range(9)]
    cd = pd.DataFrame(rng.random((50, 9)), columns=feats)
    labels = pd.DataFrame({"characteristic": feats + ["zz"], "cluster": list("aabbbccdd") + ["a"],
                           "direction": [1, -1, 1, 1, -1, 1, -1, 1, 1, 1]})
    cr = gf["build_cluster_ranks"](cd, labels, ["a", "b", "c", "d"], feats)
    cd.to_csv(os.path.join(OUT, "cluster_in.csv"), index=False)
    labels.to_csv(os.path.join(OUT, "cluster_labels.csv"), index=False)
    cr.to_csv(os.path.join(OUT, "cluster_out.csv"), index=False)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
