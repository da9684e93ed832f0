#!/usr/bin/env python3
"""Daily-OLS diagnostics on the tests' small panel: the HIP kernel (pivoted LU + Jacobi pinv
fallback) vs the torch oracle (solve_ex + pinv), per day; prints NaN counts, the largest
coefficient difference and the rank structure of the singular days."""
import json
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pfml.config import Config
    from pfml.data import acquire, synthetic as syn
    from pfml.models import prep, risk
    d = tempfile.mkdtemp(prefix="pfml_diag_")
    spec = syn.small_spec()
    syn.write_raw(syn.generate(spec), d)
    cfg = syn.settings_for_small(Config.default().override([f"run.data_dir={d}"]), spec)
    acquire.get_additional_data(cfg)
    acquire.sp500_subset(cfg)
    prep.prepare_data(cfg)
    cap = {}
    orig = risk.daily_ols

    def spy(X, y, day, device):
        cap.update(X=X.copy(), y=y.copy(), day=day.copy())
        return orig(X, y, day, device)

    risk.daily_ols = spy
    chars, daily, labels = risk._load_risk_inputs(cfg)
    cs = cfg.settings["cov_set"]
    bg = risk.estimate_cov_frames_pandas(chars, daily, labels, cs, "cuda")
    bc = risk.estimate_cov_frames_pandas(chars, daily, labels, cs, "cpu")
    X, y, day = cap["X"], cap["y"], cap["day"]
    _, cg, rg, ng = orig(X, y, day, "cuda")
    _, cc, rc, nc = orig(X, y, day, "cpu")
    zero_cols = np.where(np.abs(X).sum(0) == 0)[0].tolist()
    out = {"rows": int(X.shape[0]), "K": int(X.shape[1]), "zero_cols": zero_cols,
           "pinv_gpu": int(ng), "pinv_cpu": int(nc),
           "coef_nan_gpu": int(np.isnan(cg).any(1).sum()), "coef_nan_cpu": int(np.isnan(cc).any(1).sum()),
           "coef_maxdiff": float(np.nanmax(np.abs(cg - cc))),
           "coef_scale": float(np.nanmax(np.abs(cc))),
           "F_nan_gpu": int(np.isnan(bg.F).sum()), "F_nan_cpu": int(np.isnan(bc.F).sum()),
           "ivol_nan_gpu": int(np.isnan(bg.ivol).sum()), "ivol_nan_cpu": int(np.isnan(bc.ivol).sum())}
    bad = np.where(np.isnan(cg).any(1))[0]
    if bad.size:
        gs = np.r_[0, np.flatnonzero(np.diff(day)) + 1, len(day)]
        dd = int(bad[0])
        Xd = X[gs[dd]:gs[dd + 1]]
        out["first_nan_day"] = {"day": dd, "rows": int(Xd.shape[0]),
                                "rank": int(np.linalg.matrix_rank(Xd)),
                                "coef_gpu": cg[dd].tolist(), "coef_cpu": cc[dd].tolist()}
    nanF = np.argwhere(np.isnan(bg.F))
    if nanF.size:
        out["first_nan_F"] = nanF[:5].tolist()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
