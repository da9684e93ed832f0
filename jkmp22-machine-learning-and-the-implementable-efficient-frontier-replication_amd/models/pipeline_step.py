"""Tiny end-to-end step used by ``__graft_entry__.smoke()`` and the smoke tests: the S4
per-month input step (RFF signals, vol scales, Barra Sigma, m_func, the (24) Horner chains,
the LU solves, the (25) summands) for a few PFML months of a small synthetic universe,
followed by the S5 + S6 grid search (window sums, ridge grid, utilities, scores) on them."""
from __future__ import annotations

import numpy as np
import torch

from ..config import Config
from ..utils.dates import pfml_date_grids
from .search import PfmlReals, grid_search, validation_scores


def tiny_end_to_end(device: torch.device) -> dict:
    from ..data.synthetic import engine_inputs
    from .pfml_inputs import make_s4_plan, run_plan
    cfg = Config.default().override(["pf_ml.p_vec=[8,16]", "pf.dates.start_year=2001",
                                     "pf.dates.end_yr=2003"])
    cfg.run.compat_mode = False                     # two distinct g signal blocks
    chars, barra, wealth, rf = engine_inputs(n_stocks=40, start="1993-01-31",
                                             end="2004-12-31")
    grids = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"],
                            2001, 10)
    m2 = grids["m2"]
    months = m2[(m2 >= 1997 * 12) & (m2 <= 2003 * 12 + 10)]
    plan = make_s4_plan(cfg, chars, barra, wealth, rf, device, months)
    inp = run_plan(plan, cfg)
    reals = PfmlReals(months, inp.reals.r_tilde, inp.reals.denom)
    res = grid_search(reals, cfg)
    _, cum, rank = validation_scores(res.obj, 1, False)
    return {"s4_months": len(months), "r_tilde": inp.reals.r_tilde, "denom": inp.reals.denom,
            "signal_t0": inp.signal_t[0][0], "beta": res.beta, "obj": res.obj,
            "cum_obj": cum, "rank": rank}
