"""Tiny end-to-end step used by ``__graft_entry__.smoke()`` and the smoke tests."""
from __future__ import annotations

import numpy as np
import torch

from ..config import Config
from ..utils.dates import mi_from_ym
from .search import PfmlReals, grid_search, validation_scores


def tiny_end_to_end(device: torch.device) -> dict:
    cfg = Config.default().override(["pf_ml.p_vec=[8,16]", "pf.dates.start_year=2001",
                                     "pf.dates.end_yr=2003"])
    G, P = 2, 17
    months = np.arange(mi_from_ym(1996, 1), mi_from_ym(2003, 11) + 1)
    T = len(months)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(G * T, 24, P, generator=g, dtype=torch.float64)
    D = (X.transpose(1, 2) @ X / 24).view(G, T, P, P).to(device)
    r = (0.1 * torch.randn(G, T, P, generator=g, dtype=torch.float64)).to(device)
    res = grid_search(PfmlReals(months, r, D), cfg)
    _, cum, rank = validation_scores(res.obj, 1, True)
    return {"beta": res.beta, "obj": res.obj, "cum_obj": cum, "rank": rank}
