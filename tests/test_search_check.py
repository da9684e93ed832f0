"""``--check``: the sampled fp64 CPU-oracle comparison of the grid search."""
import numpy as np
import pytest
import torch


def _reals(device):
    from pfml.config import Config
    from pfml.models.search import PfmlReals
    from pfml.utils.dates import mi_from_ym
    cfg = Config.default().override(["pf_ml.p_vec=[8,16]", "pf.dates.start_year=2002",
                                     "pf.dates.end_yr=2006"])
    G, P = 2, 17
    months = np.arange(mi_from_ym(1995, 1), mi_from_ym(2006, 11) + 1)
    g = torch.Generator().manual_seed(3)
    X = torch.randn(G * len(months), 30, P, generator=g, dtype=torch.float64)
    D = (X.transpose(1, 2) @ X / 30).view(G, len(months), P, P)
    r = 0.1 * torch.randn(G, len(months), P, generator=g, dtype=torch.float64)
    return cfg, PfmlReals(months, r.to(device), D.to(device).contiguous())


def _run(device):
    from pfml.models.search import check_against_oracle, grid_search
    cfg, reals = _reals(device)
    grid = grid_search(reals, cfg)
    return check_against_oracle(grid, reals, cfg, ncells=4)


def test_check_cpu():
    out = _run("cpu")
    assert out["cells"] == 4
    assert out["beta_max_rel_err"] < 1e-10 and out["obj_max_rel_err"] < 1e-10


@pytest.mark.gpu
def test_check_gpu(gpu):
    out = _run(gpu)
    assert out["cells"] == 4
    assert out["beta_max_rel_err"] < 1e-8 and out["obj_max_rel_err"] < 1e-8


def test_cli_check_flag():
    from pfml.cli import main
    import argparse  # noqa: F401
    with pytest.raises(SystemExit):
        main(["--help"])


def test_nonfinite_cells_recomputed_on_cpu_oracle():
    """S5 failure recovery: a poisoned (g, year, p) cell is detected and its
    coefficients and validation utilities are recomputed from scratch by the fp64 CPU oracle,
    matching the clean grid search."""
    import numpy as np
    import torch
    from pfml.config import Config
    from pfml.models.search import (PfmlReals, grid_search, nonfinite_cells, recompute_cells)
    from pfml.utils.dates import mi_from_ym
    cfg = Config.default().override(["pf_ml.p_vec=[8,16]", "pf.dates.start_year=2001",
                                     "pf.dates.end_yr=2006"])
    G, P = 2, 17
    months = np.arange(mi_from_ym(1995, 1), mi_from_ym(2006, 11) + 1)
    T = len(months)
    g = torch.Generator().manual_seed(3)
    X = torch.randn(G * T, 30, P, generator=g, dtype=torch.float64)
    D = (X.transpose(1, 2) @ X / 30).view(G, T, P, P)
    r = 0.1 * torch.randn(G, T, P, generator=g, dtype=torch.float64)
    reals = PfmlReals(months, r, D)
    clean = grid_search(reals, cfg)
    grid = grid_search(reals, cfg)
    assert nonfinite_cells(grid) == []
    grid.beta[1, 2, 1, 40, 3] = float("nan")
    grid.beta[0, 0, 0, :, 0] = float("inf")
    yi = 2
    rows = np.nonzero(grid.val_year == grid.years_local[yi])[0]
    grid.obj[rows, 1, 1] = float("nan")
    bad = nonfinite_cells(grid)
    assert bad == [(0, 0, 0), (1, 2, 1)]
    res = recompute_cells(grid, reals, bad)
    assert res == {"recomputed": 2, "singular": 0}
    assert nonfinite_cells(grid) == []
    assert torch.allclose(grid.beta, clean.beta, rtol=1e-10, atol=1e-14)
    assert torch.allclose(grid.obj, clean.obj, rtol=1e-10, atol=1e-14)


def test_coop_k_policy_big_cells_share(monkeypatch):
    """The cooperative band reduction's workgroups per big cell (ops/ridge.py::coop_k): the
    p = 512 cells share ~42 % of the CUs - K = 1 / 2 / 4 / 8 for the 106 / 53 / 27 / 13 big
    cells of a 1 / 2 / 4 / 8-rank grid (the measured optimum, profiles/r04_coop_k_sweep.json),
    16 at most, 1 for the smaller cells; PFML_COOP_K forces the big cells' K."""
    from pfml.ops.ridge import COOP_KMAX, coop_k
    monkeypatch.delenv("PFML_COOP_K", raising=False)
    for nbig, want in ((106, 1), (53, 2), (27, 4), (26, 4), (14, 8), (13, 8), (1, COOP_KMAX)):
        k = coop_k(np.array([513] * nbig + [257, 129, 65]), 256)
        assert (k[:nbig] == want).all() and (k[nbig:] == 1).all(), (nbig, k[:3])
    assert (coop_k(np.array([129] * 5 + [65]), 256) == 1).all()   # no n > 256 cell: K = 1
    monkeypatch.setenv("PFML_COOP_K", "3")
    assert coop_k(np.array([513] * 106 + [65]), 256)[0] == 3


@pytest.mark.gpu
def test_coop_timeout_poisons_and_guard_recovers(gpu, monkeypatch):
    """A cooperative hand-off that times out never yields silent garbage: with the poll bound
    forced down to one poll (K = 2 workgroups per big cell) the timed-out cells come back as
    NaN betas, are counted (coop_errors), and the S5 recovery (nonfinite_cells ->
    recompute_cells, the reference's np.linalg.solve per lambda) ends with the CPU oracle's
    betas and utilities (PFML_Search_Coef.py:131-133)."""
    from pfml.config import Config
    from pfml.models.search import (PfmlReals, grid_search, nonfinite_cells, recompute_cells)
    from pfml.ops import ridge as rg
    from pfml.utils.dates import mi_from_ym
    cfg = Config.default().override(["pf_ml.p_vec=[32,64]", "pf.dates.start_year=2002",
                                     "pf.dates.end_yr=2006"])
    G, P = 2, 65
    months = np.arange(mi_from_ym(1995, 1), mi_from_ym(2006, 11) + 1)
    g = torch.Generator().manual_seed(5)
    X = torch.randn(G * len(months), 90, P, generator=g, dtype=torch.float64)
    D = (X.transpose(1, 2) @ X / 90).view(G, len(months), P, P)
    r = 0.1 * torch.randn(G, len(months), P, generator=g, dtype=torch.float64)
    clean = grid_search(PfmlReals(months, r, D), cfg)
    reals = PfmlReals(months, r.to(gpu), D.to(gpu).contiguous())
    monkeypatch.setenv("PFML_COOP_K", "2")
    rg.set_coop_spin_max(1)
    try:
        grid = grid_search(reals, cfg, gather=False)
        nto = rg.coop_errors()
    finally:
        rg.set_coop_spin_max(0)
    assert nto > 0
    bad = nonfinite_cells(grid)
    assert len(bad) >= 1
    res = recompute_cells(grid, reals, bad)
    assert res["recomputed"] == len(bad) and res["singular"] == 0
    assert nonfinite_cells(grid) == []
    assert torch.allclose(grid.beta.cpu(), clean.beta, rtol=1e-9, atol=1e-12)
    assert torch.allclose(grid.obj.cpu(), clean.obj, rtol=1e-9, atol=1e-12)
    # back at the default bound: no timeouts
    grid2 = grid_search(reals, cfg, gather=False)
    assert rg.coop_errors() == 0
    assert torch.allclose(grid2.beta.cpu(), clean.beta, rtol=1e-9, atol=1e-12)
