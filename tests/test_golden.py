"""Parity against golden fixtures frozen from the REFERENCE's own functions
(tools/make_golden.py: General_functions.py / Estimate Covariance Matrix.py functions run on
synthetic inputs).  Runs without the reference checkout."""
import os

import numpy as np
import pandas as pd
import pytest
import torch

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _npz(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


@pytest.mark.parametrize("tag", ["n40", "n25_notc", "prod_tc", "prod_notc"])
def test_m_func_golden(tag):
    from pfml.ops.linalg import m_func
    z = _npz(f"m_func_{tag}.npz")
    w, mu, rf, g = z["scal"]
    got = m_func(torch.tensor(z["sigma"])[None], torch.tensor(z["lam"])[None],
                 torch.tensor([w]), torch.tensor([rf]), float(mu), float(g), 10)[0].numpy()
    ref = z["m"]
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-12


def test_create_cov_golden():
    from pfml.models.risk import BarraCov, create_cov
    z = _npz("create_cov.npz")
    b = BarraCov(months=np.array([0]), offsets=np.array([0, len(z["ids"])]), ids=z["ids"],
                 X=z["X"], ivol=z["ivol"], F=z["F"][None], factors=["f"] * z["F"].shape[0])
    _, S = create_cov(b, 0, ids=z["sub"])
    assert np.allclose(S, z["sigma"], rtol=1e-13, atol=1e-16)


def test_weighted_cov_cor_golden():
    from pfml.models.risk import weighted_cov
    z = _npz("weighted_cov.npz")
    X, w = torch.tensor(z["X"])[None], torch.tensor(z["w"])[None]
    assert np.allclose(weighted_cov(X, w, cor=False)[0].numpy(), z["cov"], rtol=1e-12)
    assert np.allclose(weighted_cov(X, w, cor=True)[0].numpy(), z["cor"], rtol=1e-12)


def test_ewma_vol_golden():
    from pfml import runtime as rt
    z = _npz("ewma_vol.npz")
    lam = 0.5 ** (1 / 126)
    got = rt.ewma_vol(z["x"], np.array([0, len(z["x"])]), lam, 63)
    assert np.allclose(got, z["vol"], equal_nan=True, rtol=1e-13)
    short = z["x"][:50]
    got2 = rt.ewma_vol(short, np.array([0, 50]), lam, 63)
    assert np.all(np.isnan(got2)) and np.all(np.isnan(z["vol_short"]))


def test_investment_universe_golden():
    from pfml import runtime as rt
    z = _npz("universe.npz")
    got = rt.investment_universe(z["add"], z["delete"], np.array([0, len(z["add"])]))
    assert np.array_equal(got, z["included"])


def test_wealth_func_golden():
    from pfml.models.prep import wealth_func
    rf = pd.read_csv(os.path.join(G, "wealth_rf.csv"), parse_dates=["eom"])
    mk = pd.read_csv(os.path.join(G, "wealth_market.csv"), parse_dates=["eom_ret"])
    ref = pd.read_csv(os.path.join(G, "wealth_out.csv"), parse_dates=["eom"])
    got = wealth_func(1e10, pd.Timestamp("1994-12-31"), mk, rf)
    assert list(got.columns) == list(ref.columns)
    assert (got["eom"].values == ref["eom"].values).all()
    assert np.allclose(got["wealth"], ref["wealth"], rtol=1e-13)
    assert np.allclose(got["mu_ld1"], ref["mu_ld1"], equal_nan=True)


def test_categorize_sic_golden():
    from pfml.models.prep import categorize_sic
    ref = pd.read_csv(os.path.join(G, "ff12.csv"))
    assert (categorize_sic(ref["sic"].to_numpy()) == ref["ff12"].to_numpy()).all()


def test_lead_returns_golden():
    from pfml.models.prep import lead_returns
    inp = pd.read_csv(os.path.join(G, "lead_in.csv"), parse_dates=["eom"])
    ref = pd.read_csv(os.path.join(G, "lead_out.csv"), parse_dates=["eom"])
    got = lead_returns(inp, h=12).sort_values(["id", "eom"]).reset_index(drop=True)
    ref = ref.sort_values(["id", "eom"]).reset_index(drop=True)
    assert len(got) == len(ref)
    assert (got["id"].values == ref["id"].values).all()
    assert (got["eom"].values == ref["eom"].values).all()
    assert np.allclose(got["ret_ld1"], ref["ret_ld1"], rtol=1e-14)


def test_cluster_ranks_golden():
    from pfml.models.risk import cluster_ranks
    cd = pd.read_csv(os.path.join(G, "cluster_in.csv"))
    labels = pd.read_csv(os.path.join(G, "cluster_labels.csv"))
    ref = pd.read_csv(os.path.join(G, "cluster_out.csv"))
    feats = list(cd.columns)
    clusters, R = cluster_ranks(cd, labels, feats)
    assert clusters == ["a", "b", "c", "d"]
    assert np.allclose(R, ref[clusters].to_numpy(), rtol=1e-13)
