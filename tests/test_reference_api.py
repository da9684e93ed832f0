"""pfml.reference_api - the reference-named function surface - against the golden fixtures
frozen from the reference's own functions (tests/golden, tools/make_golden.py).  Where no
fixture exists (mean / median lead imputation, the best_hps helpers) the expected values are
the reference behaviour restated in plain pandas ("parity unpinned": no reference output
covers them)."""
import os

import numpy as np
import pandas as pd
import pytest

from pfml import reference_api as ra

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

NAMES = {"get_settings", "get_features", "wealth_func", "long_horizon_ret", "categorize_sic",
         "size_screen_fun", "investment_universe", "addition_deletion_fun", "ecdf_transform",
         "build_cluster_ranks", "weighted_cov_wt", "weighted_cor_wt", "pfml_feat_fun",
         "create_cov", "create_lambda", "m_func", "rff", "denom_sum_fun", "ewma_vol",
         "initial_weights_new", "compute_stats", "pf_ts_fun"}


def _npz(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_surface_complete():
    assert NAMES <= set(ra.__all__)
    for n in NAMES:
        assert callable(getattr(ra, n)), n


@pytest.mark.parametrize("tag", ["n40", "n25_notc"])
def test_m_func(tag):
    z = _npz(f"m_func_{tag}.npz")
    w, mu, rf, g = z["scal"]
    got = ra.m_func(w, mu, rf, z["sigma"] * g, g, np.diag(z["lam"]), 10)
    assert np.abs(got - z["m"]).max() / np.abs(z["m"]).max() < 1e-12


def test_create_cov_and_lambda():
    z = _npz("create_cov.npz")
    ids = z["ids"]
    x = {"fct_load": pd.DataFrame(z["X"], index=ids), "fct_cov": pd.DataFrame(z["F"]),
         "ivol_vec": pd.Series(z["ivol"], index=ids)}
    S = ra.create_cov(x, ids=z["sub"])
    assert isinstance(S, pd.DataFrame) and list(S.index) == list(z["sub"])
    assert np.allclose(S.to_numpy(), z["sigma"], rtol=1e-13, atol=1e-16)
    lam = {int(i): 0.1 * (k + 1) for k, i in enumerate(ids)}
    got = np.diag(ra.create_lambda(lam, [int(i) for i in z["sub"]]))
    assert np.allclose(got, [lam[int(i)] for i in z["sub"]])
    assert np.array_equal(ra.create_lambda(np.arange(5.0), [1, 3]), np.diag([1.0, 3.0]))


def test_weighted_cov_cor():
    z = _npz("weighted_cov.npz")
    df = pd.DataFrame(z["X"], columns=[f"c{i}" for i in range(z["X"].shape[1])])
    cov = ra.weighted_cov_wt(df, z["w"])
    cor = ra.weighted_cor_wt(df, z["w"])
    assert list(cov.columns) == list(df.columns) and list(cor.index) == list(df.columns)
    assert np.allclose(cov.to_numpy(), z["cov"], rtol=1e-12)
    assert np.allclose(cor.to_numpy(), z["cor"], rtol=1e-12)
    assert np.all(np.diag(cor.to_numpy()) == 1.0)


def test_ewma_vol_and_universe():
    z = _npz("ewma_vol.npz")
    lam = 0.5 ** (1 / 126)
    assert np.allclose(ra.ewma_vol(z["x"], lam, 63), z["vol"], equal_nan=True, rtol=1e-13)
    assert np.all(np.isnan(ra.ewma_vol(z["x"][:50], lam, 63)))
    u = _npz("universe.npz")
    assert np.array_equal(ra.investment_universe(u["add"], u["delete"]), u["included"])


def test_wealth_sic_features():
    rf = pd.read_csv(os.path.join(G, "wealth_rf.csv"), parse_dates=["eom"])
    mk = pd.read_csv(os.path.join(G, "wealth_market.csv"), parse_dates=["eom_ret"])
    ref = pd.read_csv(os.path.join(G, "wealth_out.csv"), parse_dates=["eom"])
    got = ra.wealth_func(1e10, "1994-12-31", mk, rf)
    assert list(got.columns) == list(ref.columns)
    assert np.allclose(got["wealth"], ref["wealth"], rtol=1e-13)
    ff = pd.read_csv(os.path.join(G, "ff12.csv"))
    assert (ra.categorize_sic(ff["sic"].to_numpy()) == ff["ff12"].to_numpy()).all()
    assert ra.categorize_sic(float(ff["sic"].iloc[0])) == ff["ff12"].iloc[0]
    assert ra.pfml_feat_fun(4) == ["constant", "rff1_cos", "rff2_cos", "rff1_sin", "rff2_sin"]
    assert len(ra.get_features()) == 115
    settings, pf_set = ra.get_settings()
    assert pf_set["gamma_rel"] == 10


def test_long_horizon_ret():
    inp = pd.read_csv(os.path.join(G, "lead_in.csv"), parse_dates=["eom"])
    ref = pd.read_csv(os.path.join(G, "lead_out.csv"), parse_dates=["eom"])
    cols = [f"ret_ld{l}" for l in range(1, 13)]
    got = ra.long_horizon_ret(inp, 12)
    assert list(got.columns) == ["id", "eom"] + cols
    assert not got[cols].isna().any().any()
    got = got.sort_values(["id", "eom"]).reset_index(drop=True)
    ref = ref.sort_values(["id", "eom"]).reset_index(drop=True)
    assert (got["id"].values == ref["id"].values).all()
    assert np.allclose(got["ret_ld1"], ref["ret_ld1"], rtol=1e-14)
    # mean / median (parity unpinned): the per-eom column fill of General_functions.py:282-286
    raw = ra.long_horizon_ret(inp, 12, impute="none")
    assert raw[cols].isna().any().any()
    for how in ("mean", "median"):
        exp = raw.copy()
        # (groupby's own mean / median: an all-NaN group gives NaN without numpy's warning)
        exp[cols] = raw[cols].fillna(raw.groupby("eom")[cols].transform(how))
        pd.testing.assert_frame_equal(ra.long_horizon_ret(inp, 12, impute=how), exp)


def test_size_screen_fun():
    chars = pd.DataFrame({"eom": pd.to_datetime(["2001-01-31"] * 4),
                          "me": [4.0, 1.0, 3.0, 2.0], "valid_data": [True, True, True, False],
                          "size_grp": ["mega", "micro", "large", "small"]})
    c = chars.copy()
    ra.size_screen_fun(c, "all")
    assert c["valid_size"].tolist() == [True, True, True, False]
    c = chars.copy()
    ra.size_screen_fun(c, "top2")
    assert c["valid_size"].tolist() == [True, False, True, False]
    with pytest.raises(ValueError):
        ra.size_screen_fun(chars.copy(), "weird")


def test_ecdf_and_cluster_ranks():
    e = ra.ecdf_transform(pd.Series([3.0, np.nan, 1.0, 2.0, 2.0]))
    assert np.allclose(e.to_numpy(), [1.0, np.nan, 0.25, 0.75, 0.75], equal_nan=True)
    cd = pd.read_csv(os.path.join(G, "cluster_in.csv"))
    labels = pd.read_csv(os.path.join(G, "cluster_labels.csv"))
    ref = pd.read_csv(os.path.join(G, "cluster_out.csv"))
    got = ra.build_cluster_ranks(cd, labels, ["a", "b", "c", "d"], list(cd.columns))
    assert np.allclose(got.to_numpy(), ref[["a", "b", "c", "d"]].to_numpy(), rtol=1e-13)


def test_denom_sum_and_rff():
    rng = np.random.default_rng(0)
    mats = [rng.normal(size=(4, 4)) for _ in range(5)]
    train = {pd.Timestamp(2000, m + 1, 28): {"denom": d, "r_tilde": None}
             for m, d in enumerate(mats)}
    assert np.allclose(ra.denom_sum_fun(train), sum(mats))
    X, W = rng.normal(size=(10, 3)), rng.normal(size=(3, 4))
    out = ra.rff(X, W=W, g=123.0)
    assert np.allclose(out["X_cos"], np.cos(X @ W)) and np.allclose(out["X_sin"], np.sin(X @ W))
    assert ra.rff(X, p=8, g=0.5, seed=1)["W"].shape == (3, 4)


def test_best_hps_helpers():
    d = pd.DataFrame({"id": [1, 2, 3, 1, 2],
                      "eom": pd.to_datetime(["2001-01-31"] * 3 + ["2001-02-28"] * 2),
                      "me": [1.0, 3.0, 4.0, 2.0, 2.0]})
    vw = ra.initial_weights_new(d, "vw")
    assert list(vw.columns) == ["id", "eom", "w_start", "w"]
    assert np.allclose(vw["w_start"].iloc[:3], [0.125, 0.375, 0.5])
    assert vw["w_start"].iloc[3:].isna().all() and vw["w"].isna().all()
    assert np.allclose(ra.initial_weights_new(d, "ew")["w_start"].iloc[:3], 1 / 3)
    with pytest.raises(ValueError):
        ra.initial_weights_new(d, "xx")
    grp = pd.DataFrame({"w": [0.5, -0.2], "w_start": [0.4, 0.0], "ret_ld1": [0.01, 0.02],
                        "lambda": [1e-3, 2e-3], "wealth": [1e6, 1e6]})
    s = ra.compute_stats(grp)
    assert np.isclose(s["inv"], 0.7) and np.isclose(s["shorting"], 0.2)
    assert np.isclose(s["turnover"], 0.3) and np.isclose(s["r"], 0.001)
    assert np.isclose(s["tc"], 1e6 / 2 * (1e-3 * 0.01 + 2e-3 * 0.04))
    data = pd.DataFrame({"id": [1, 2, 1, 2],
                         "eom": pd.to_datetime(["2001-01-31"] * 2 + ["2001-02-28"] * 2),
                         "ret_ld1": [0.01, -0.02, 0.03, 0.0], "lambda": [1e-3, 2e-3, 1e-3, 2e-3]})
    w = data[["id", "eom"]].assign(w=[0.6, 0.4, 0.5, 0.5], w_start=[0.5, 0.5, 0.55, 0.45])
    wealth = pd.DataFrame({"eom": pd.to_datetime(["2001-01-31", "2001-02-28"]),
                           "wealth": [1e9, 1.1e9]})
    out = ra.pf_ts_fun(w, data, wealth, 10)
    assert list(out.columns) == ["inv", "shorting", "turnover", "r", "tc", "eom_ret"]
    for k, (_, grp) in enumerate(data.merge(w).merge(wealth).groupby("eom")):
        s = ra.compute_stats(grp)
        for c in ("inv", "shorting", "turnover", "r", "tc"):
            assert np.isclose(out[c].iloc[k], s[c]), c
