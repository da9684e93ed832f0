"""S4-S9 parity against outputs frozen from the REFERENCE's own stage scripts
(tools/make_golden_pipeline.py exec'd PFML_Input_Data.py ... PFML_best_hps.py verbatim on this
small synthetic dataset): per-month r_tilde / risk / tc / denom (PFML_Input_Data.py:318-491),
ridge coefficients incl. lambda = 0 (PFML_Search_Coef.py:102-137), validation.csv rows with the
Q2 accumulation, expanding-mean cum_obj and dense rank (PFML_hp_reals.py:60-130), and
weights.csv / pf.csv / pf_summary.csv (PFML_best_hps.py:137-358), compat mode, fp64; the CPU
path, and (``-m gpu``) the whole pipeline on the device - every HIP stage against the
reference's own numbers.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest
import torch

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_pipeline")
RTOL = 1e-10


@pytest.fixture(scope="module", params=["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def ref_run(request, tmp_path_factory):
    """The golden's inputs regenerated through this engine's L0-L3 (deterministic), then the
    engine's pipeline from pfml-input to pfml-best-hps on them (CPU oracle or device)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(G), "..", "..", "tools"))
    import make_golden_pipeline as mk
    from pfml.config import get_features
    from pfml.pipeline import Pipeline
    meta = json.load(open(os.path.join(G, "meta.json")))
    d = str(tmp_path_factory.mktemp("ref_pipeline"))
    cfg = mk.engine_inputs(d)
    mk.small_rff_w(d, len(get_features()), cfg.p_max // 2, seed=meta["rff_w_seed"])
    if not mk.fingerprint_matches(mk.input_fingerprint(d), meta["input_fingerprint"]):
        pytest.fail("regenerated L0-L3 inputs differ from the golden's (L2/L3 changed?): "
                    "re-freeze with tools/make_golden_pipeline.py")
    cfg = cfg.override([f"run.artifact_dir={os.path.join(d, 'art')}"])
    p = Pipeline(cfg, device=request.param)
    p.run(["pfml-input", "pfml-search-coef", "pfml-hp-reals", "pfml-aim", "pfml-hps",
           "pfml-best-hps"])
    return cfg, p, d


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def test_s4_summands_match_reference(ref_run):
    from pfml.data import io
    from pfml.models.pfml_inputs import build_inputs, to_reference_order
    from pfml.models.risk import BarraCov
    from pfml.config import get_features
    from pfml.utils.dates import month_index
    cfg, p, d = ref_run
    z = np.load(os.path.join(G, "s4_reals.npz"), allow_pickle=False)
    months = month_index(pd.to_datetime(z["months"]))
    st = p.state
    out = build_inputs(cfg, st["chars"], st["barra"], st["wealth"], st["risk_free"], p.device,
                       months=months, keep_risk_tc=True)
    Pm = cfg.p_max
    for i in range(len(months)):
        rt = to_reference_order(out.reals.r_tilde[0, i], Pm).cpu().numpy()
        rk = to_reference_order(out.reals.risk[0, i], Pm, dims=(0, 1)).cpu().numpy()
        tc = to_reference_order(out.reals.tc[0, i], Pm, dims=(0, 1)).cpu().numpy()
        dn = to_reference_order(out.reals.denom[0, i], Pm, dims=(0, 1)).cpu().numpy()
        assert _rel(rt, z[f"r_tilde_{i}"]) < RTOL
        assert _rel(rk, z[f"risk_{i}"]) < RTOL
        assert _rel(tc, z[f"tc_{i}"]) < RTOL
        assert _rel(dn, z[f"denom_{i}"]) < RTOL


def test_ridge_coefficients_match_reference(ref_run):
    cfg, p, d = ref_run
    z = np.load(os.path.join(G, "coef.npz"), allow_pickle=False)
    grid = p.state["grid"]
    years = list(np.asarray(grid.years_local))
    for key in z.files:
        y, pp, li = (int(v) for v in key.split("_"))
        b = grid.beta[0, years.index(y), cfg.p_vec.index(pp), li, : pp + 1].cpu().numpy()
        h = pp // 2
        # internal [const, cos1, sin1, ...] -> reference [const, cos1..cos_h, sin1..sin_h]
        perm = np.r_[0, 1 + 2 * np.arange(h), 2 + 2 * np.arange(h)]
        assert _rel(b[perm], z[key]) < 1e-9, key


def test_validation_rows_match_reference(ref_run):
    cfg, p, d = ref_run
    ref = pd.read_csv(os.path.join(G, "validation_sample.csv"))
    got = pd.read_csv(os.path.join(d, "validation.csv"))
    meta = json.load(open(os.path.join(G, "meta.json")))
    assert len(got) == meta["validation_rows"]
    assert list(got.columns) == [c for c in ref.columns if c != "row"]
    g = got.iloc[ref["row"].to_numpy()]
    for c in ("eom", "eom_ret"):
        assert (pd.to_datetime(g[c]).to_numpy() == pd.to_datetime(ref[c]).to_numpy()).all(), c
    for c in ("l", "p", "hp_end", "g", "rank"):
        assert (g[c].to_numpy() == ref[c].to_numpy()).all(), c
    for c in ("obj", "cum_obj"):
        assert np.allclose(g[c].to_numpy(), ref[c].to_numpy(), rtol=RTOL, atol=1e-14), c


@pytest.mark.parametrize("name", ["weights.csv", "pf.csv", "pf_summary.csv"])
def test_portfolio_csvs_match_reference(ref_run, name):
    cfg, p, d = ref_run
    ref = pd.read_csv(os.path.join(G, name))
    got = pd.read_csv(os.path.join(d, name))
    assert list(got.columns) == list(ref.columns)
    assert len(got) == len(ref)
    for c in ref.columns:
        if ref[c].dtype.kind in "fc":
            assert np.allclose(got[c].to_numpy(), ref[c].to_numpy(), rtol=RTOL, atol=1e-14,
                               equal_nan=True), (name, c, _rel(got[c].fillna(0), ref[c].fillna(0)))
        else:
            assert (got[c].astype(str).to_numpy() == ref[c].astype(str).to_numpy()).all(), (name, c)
