"""Stage tests on the synthetic small panel (CPU fp64 path) against independent oracles."""
import os

import numpy as np
import pandas as pd
import pytest
import torch

from oracle import month_ref


def _load(cfg):
    from pfml.config import get_features
    from pfml.data import io
    from pfml.models.risk import BarraCov
    d = cfg.run.data_dir
    chars = io.read_processed_chars(d, get_features())
    barra = BarraCov.load(os.path.join(d, "Barra_Cov.npz"))
    wealth = pd.read_csv(os.path.join(d, "wealth_processed.csv"), parse_dates=["eom"])
    rf = io.read_risk_free(d)
    return chars, barra, wealth, rf


def test_prep_outputs_schema(small_data):
    from pfml.data.io import CSV_COLUMNS
    d = small_data.run.data_dir
    w = pd.read_csv(os.path.join(d, "wealth_processed.csv"))
    assert list(w.columns) == CSV_COLUMNS["wealth_processed.csv"]
    cl = pd.read_csv(os.path.join(d, "cluster_labels_processed.csv"))
    assert list(cl.columns) == CSV_COLUMNS["cluster_labels_processed.csv"]
    assert cl.iloc[-1].tolist() == ["rvol_252d", -1, "low_risk"]
    chars, *_ = _load(small_data)
    assert chars["valid"].any()
    # every valid row has its full 12-month lookback (Prepare_Data.py:412-441)
    from pfml.utils.dates import month_index
    c = chars.sort_values(["id", "eom"])
    mi = month_index(c["eom"])
    lag = c.groupby("id")["eom"].shift(12)
    ok = ~lag.isna()
    diff = mi[ok.to_numpy()] - month_index(lag[ok])
    assert np.all(diff[c["valid"].to_numpy()[ok.to_numpy()]] == 12)
    feats = chars[[f for f in chars.columns if f.startswith("ret_12_1")]]
    assert feats.min().min() >= 0.0 and feats.max().max() <= 1.0


def test_wealth_func_matches_definition():
    from pfml.models.prep import wealth_func
    rf = pd.DataFrame({"eom": pd.date_range("2000-01-31", periods=5, freq="ME"),
                       "rf": [0.001, 0.002, 0.001, 0.0, 0.003]})
    mk = pd.DataFrame({"eom_ret": rf["eom"], "mkt_vw_exc": [0.01, -0.02, 0.03, 0.0, 0.01]})
    w = wealth_func(100.0, pd.Timestamp("2000-05-31"), mk, rf)
    tret = (mk["mkt_vw_exc"] + rf["rf"]).to_numpy()
    # backward cumulative product of (1 - tret), inclusive (quirk Q4)
    exp = 100.0 * np.cumprod((1 - tret)[::-1])[::-1]
    assert np.allclose(w["wealth"].to_numpy()[:-1], exp)
    assert w["eom"].iloc[0] == pd.Timestamp("1999-12-31")
    assert np.isnan(w["mu_ld1"].iloc[-1]) and w["wealth"].iloc[-1] == 100.0


def test_categorize_sic_examples():
    from pfml.models.prep import categorize_sic
    got = categorize_sic([150, 3711, 3715, 1311, 2834, 3693, 7372, 4813, 4911, 5311, 6021,
                          1000, np.nan])
    assert list(got) == ["NoDur", "Durbl", "Manuf", "Enrgy", "Hlth", "Hlth", "BusEq", "Telcm",
                         "Utils", "Shops", "Money", "Other", "Other"]


def test_barra_covariance_psd(small_data):
    from pfml.models.risk import create_cov
    _, barra, *_ = _load(small_data)
    assert barra.F.shape[1:] == (25, 25)
    mi = barra.months[len(barra.months) // 2]
    ids, S = create_cov(barra, mi)
    assert np.allclose(S, S.T)
    assert np.linalg.eigvalsh(S).min() > 0


def test_weighted_cov_matches_definition():
    from pfml.models.risk import weighted_cov
    rng = np.random.default_rng(0)
    X = rng.normal(size=(50, 4))
    w = rng.uniform(0.1, 1.0, 50)
    wn = w / w.sum()
    mu = wn @ X
    Xc = (X - mu) * np.sqrt(wn)[:, None]
    ref = Xc.T @ Xc / (1 - (wn ** 2).sum())
    got = weighted_cov(torch.tensor(X)[None], torch.tensor(w)[None], cor=False)[0].numpy()
    assert np.allclose(got, ref, rtol=1e-12)
    sd = np.sqrt(np.diag(ref))
    cref = ref / np.outer(sd, sd)
    np.fill_diagonal(cref, 1.0)
    gotc = weighted_cov(torch.tensor(X)[None], torch.tensor(w)[None], cor=True)[0].numpy()
    assert np.allclose(gotc, cref, rtol=1e-12)


def _oracle_month(cfg, chars, barra, wealth, rf, W, d):
    """Reference-order computation of one month (standardisation done pandas-style)."""
    from pfml.config import get_features
    from pfml.models.pfml_inputs import Panel, vol_scales
    from pfml.utils.dates import month_index, pfml_date_grids
    feats = get_features()
    panel = Panel.from_chars(chars, feats)
    grids = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"],
                            1971, 10)
    vol = vol_scales(panel, barra, grids["lb"])
    rows = panel.valid_rows(d)
    ids = panel.ids[rows]
    half = W.shape[1]
    S_win, gt_win = [], []
    for th in range(13):
        rr = panel.rows(d - th, ids)
        Z = panel.feats[rr] @ W
        s = np.concatenate([np.cos(Z), np.sin(Z)], 1)
        s = s - s.mean(0)
        s = np.concatenate([s, np.ones((len(rr), 1))], 1)        # feat_cons: rff..., constant
        s = s * np.sqrt(1.0 / (s ** 2).sum(0))
        s = s / vol[rr][:, None]
        S_win.append(s)
        g = (1 + panel.cols["tr_ld0"][rr]) / (1 + panel.cols["mu_ld0"][rr])
        gt_win.append(np.nan_to_num(g, nan=1.0))
    bids, X, F, iv = barra.slice(d)
    pos = np.searchsorted(bids, ids)
    Sigma = X[pos] @ F @ X[pos].T + np.diag(iv[pos])
    lam = panel.cols["lambda"][rows]
    w = wealth.set_index(month_index(wealth["eom"]))["wealth"][d]
    rfv = rf.set_index(month_index(rf["eom"]))["rf"][d]
    r = panel.cols["ret_ld1"][rows]
    out = month_ref(np.stack(S_win), np.stack(gt_win), r, Sigma, lam, w, rfv,
                    cfg.pf_set["mu"], cfg.pf_set["gamma_rel"])
    # feat_cons order (rff1_cos..rff_h_cos, rff1_sin.., constant) -> feat_all (constant first)
    perm = np.r_[2 * half, np.arange(2 * half)]
    rt, risk, tc, m = out
    return rt[perm], risk[np.ix_(perm, perm)], tc[np.ix_(perm, perm)]


def test_pfml_inputs_match_reference_order_oracle(small_data):
    from pfml.config import get_features
    from pfml.models.pfml_inputs import build_inputs, to_reference_order
    from pfml.utils.dates import pfml_date_grids
    cfg = small_data
    chars, barra, wealth, rf = _load(cfg)
    grids = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"],
                            1971, 10)
    months = grids["m2"][[0, 7, 40]]
    out = build_inputs(cfg, chars, barra, wealth, rf, "cpu", months=months, keep_risk_tc=True)
    Pm = cfg.p_max
    W = out.rff_w[0]
    for i, d in enumerate(months):
        rt, risk, tc = _oracle_month(cfg, chars, barra, wealth, rf, W, int(d))
        e_rt = to_reference_order(out.reals.r_tilde[0, i], Pm).numpy()
        e_rk = to_reference_order(out.reals.risk[0, i], Pm, dims=(0, 1)).numpy()
        e_tc = to_reference_order(out.reals.tc[0, i], Pm, dims=(0, 1)).numpy()
        assert np.abs(e_rt - rt).max() / np.abs(rt).max() < 1e-10
        assert np.abs(e_rk - risk).max() / np.abs(risk).max() < 1e-10
        assert np.abs(e_tc - tc).max() / np.abs(tc).max() < 1e-10
        # compat (Q1): both g identical
        assert torch.equal(out.reals.denom[0, i], out.reals.denom[1, i])


def test_s9_m_cache_fp64_only_and_universe_guard(small_data):
    """S4 keeps m_tilde for S9 only when its Sigma is fp64 (S9's recursion is specified in
    fp64 whatever run.precision says), and S9 reuses a kept month only for exactly its
    universe: same row count AND the same ids in the same order."""
    from pfml.models.pfml_inputs import build_inputs
    from pfml.models.portfolio import m_cache_positions
    from pfml.utils.dates import pfml_date_grids
    cfg = small_data
    chars, barra, wealth, rf = _load(cfg)
    grids = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"],
                            1971, 10)
    months = grids["m2"][[3, 9]]
    res = build_inputs(cfg, chars, barra, wealth, rf, "cpu", months=months, keep_m=months)
    mk = res.m_keep
    assert mk is not None and list(mk["months"]) == list(months)
    assert len(mk["ids"]) == 2 and all(len(i) == n for i, n in zip(mk["ids"], mk["n"]))
    low = cfg.override(["run.precision=fp32"])
    assert build_inputs(low, chars, barra, wealth, rf, "cpu", months=months,
                        keep_m=months).m_keep is None
    N = int(mk["mt"].shape[-1])
    ids = [np.asarray(i) for i in mk["ids"]]
    pos = m_cache_positions(mk, months, np.asarray(mk["n"]), ids, N, "cpu")
    assert pos is not None and pos.tolist() == [0, 1]
    swapped = [ids[0], ids[1][::-1].copy()]                 # same count, other row order
    assert m_cache_positions(mk, months, np.asarray(mk["n"]), swapped, N, "cpu") is None
    other = [ids[0], ids[1] + 1]                             # same count, other universe
    assert m_cache_positions(mk, months, np.asarray(mk["n"]), other, N, "cpu") is None
    assert m_cache_positions(mk, months[:1], np.asarray(mk["n"])[:1], ids[:1], N, "cpu").tolist() == [0]


def test_m_func_matches_sqrtm_reference():
    from oracle import m_func_ref
    from pfml.ops.linalg import m_func
    rng = np.random.default_rng(3)
    N, K = 40, 6
    X = rng.normal(size=(N, K))
    F = np.cov(rng.normal(size=(K, 100))) * 2e-2
    S = X @ F @ X.T + np.diag(rng.uniform(0.01, 0.03, N) ** 2 * 21)
    lam = 0.2 / rng.uniform(1e7, 1e9, N)
    ref = m_func_ref(3e9, 0.007, 0.002, S * 10, 10, lam, 10)
    got = m_func(torch.tensor(S)[None], torch.tensor(lam)[None], torch.tensor([3e9], dtype=torch.float64),
                 torch.tensor([0.002], dtype=torch.float64), 0.007, 10, 10)[0].numpy()
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-12


def test_pipeline_cli_resume_and_fault_injection(small_data, tmp_path):
    """End-to-end S4..S9 through the CLI entry point; a checkpointed rerun resumes (skips
    every stage); a poisoned S4 month, S5 coefficient cell and S9 w_start are detected and
    recomputed to identical outputs."""
    import shutil
    from pfml.cli import main
    from pfml.pipeline import Pipeline
    d = small_data.run.data_dir
    base = ["--data-dir", d, "--artifact-dir", str(tmp_path / "art"), "--device", "cpu",
            "--set", "pf.dates.start_year=1999", "--set", "pf.dates.end_yr=2012",
            "--set", "pf.dates.split_years=3", "--set", "cov_set.obs=400",
            "--set", "screens.start=1990-01-31", "--set", "screens.end=2012-12-31",
            "--set", "split.test_end=2012-12-31"]
    stages = "pfml-input,pfml-search-coef,pfml-hp-reals,pfml-aim,pfml-hps,pfml-best-hps"
    assert main(["stages", stages] + base + ["--checkpoint"]) == 0
    pf1 = pd.read_csv(os.path.join(d, "pf.csv"))
    summ1 = pd.read_csv(os.path.join(d, "pf_summary.csv"))
    # resume: invalidate the last two stages only -> they rerun from saved artifacts
    from pfml.utils.artifacts import ArtifactStore
    store = ArtifactStore(str(tmp_path / "art"))
    store.invalidate("pfml-hps")
    store.invalidate("pfml-best-hps")
    os.remove(os.path.join(d, "pf.csv"))
    assert main(["stages", stages] + base + ["--checkpoint"]) == 0
    pf_r = pd.read_csv(os.path.join(d, "pf.csv"))
    assert np.allclose(pf1[["r", "tc"]].to_numpy(), pf_r[["r", "tc"]].to_numpy(), rtol=1e-12)
    # fault injection: poisoned first month is recomputed -> identical outputs
    assert main(["stages", stages] + base + ["--set", "run.fault_inject=pfml-input"]) == 0
    pf2 = pd.read_csv(os.path.join(d, "pf.csv"))
    summ2 = pd.read_csv(os.path.join(d, "pf_summary.csv"))
    assert np.allclose(pf1[["r", "tc"]].to_numpy(), pf2[["r", "tc"]].to_numpy(), rtol=1e-10)
    assert np.allclose(summ1[["r", "sr"]].to_numpy(), summ2[["r", "sr"]].to_numpy(), rtol=1e-10)
    from pfml.utils.log import COUNTERS
    assert COUNTERS.as_dict().get("pfml_input.recomputed_months", 0) >= 1
    # S5: a poisoned coefficient cell is recomputed on the CPU oracle -> identical outputs
    assert main(["stages", stages] + base + ["--set", "run.fault_inject=pfml-search-coef"]) == 0
    pf3 = pd.read_csv(os.path.join(d, "pf.csv"))
    assert np.allclose(pf1[["r", "tc"]].to_numpy(), pf3[["r", "tc"]].to_numpy(), rtol=1e-10)
    assert COUNTERS.as_dict().get("pfml_search.recomputed_cells", 0) >= 1
    # S9: a poisoned w_start is detected and the recursion recomputed -> identical outputs
    assert main(["stages", "pfml-best-hps"] + base + ["--checkpoint", "--set",
                                                       "run.fault_inject=pfml-best-hps"]) == 0
    pf4 = pd.read_csv(os.path.join(d, "pf.csv"))
    assert np.allclose(pf1[["r", "tc"]].to_numpy(), pf4[["r", "tc"]].to_numpy(), rtol=1e-10)
    assert COUNTERS.as_dict().get("pfml_best_hps.recomputed", 0) >= 1


def test_gemm_fp32_precision_cpu():
    """precision=fp32 (sgemm operands/accumulation, fp64 in/out) honours op flags, alpha/beta
    and out, within fp32 rounding of the fp64 product."""
    import torch
    from pfml.ops.gemm import gemm, gemm_prec
    g = torch.Generator().manual_seed(1)
    A = torch.randn(3, 40, 30, generator=g, dtype=torch.float64)
    B = torch.randn(3, 50, 40, generator=g, dtype=torch.float64)
    C0 = torch.randn(3, 30, 50, generator=g, dtype=torch.float64)
    ref = gemm(A, B, trans_a=True, trans_b=True, alpha=0.5)
    got = gemm_prec(A, B, "fp32", trans_a=True, trans_b=True, alpha=0.5)
    assert got.dtype == torch.float64
    assert (got - ref).abs().max() / ref.abs().max() < 1e-5
    out = C0.clone()
    gemm_prec(A, B, "fp32", trans_a=True, trans_b=True, beta=2.0, out=out)
    assert torch.allclose(out, 2.0 * C0 + gemm(A, B, trans_a=True, trans_b=True), atol=1e-4)


def test_validation_scores_nan_semantics_cpu():
    """pandas semantics of PFML_hp_reals.py:109-122 on a NaN utility: expanding mean skips
    NaN, dense descending rank leaves NaN unranked."""
    import pandas as pd
    from pfml.models.search import validation_scores
    g = torch.Generator().manual_seed(0)
    obj = torch.randn(6, 1, 1, 4, generator=g, dtype=torch.float64)
    obj[:2, 0, 0, 1] = float("nan")
    obj[:, 0, 0, 3] = float("nan")
    _, cum, rank = validation_scores(obj, 0, False)
    df = pd.DataFrame({"obj": obj.reshape(6, 4).T.reshape(-1).numpy(),
                       "l": np.repeat(np.arange(4), 6), "m": np.tile(np.arange(6), 4)})
    df["cum"] = df.groupby("l")["obj"].transform(lambda x: x.expanding().mean())
    df["rank"] = df.groupby("m")["cum"].rank(method="dense", ascending=False)
    exp_c = df.pivot(index="m", columns="l", values="cum").to_numpy()
    exp_r = df.pivot(index="m", columns="l", values="rank").to_numpy()
    assert np.allclose(cum.reshape(6, 4).numpy(), exp_c, equal_nan=True, rtol=1e-14)
    assert np.array_equal(np.nan_to_num(rank.reshape(6, 4).numpy(), nan=-1),
                          np.nan_to_num(exp_r, nan=-1))


def test_estimate_cov_batched_matches_pandas_form(small_data):
    """S3 batched form (integer-key merges, segmented z-score / medians, no per-month loop)
    equals the pandas-bound form (groupby lambdas, frame merges, month loop)."""
    from pfml.models import risk
    chars, daily, labels = risk._load_risk_inputs(small_data)
    cs = small_data.settings["cov_set"]
    a = risk.estimate_cov_frames(chars, daily, labels, cs, "cpu")
    b = risk.estimate_cov_frames_pandas(chars, daily, labels, cs, "cpu")
    assert np.array_equal(a.months, b.months) and np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.ids, b.ids) and a.factors == b.factors
    assert np.allclose(a.X, b.X, rtol=1e-12, atol=1e-12, equal_nan=True)
    # (atol relative to the scale: a stock whose residuals are rounding noise has ivol ~1e-31)
    assert np.allclose(a.F, b.F, rtol=1e-10, atol=1e-12 * np.abs(b.F).max())
    assert np.allclose(a.ivol, b.ivol, rtol=1e-10, atol=1e-10 * np.abs(b.ivol).max())


def test_universe_plot_and_counts(small_data):
    """Prepare_Data.py:459-477: the investable-universe figure and its per-month valid counts
    are written next to the processed data."""
    from pfml.data import io
    from pfml.config import get_features
    d = os.path.join(small_data.run.data_dir, "plots")
    assert os.path.exists(os.path.join(d, "investable_universe.png"))
    vc = pd.read_csv(os.path.join(d, "universe_counts.csv"))
    chars = io.read_processed_chars(small_data.run.data_dir, get_features())
    ref = chars.loc[chars["valid"].astype(bool)].groupby("eom").size()
    assert vc["N"].tolist() == ref.tolist()
    assert vc["N"].sum() == int(chars["valid"].sum())


def test_pct_rank_rows_matches_pandas():
    """Native segmented percentile ranks of a row-major panel (runtime/panel.cpp
    pfml_pct_rank_rows) == pandas groupby(eom).rank(pct=True) per column, with exact zeros at
    0 (quirk Q15) and NaN imputed to 0.5 (Prepare_Data.py:324-374)."""
    from pfml import runtime as rt
    rng = np.random.default_rng(3)
    n, k = 4000, 6
    X = rng.integers(-3, 4, size=(n, k)).astype(float) + rng.random((n, k)) * (rng.random((n, k)) < 0.5)
    X[rng.random(X.shape) < 0.1] = np.nan
    month = rng.integers(0, 30, n)
    ids = rng.permutation(n)
    pe = np.lexsort((ids, month))
    seg = rt.group_starts(month[pe])
    got = rt.pct_rank_rows(X, pe, seg, zero_keep=True, impute=0.5)
    df = pd.DataFrame(X)
    ref = df.groupby(month).rank(pct=True).to_numpy()
    ref[X == 0.0] = 0.0
    ref[np.isnan(ref)] = 0.5
    assert np.allclose(got, ref, rtol=0, atol=1e-15)
    raw = rt.pct_rank_rows(X, pe, seg)
    assert np.array_equal(np.isnan(raw), np.isnan(X))


def test_factor_cov_zero_variance_modes_cpu():
    """CPU form of test_gpu_risk.py::test_factor_cov_zero_variance_modes_gpu: compat NaN
    correlations for a zero-variance factor (the reference's division), corrected 0."""
    from zero_var_check import check_zero_variance_modes
    check_zero_variance_modes("cpu")


def test_exposureless_factor_keeps_finite_cov_in_compat():
    """S3 compat: a factor with exactly-zero coefficients over a window (the device pinv's
    answer for a factor without exposure; the reference's LAPACK pinv leaves 1e-17 noise, so
    its correlations are finite) gets a zero F row / column, while an exposed factor with
    exactly constant returns keeps the reference's NaN correlations."""
    import torch
    from pfml.models.risk import _zero_exposureless
    from pfml.ops.risk_kernels import ewma_factor_cov
    g = torch.Generator().manual_seed(5)
    days, K, obs = 400, 5, 300
    fr = torch.randn(days, K, generator=g, dtype=torch.float64) * 0.01
    fr[:350, 1] = 0.0                       # no exposure until day 350
    fr[:, 3] = 0.002                        # exposed, exactly constant
    ends = np.array([340, 400])
    tr = np.arange(obs, 0, -1, dtype=np.float64)
    w = 0.99 ** tr
    Fm = ewma_factor_cov(fr, ends, obs, w, w, scale=21.0, nan_cor=True).numpy()
    assert np.isnan(Fm[0, 1, 0]) and np.isnan(Fm[0, 3, 0])
    _zero_exposureless(Fm, fr, ends, obs)
    assert (Fm[0, 1, :] == 0).all() and (Fm[0, :, 1] == 0).all()
    assert np.isnan(Fm[0, 3, 0]) and np.isnan(Fm[1, 3, 0])
    assert np.isfinite(Fm[1, 1, [0, 2, 4]]).all()           # exposed in window 2


def test_dgemm_auto_tile_rule():
    """Host mirror of the DGEMM's auto tile choice (ops/gemm.py _auto_cfg, csrc/gemm_f64.hip
    dgemm_chunk): 128 x 64 LDS-DMA tiles on the S4 shapes, 64 x 64 when a launch would have
    fewer 128 x 64 tiles than CUs (the per-rank inverse products of a many-GPU run), 128 x 128
    for large matrices, square 64 x 64 in the symmetric mode."""
    from pfml.ops.gemm import _SMALL_TILES, _auto_cfg
    assert _SMALL_TILES == 256
    assert _auto_cfg(490, 2006, 490, batch=92) == 8           # Horner step, 92-month rank
    assert _auto_cfg(245, 245, 245, batch=244) == 8           # inverse top level, one GPU
    assert _auto_cfg(245, 245, 245, batch=31) == 7            # the same at 31 months / batch
    assert _auto_cfg(490, 490, 490, sym=True, batch=1) == 7
    assert _auto_cfg(2048, 2048, 512, batch=1) == 6


def test_block_add_row_scale_cpu():
    """la.block_add on strided [B, M, N] views: X + Y, and X + diag(s) Y (omega_chg = omega -
    diag(D_0) omega_l1) exactly as torch's addcmul."""
    from pfml.ops import linalg as la
    g = torch.Generator().manual_seed(7)
    big = torch.randn(2, 3, 9, 40, generator=g, dtype=torch.float64)
    X, Y = big[0, :, :, :25], big[1, :, :, 5:30]
    s = torch.randn(3, 9, generator=g, dtype=torch.float64)
    out = torch.empty(3, 9, 25, dtype=torch.float64)
    assert torch.equal(la.block_add(out, X, Y), X + Y)
    assert torch.equal(la.block_add(out, X, Y, y_row_scale=-s),
                       torch.addcmul(X, -s.unsqueeze(-1), Y))
