"""Risk-model kernels (csrc/risk.hip, K21-K23) vs the fp64 CPU oracle of the same op."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_daily_ols_matches_lstsq(gpu):
    from pfml.ops.risk_kernels import daily_ols
    rng = np.random.default_rng(0)
    K = 25
    sizes = [1, 30, 64, 65, 200, 513, 7]
    off = np.r_[0, np.cumsum(sizes)]
    R = off[-1]
    X = rng.standard_normal((R, K))
    X[:, :12] = (rng.integers(0, 12, R)[:, None] == np.arange(12)[None, :])   # FF12 dummies
    y = rng.standard_normal(R) * 0.02
    coef, resid, nbad = daily_ols(torch.tensor(X, device=gpu), torch.tensor(y, device=gpu),
                                  torch.tensor(off))
    coef, resid = coef.cpu().numpy(), resid.cpu().numpy()
    for d in range(len(sizes)):
        a, b = off[d], off[d + 1]
        Xd, yd = X[a:b], y[a:b]
        try:
            ref = np.linalg.solve(Xd.T @ Xd, Xd.T @ yd)
        except np.linalg.LinAlgError:
            ref = np.linalg.pinv(Xd.T @ Xd) @ (Xd.T @ yd)
        if b - a >= K and np.linalg.matrix_rank(Xd) == K:
            assert np.allclose(coef[d], ref, rtol=1e-8, atol=1e-10), d
            assert np.allclose(resid[a:b], yd - Xd @ ref, atol=1e-10), d
    # the 1-row day is exactly singular: pinv fallback applied
    assert nbad >= 1
    assert np.all(np.isfinite(coef)) and np.all(np.isfinite(resid))


def test_daily_ols_pinv_on_device(gpu):
    """Exactly singular days (duplicated factor column; an all-zero dummy) hit LinAlgError in
    the reference and take pinv(X'X) X'y: the kernel does that itself (Jacobi) - the
    minimum-norm coefficients match numpy's pinv, no host fallback runs."""
    from pfml.ops.risk_kernels import daily_ols
    rng = np.random.default_rng(3)
    K = 25
    sizes = [120, 80, 300]
    off = np.r_[0, np.cumsum(sizes)]
    X = rng.standard_normal((off[-1], K))
    y = rng.standard_normal(off[-1]) * 0.02
    X[off[0]:off[1], 24] = X[off[0]:off[1], 23]          # day 0: duplicated column
    X[off[1]:off[2], 5] = 0.0                            # day 1: empty dummy column
    coef, resid, nbad = daily_ols(torch.tensor(X, device=gpu), torch.tensor(y, device=gpu),
                                  torch.tensor(off))
    coef, resid = coef.cpu().numpy(), resid.cpu().numpy()
    assert nbad == 2
    for d in range(3):
        a, b = off[d], off[d + 1]
        Xd, yd = X[a:b], y[a:b]
        try:
            ref = np.linalg.solve(Xd.T @ Xd, Xd.T @ yd)
        except np.linalg.LinAlgError:
            ref = np.linalg.pinv(Xd.T @ Xd) @ (Xd.T @ yd)
        assert np.allclose(coef[d], ref, rtol=1e-7, atol=1e-10), (d, np.abs(coef[d] - ref).max())
        assert np.allclose(resid[a:b], yd - Xd @ ref, atol=1e-9), d


def test_ewma_factor_cov_matches_cov_wt(gpu):
    from pfml.ops.risk_kernels import ewma_factor_cov
    rng = np.random.default_rng(1)
    days, K, obs = 700, 25, 300
    fr = rng.standard_normal((days, K)) * 0.01 + 0.001
    tr = np.arange(obs, 0, -1, dtype=np.float64)
    w_cor = (0.5 ** (1 / 90.0)) ** tr
    w_var = (0.5 ** (1 / 30.0)) ** tr
    ends = np.array([5, 64, 300, 301, 512, 700])
    F_cpu, c_cpu, v_cpu = ewma_factor_cov(torch.tensor(fr), ends, obs, w_cor, w_var,
                                          return_parts=True)
    F, c, v = ewma_factor_cov(torch.tensor(fr, device=gpu), ends, obs, w_cor, w_var,
                              return_parts=True)
    assert torch.allclose(F.cpu(), F_cpu, rtol=1e-11, atol=1e-16)
    assert torch.allclose(c.cpu(), c_cpu, rtol=1e-11, atol=1e-12)
    assert torch.allclose(v.cpu(), v_cpu, rtol=1e-11, atol=1e-18)


def test_ewma_vol_matches_numba_semantics(gpu):
    from pfml import runtime as rt
    from pfml.ops.risk_kernels import ewma_vol
    rng = np.random.default_rng(2)
    sizes = [10, 63, 64, 65, 300, 1000, 130]
    gs = np.r_[0, np.cumsum(sizes)]
    x = rng.standard_normal(gs[-1]) * 0.02
    x[rng.random(gs[-1]) < 0.05] = np.nan
    x[gs[5]:gs[5] + 62] = np.nan          # only one valid obs in the start window -> all NaN
    x[gs[5] + 10] = 0.01
    lam = 0.5 ** (1 / 126)
    ref = rt.ewma_vol(x, gs, lam, 63)
    out = ewma_vol(torch.tensor(x, device=gpu), gs, lam, 63).cpu().numpy()
    assert np.array_equal(np.isnan(out), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.allclose(out[ok], ref[ok], rtol=1e-12, atol=0)


def test_estimate_cov_device_matches_pandas_form(gpu, small_data):
    """The batched S3 (segmented z-score / medians, integer-key merges) vs the pandas-bound
    form, both with the HIP OLS / EWMA kernels (the CPU OLS differs on the thin early days,
    where pinv of a numerically rank-deficient X'X is cutoff-sensitive)."""
    from pfml.models import risk
    chars, daily, labels = risk._load_risk_inputs(small_data)
    cs = small_data.settings["cov_set"]
    a = risk.estimate_cov_frames(chars, daily, labels, cs, "cuda")
    b = risk.estimate_cov_frames_pandas(chars, daily, labels, cs, "cuda")
    assert np.array_equal(a.ids, b.ids) and np.array_equal(a.offsets, b.offsets)
    assert np.allclose(a.X, b.X, rtol=1e-12, atol=1e-12, equal_nan=True)
    # a factor with no members on the small panel has sd 0 -> NaN correlations (cov.wt too)
    assert np.array_equal(np.isnan(a.F), np.isnan(b.F))
    assert np.allclose(a.F, b.F, rtol=1e-9, atol=1e-12 * np.nanmax(np.abs(b.F)), equal_nan=True)
    assert np.allclose(a.ivol, b.ivol, rtol=1e-9, atol=1e-10 * np.abs(b.ivol).max())


def test_factor_cov_zero_variance_modes_gpu(gpu):
    """A factor with no exposure (an all-zero return column: zero variance) on the device:
    compat mode gives the reference's weighted_cor_wt NaN correlations (General_functions.py:827:
    cov / outer(sd, sd), diagonal 1), so F is NaN in that row / column off the diagonal;
    corrected mode gives 0 there.  Every other entry matches the CPU oracle in both modes."""
    from zero_var_check import check_zero_variance_modes
    check_zero_variance_modes(gpu)
