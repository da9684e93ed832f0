"""L2 / L3 parity against the REFERENCE's own Prepare_Data.py and "Estimate Covariance
Matrix.py" (frozen by tools/make_golden_l2l3.py on the same synthetic raw files + L0 the
small_data fixture starts from).

Factors_processed: row count, per-column fingerprints over ALL rows and 1500 sampled rows
(ids, flags and dates exact, values at 1e-10); wealth_processed.csv and
cluster_labels_processed.csv; the Barra objects (fct_load / fct_cov / ivol_vec) of every month by
fingerprint and of three months element by element.  The device form of S3 is checked
against the same golden under -m gpu."""
import json
import os
import shutil
import sqlite3

import numpy as np
import pandas as pd
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_l2l3")
EXACT = {"id", "eom", "eom_ret", "valid", "valid_data", "valid_size", "sic", "ff49", "size_grp",
         "crsp_exchcd", "add", "delete", "valid_temp"}


def _num(col: pd.Series):
    if col.dtype == bool or col.dtype.kind == "b":
        return col.to_numpy().astype(np.float64)
    if np.issubdtype(col.dtype, np.datetime64):
        return col.to_numpy().astype("datetime64[D]").astype(np.int64).astype(np.float64)
    if col.dtype.kind in "iuf":
        return col.to_numpy(np.float64)
    return None


def _fp(a):
    a = np.asarray(a, np.float64).ravel()
    nan = np.isnan(a)
    v = a[~nan]
    return np.array([a.size, nan.sum(), v.sum(), np.abs(v).sum(), (v * v).sum()], np.float64)


def _close_fp(got, ref, rtol=1e-10):
    got, ref = np.asarray(got), np.asarray(ref)
    if got[0] != ref[0] or got[1] != ref[1]:
        return False
    scale = max(abs(ref[3]), 1e-300)
    return bool(abs(got[2] - ref[2]) <= rtol * scale and abs(got[3] - ref[3]) <= rtol * scale
                and abs(got[4] - ref[4]) <= rtol * max(abs(ref[4]), 1e-300))


def _engine_factors(data_dir):
    with sqlite3.connect(os.path.join(data_dir, "JKP_US_SP500.db")) as con:
        df = pd.read_sql_query("SELECT * FROM Factors_processed", con,
                               parse_dates=["eom", "eom_ret"])
    return df.sort_values(["id", "eom"]).reset_index(drop=True)


def test_factors_processed_matches_reference(small_data):
    meta = json.load(open(os.path.join(GOLD, "factors_meta.json")))
    fp = _engine_factors(small_data.run.data_dir)
    assert len(fp) == meta["rows"]
    missing = [c for c in meta["columns"] if c not in fp.columns]
    assert not missing, missing
    bad = []
    for c, ref in meta["fingerprint"].items():
        got = _fp(_num(fp[c]))
        if c in EXACT:
            if not np.array_equal(got, np.asarray(ref)):
                bad.append(c)
        elif not _close_fp(got, ref):
            bad.append(c)
    assert not bad, bad
    assert fp["ff12"].astype(str).value_counts().sort_index().to_dict() == meta["ff12_counts"]
    z = np.load(os.path.join(GOLD, "factors_sample.npz"), allow_pickle=False)
    rows, cols, vals = z["rows"], [str(c) for c in z["cols"]], z["values"]
    assert (fp["ff12"].astype(str).to_numpy()[rows] == z["ff12"]).all()
    for j, c in enumerate(cols):
        got, ref = _num(fp[c])[rows], vals[:, j]
        if c in EXACT:
            assert np.array_equal(got, ref, equal_nan=True), c
        else:
            assert np.allclose(got, ref, rtol=1e-10, atol=1e-14, equal_nan=True), c


def test_wealth_and_cluster_labels_match_reference(small_data):
    d = small_data.run.data_dir
    a = pd.read_csv(os.path.join(d, "wealth_processed.csv"))
    b = pd.read_csv(os.path.join(GOLD, "wealth_processed.csv"))
    assert list(a.columns) == list(b.columns) and len(a) == len(b)
    assert (a["eom"] == b["eom"]).all()
    for c in ("wealth", "mu_ld1"):
        assert np.allclose(a[c], b[c], rtol=1e-12, equal_nan=True), c
    a = pd.read_csv(os.path.join(d, "cluster_labels_processed.csv"))
    b = pd.read_csv(os.path.join(GOLD, "cluster_labels_processed.csv"))
    assert list(a.columns) == list(b.columns)
    pd.testing.assert_frame_equal(a, b, check_dtype=False)


def _check_barra(b):
    from pfml.utils.dates import month_end
    z = np.load(os.path.join(GOLD, "barra.npz"), allow_pickle=False)
    months = [str(pd.Timestamp(month_end(int(m))[0]).date()) for m in b.months]
    assert months == [str(m) for m in z["months"]]
    assert [str(f) for f in b.factors] == [str(f) for f in z["factors"]]
    for k, m in enumerate(b.months):
        ids, X, F, iv = b.slice(int(m))
        ref = z["fingerprints"][k]
        got = np.concatenate([_fp(X), _fp(F), _fp(iv), [float(np.asarray(ids, np.int64).sum())]])
        assert got[15] == ref[15], ("ids", months[k])
        for s in range(3):
            assert _close_fp(got[5 * s:5 * s + 5], ref[5 * s:5 * s + 5]), (months[k], s)
    for i in range(3):
        m = str(z[f"pick{i}_month"])
        mi = int(b.months[months.index(m)])
        ids, X, F, iv = b.slice(mi)
        assert np.array_equal(np.asarray(ids, np.int64), z[f"pick{i}_ids"])
        # entrywise to 1e-10 of each object's scale (near-zero factor covariances carry only
        # the rounding of the larger terms they are sums of; measured 4e-15 of max |F|)
        for got, ref in ((X, z[f"pick{i}_load"]), (F, z[f"pick{i}_cov"]),
                         (iv, z[f"pick{i}_ivol"])):
            assert np.allclose(got, ref, rtol=1e-10, atol=1e-10 * np.abs(ref).max()), m


def test_barra_cov_matches_reference(small_data):
    from pfml.models.risk import BarraCov
    _check_barra(BarraCov.load(os.path.join(small_data.run.data_dir, "Barra_Cov.npz")))


@pytest.mark.gpu
def test_barra_cov_device_matches_reference(small_data, tmp_path, gpu):
    """S3 on the MI355X (device daily panel, HIP OLS / EWMA kernels) vs the reference's L3."""
    from pfml.models import risk
    from pfml.models.risk import BarraCov
    d = str(tmp_path / "dev")
    shutil.copytree(small_data.run.data_dir, d)
    cfg = small_data.override([f"run.data_dir={d}"])
    risk.estimate_cov(cfg, device=str(gpu))
    _check_barra(BarraCov.load(os.path.join(d, "Barra_Cov.npz")))
