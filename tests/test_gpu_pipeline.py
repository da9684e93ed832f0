"""Device (HIP) path of the per-month engine and the pipeline vs the fp64 CPU path."""
import os

import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rand(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g, dtype=torch.float64)


@pytest.mark.parametrize("n,b", [(17, 3), (64, 2), (100, 4), (200, 3), (513, 2)])
def test_spd_inverse(gpu, n, b):
    from pfml.ops.linalg import spd_inverse
    X = _rand(b, n + 10, n, seed=n)
    A = X.transpose(1, 2) @ X / n + 0.1 * torch.eye(n, dtype=torch.float64)
    inv = spd_inverse(A.to(gpu)).cpu()
    err = (inv @ A - torch.eye(n, dtype=torch.float64)).abs().max().item()
    assert err < 1e-10, err


def test_spd_inverse_lu_fallback(gpu):
    """An indefinite matrix trips the pivot check and falls back to pivoted LU."""
    from pfml.ops.linalg import spd_inverse
    A = torch.tensor([[0.0, 1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 2.0]], dtype=torch.float64)
    inv = spd_inverse(A.to(gpu)).cpu()
    assert torch.allclose(inv @ A, torch.eye(3, dtype=torch.float64), atol=1e-14)


def test_m_func_gpu_matches_cpu(gpu):
    from pfml.ops.linalg import m_func
    rng = np.random.default_rng(0)
    B, N, K = 3, 80, 10
    X = rng.normal(size=(B, N, K))
    F = np.stack([np.cov(rng.normal(size=(K, 200))) * 2e-2 for _ in range(B)])
    S = np.einsum("bik,bkl,bjl->bij", X, F, X) + np.stack([np.diag(rng.uniform(0.01, 0.03, N) ** 2 * 21) for _ in range(B)])
    lam = 0.2 / rng.uniform(1e7, 1e9, (B, N))
    f64 = dict(dtype=torch.float64)
    args = (torch.tensor(S), torch.tensor(lam), torch.tensor([1e10, 5e9, 2e10], **f64),
            torch.tensor([0.003, 0.001, 0.0], **f64), 0.007, 10.0, 10)
    ref = m_func(*args)
    got = m_func(*[a.to(gpu) if isinstance(a, torch.Tensor) else a for a in args]).cpu()
    assert (got - ref).abs().max().item() / ref.abs().max().item() < 1e-12


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("N", [37, 96])
def test_mf_sym_modes(gpu, mode, N):
    """csrc/s4.hip fused symmetric passes vs their torch oracle (asymmetric inputs, so the
    LDS mirror-tile symmetrisation is exercised)."""
    from pfml.ops.linalg import mf_sym
    B = 3
    X, Y = _rand(B, N, N, seed=1), _rand(B, N, N, seed=2)
    kw = dict(svec=_rand(B, seed=3).abs() + 0.5, cvec=_rand(B, seed=4).abs() + 1.0,
              a=_rand(B, N, seed=5).abs() + 0.1, mask=(torch.rand(B, N) > 0.2).double(), d=1.5)
    ref = mf_sym(mode, X, Y, torch.empty_like(X), **kw)
    kd = {k: (v.to(gpu) if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    got = mf_sym(mode, X.to(gpu), Y.to(gpu), torch.empty_like(X).to(gpu), **kd).cpu()
    assert (got - ref).abs().max().item() / ref.abs().max().item() < 1e-14
    assert torch.equal(got, got.transpose(1, 2))                  # exactly symmetric


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("N", [490, 64])
def test_mf_flat_stream_bitwise(gpu, mode, N):
    """The flat passes' row-stream kernel (exactly symmetric inputs, csrc/s4.hip
    mfunc_flat_kernel) give bitwise the tiled symmetrising kernel's result."""
    from pfml.ops.linalg import mf_sym
    B = 3
    X, Y = _rand(B, N, N, seed=11), _rand(B, N, N, seed=12)
    X, Y = (X + X.transpose(1, 2)).to(gpu), (Y + Y.transpose(1, 2)).to(gpu)
    kw = dict(svec=_rand(B, seed=3).abs() + 0.5, cvec=_rand(B, seed=4).abs() + 1.0,
              a=_rand(B, N, seed=5).abs() + 0.1, mask=(torch.rand(B, N) > 0.2).double(), d=1.5)
    kd = {k: (v.to(gpu) if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    flat = mf_sym(mode, X, Y, torch.empty_like(X), flat=True, **kd)
    tiled = mf_sym(mode, X, Y, torch.empty_like(X), flat=False, **kd)
    assert torch.equal(flat, tiled)


def test_db_sqrt_device_matches_eigh(gpu):
    """Fixed-count, sync-free Denman-Beavers (device mu scaling) vs an eigh square root."""
    from pfml.ops.linalg import DB_ITERS, DB_SCALED_ITERS, _db_sqrt
    B, N = 2, 200
    X = _rand(B, N + 40, N, seed=7)
    S = X.transpose(1, 2) @ X / N
    S = S @ S + 1e-3 * torch.eye(N, dtype=torch.float64)           # cond ~ 1e6
    e, V = torch.linalg.eigh(S)
    ref = V @ torch.diag_embed(e.sqrt()) @ V.transpose(1, 2)
    st = torch.zeros(B, dtype=torch.int32, device=gpu)
    Sd = S.to(gpu)
    ws = [torch.empty_like(Sd) for _ in range(4)]
    got = _db_sqrt(Sd, DB_ITERS, DB_SCALED_ITERS, st, ws).cpu()
    assert int(st.sum()) == 0
    # cond(S) ~ 1e6: eigh's own eigenvector error is ~1e-13 here
    assert (got - ref).abs().max().item() / ref.abs().max().item() < 1e-11


def test_db_newton_schulz_tail(gpu):
    """The Denman-Beavers Newton-Schulz tail (last step with M^-1 = 2I - M): equal to the
    all-exact steps to rounding, and a matrix whose M is still far from I at the tail
    (too few steps) is flagged for the reference-form repair instead of returned."""
    from pfml.ops.linalg import DB_ITERS, DB_SCALED_ITERS, _db_sqrt
    B, N = 3, 160
    X = _rand(B, N + 40, N, seed=17)
    S = X.transpose(1, 2) @ X / N
    S = S @ S + 1e-3 * torch.eye(N, dtype=torch.float64)
    Sd = S.to(gpu)

    def run(iters, tail, scaled=DB_SCALED_ITERS):
        st = torch.zeros(B, dtype=torch.int32, device=gpu)
        ws = [torch.empty_like(Sd) for _ in range(4)]
        return _db_sqrt(Sd, iters, scaled, st, ws, ns_tail=tail).cpu(), st.cpu()

    tail, st = run(DB_ITERS, True)
    exact, st0 = run(DB_ITERS + 1, False)
    assert int(st.sum()) == 0 and int(st0.sum()) == 0
    assert (tail - exact).abs().max().item() / exact.abs().max().item() < 1e-13
    _, st_short = run(3, True, scaled=2)            # tail after two steps: far from I
    assert st_short.tolist() == [1] * B


def test_db_mu_rows_bitwise(gpu, monkeypatch):
    """The Denman-Beavers scaling mu and the Y update's row scales from ONE device kernel
    (csrc/s4.hip db_mu_rows_kernel) give bitwise the square root of the torch form (mu kernel,
    then 0.5 / mu and 0.5 mu broadcast by torch), and the starting copies of S are not needed
    (S is only read)."""
    from pfml.ops import linalg as la
    B, N = 3, 160
    X = _rand(B, N + 40, N, seed=23)
    S = X.transpose(1, 2) @ X / N
    S = (S @ S + 1e-3 * torch.eye(N, dtype=torch.float64)).to(gpu)
    S = 0.5 * (S + S.transpose(1, 2))
    S0 = S.clone()

    def run():
        st = torch.zeros(B, dtype=torch.int32, device=gpu)
        ws = [torch.empty_like(S) for _ in range(4)]
        return la._db_sqrt(S, la.DB_ITERS, la.DB_SCALED_ITERS, st, ws, exact_sym=True).clone()

    fused = run()
    assert torch.equal(S, S0)

    def torch_rows(M, Mi, unscaled, mu, rs, es):
        la._db_mu(M, Mi, unscaled, mu)
        rs.copy_((0.5 / mu).view(B, 1).expand(B, N))
        es.copy_((0.5 * mu).view(B, 1).expand(B, N))

    monkeypatch.setattr(la, "_db_mu_rows", torch_rows)
    assert torch.equal(run(), fused)


@pytest.mark.parametrize("tc", [True, False])
def test_m_tilde_production_shape(gpu, tc):
    """m at N = 496 (padded S&P 500 width) on the device vs the reference-form torch m_func
    (LU inverses, convergence-checked square root), with padded rows."""
    from pfml.ops.linalg import m_func_reference, m_tilde
    rng = np.random.default_rng(1)
    B, N, K, n = 2, 496, 25, 489
    X = rng.normal(size=(B, N, K))
    X[:, n:] = 0.0
    F = np.stack([np.cov(rng.normal(size=(K, 300))) * 21e-4 for _ in range(B)])
    iv = rng.uniform(0.01, 0.03, (B, N)) ** 2 * 21
    iv[:, n:] = 1.0
    S = np.einsum("bik,bkl,bjl->bij", X, F, X) + np.stack([np.diag(v) for v in iv])
    w = np.array([1e10, 3e9])
    lam = 0.2 / rng.uniform(1e7, 1e9, (B, N)) if tc else np.full((B, N), 1e-16)
    lam[:, n:] = 10.0 / w[:, None]
    mask = np.zeros((B, N))
    mask[:, :n] = 1.0
    t = lambda v: torch.tensor(v, dtype=torch.float64)                      # noqa: E731
    args = (t(S), t(lam), t(w), t([0.003, 0.001]), 0.007, 10.0, 10)
    ref = m_func_reference(*args, mask=t(mask))
    mt, a = m_tilde(*[x.to(gpu) if isinstance(x, torch.Tensor) else x for x in args],
                    mask=t(mask).to(gpu))
    got = (mt * a.unsqueeze(-1) / a.unsqueeze(-2)).cpu()
    assert (got - ref).abs().max().item() / ref.abs().max().item() < 1e-12


def test_rff_and_standardize(gpu):
    from pfml.ops.panel import rff_features, standardize_signals
    X = torch.rand(300, 20, dtype=torch.float64)
    W = 0.3 * _rand(20, 16, seed=1)
    F = rff_features(X, W)
    Fd = rff_features(X.to(gpu), W.to(gpu)).cpu()
    assert torch.allclose(Fd, F, rtol=1e-12, atol=1e-13)
    Fz = torch.cat([F, torch.zeros(1, F.shape[1], dtype=torch.float64)])
    idx = torch.randint(0, 300, (2, 13, 40))
    idx[1, :, 35:] = 300                              # padding rows
    mask = torch.ones(2, 40, dtype=torch.float64)
    mask[1, 35:] = 0
    vol = torch.rand(301, dtype=torch.float64) + 0.05
    ref = standardize_signals(Fz, idx, mask, vol)
    got = standardize_signals(Fz.to(gpu), idx.to(gpu), mask.to(gpu), vol.to(gpu)).cpu()
    assert torch.allclose(got, ref, rtol=1e-11, atol=1e-12)
    # strided write into one g block of a padded, g-interleaved stack (S4 layout)
    P = F.shape[1]
    Fw = rff_features(X.to(gpu), W.to(gpu), width=P + 1, pad_rows=1)
    assert torch.equal(Fw[:300, :P].cpu(), Fd) and not Fw[300:].any() and not Fw[:, P:].any()
    # written in place into a column block of a wider table (S4's gathered-addend table)
    tab = torch.full((301, 3 * (P + 1)), 7.0, dtype=torch.float64, device=gpu)
    rff_features(X.to(gpu), W.to(gpu), width=P + 1, pad_rows=1, out=tab[:, P + 1:2 * P + 2])
    assert torch.equal(tab[:, P + 1:2 * P + 2], Fw)
    assert bool((tab[:, :P + 1] == 7.0).all()) and bool((tab[:, 2 * P + 2:] == 7.0).all())
    stack = torch.full((2, 13, 40, 2 * (P + 1)), 7.0, dtype=torch.float64, device=gpu)
    standardize_signals(Fw, idx.to(gpu), mask.to(gpu), vol.to(gpu), P=P,
                        out=stack[..., P + 1:])
    blk = stack[..., P + 1:].cpu()
    assert torch.allclose(blk[..., :P], ref, rtol=1e-11, atol=1e-12)
    assert not blk[..., P:].any() and bool((stack[..., :P + 1] == 7.0).all())
    # column statistics only (the Horner steps' gathered addends), into a g block of a wider
    # [B, TH, 2, G * (P + 1)] buffer
    from pfml.ops.panel import signal_stats
    st_ref = signal_stats(Fz, idx, mask, P, torch.empty(2, 13, 2, P + 1, dtype=torch.float64))
    st = torch.full((2, 13, 2, 2 * (P + 1)), 7.0, dtype=torch.float64, device=gpu)
    signal_stats(Fw, idx.to(gpu), mask.to(gpu), P, st[..., P + 1:])
    assert torch.allclose(st[..., P + 1:].cpu(), st_ref, rtol=1e-12, atol=1e-13)
    assert bool((st[..., :P + 1] == 7.0).all())
    # (F[idx] - mean) * scale / vol reproduces the standardised signals
    Fr = Fz[:, :P][idx]
    rec = (Fr - st_ref[:, :, 0:1, :P]) * st_ref[:, :, 1:2, :P] / vol[idx].unsqueeze(-1)
    assert torch.allclose(rec * mask.view(2, 1, 40, 1), ref, rtol=1e-11, atol=1e-12)


def test_pfml_inputs_gpu_matches_cpu(gpu, small_data):
    from pfml.config import get_features
    from pfml.data import io
    from pfml.models.pfml_inputs import build_inputs
    from pfml.models.risk import BarraCov
    from pfml.utils.dates import pfml_date_grids
    cfg = small_data
    d = cfg.run.data_dir
    chars = io.read_processed_chars(d, get_features())
    barra = BarraCov.load(os.path.join(d, "Barra_Cov.npz"))
    wealth = pd.read_csv(os.path.join(d, "wealth_processed.csv"), parse_dates=["eom"])
    rf = io.read_risk_free(d)
    g = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"], 1971, 10)
    months = g["m2"][:24]
    cpu = build_inputs(cfg, chars, barra, wealth, rf, "cpu", months=months)
    dev = build_inputs(cfg, chars, barra, wealth, rf, gpu, months=months)
    for a, b in [(dev.reals.r_tilde.cpu(), cpu.reals.r_tilde), (dev.reals.denom.cpu(), cpu.reals.denom)]:
        assert (a - b).abs().max().item() / b.abs().max().item() < 1e-11
    for g in range(len(cpu.signal_t)):
        for i in (0, 5, 23):
            assert torch.allclose(dev.signal_t[g][i].cpu(), cpu.signal_t[g][i], rtol=1e-12,
                                  atol=1e-13)


def test_s4_lag_stats_by_difference(gpu, small_data, monkeypatch):
    """Lag 1..10 statistics from per-date union sums minus each month's excluded rows
    (csrc/panel.hip date_sums / excl_stats) vs the direct gathered pass: the same summands to
    rounding, and bitwise the same whether the months run as one plan or as a sub-range (the
    union universes come from the global month grid)."""
    from pfml.config import get_features
    from pfml.data import io
    from pfml.models import pfml_inputs as PI
    from pfml.models.risk import BarraCov
    from pfml.utils.dates import pfml_date_grids
    cfg = small_data
    d = cfg.run.data_dir
    chars = io.read_processed_chars(d, get_features())
    barra = BarraCov.load(os.path.join(d, "Barra_Cov.npz"))
    wealth = pd.read_csv(os.path.join(d, "wealth_processed.csv"), parse_dates=["eom"])
    rf = io.read_risk_free(d)
    g = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"], 1971, 10)
    months = g["m2"][:30]
    monkeypatch.setattr(PI, "DSTAT", True)
    plan = PI.make_s4_plan(cfg, chars, barra, wealth, rf, gpu, months=months, batch=12)
    assert plan.du_rows is not None and int(plan.batches[0].ex_n.max()) > 0
    dif = PI.run_plan(plan, cfg)
    sub = PI.run_plan(PI.make_s4_plan(cfg, chars, barra, wealth, rf, gpu, months=months[10:],
                                      batch=7), cfg)
    assert torch.equal(sub.reals.denom, dif.reals.denom[:, 10:])
    monkeypatch.setattr(PI, "DSTAT", False)
    direct = PI.run_plan(PI.make_s4_plan(cfg, chars, barra, wealth, rf, gpu, months=months,
                                         batch=12), cfg)
    for a, b in [(dif.reals.r_tilde, direct.reals.r_tilde), (dif.reals.denom, direct.reals.denom)]:
        assert ((a - b).abs().max() / b.abs().max()).item() < 1e-12


def test_s4_two_streams_bitwise(gpu, small_data, monkeypatch):
    """S4 month batches on two streams (PFML_S4_STREAMS=2: each batch's latency-bound kernels
    overlap the other's GEMMs) give bitwise the one-stream summands, eager and as a replayed
    HIP graph (the side streams fork from and join the capture stream)."""
    import sys
    from pfml.config import get_features
    from pfml.data import io
    from pfml.models import pfml_inputs as PI
    from pfml.models.risk import BarraCov
    from pfml.utils.dates import pfml_date_grids
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    cfg = small_data
    d = cfg.run.data_dir
    chars = io.read_processed_chars(d, get_features())
    barra = BarraCov.load(os.path.join(d, "Barra_Cov.npz"))
    wealth = pd.read_csv(os.path.join(d, "wealth_processed.csv"), parse_dates=["eom"])
    rf = io.read_risk_free(d)
    g = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"], 1971, 10)
    plan = PI.make_s4_plan(cfg, chars, barra, wealth, rf, gpu, months=g["m2"][:30], batch=12)
    assert len(plan.batches) == 3
    one = PI.finish_inputs(plan, cfg, PI.run_plan(plan, cfg, defer_checks=True))
    monkeypatch.setattr(PI, "S4_STREAMS", 2)
    two = PI.finish_inputs(plan, cfg, PI.run_plan(plan, cfg, defer_checks=True))
    assert torch.equal(two.reals.denom, one.reals.denom)
    assert torch.equal(two.reals.r_tilde, one.reals.r_tilde)
    box = {}

    def step():
        box["out"] = PI.run_plan(plan, cfg, defer_checks=True)

    rep = bench.graphed(step, gpu)
    assert rep is not None
    box["out"].reals.denom.zero_()
    rep()
    torch.cuda.synchronize()
    out = PI.finish_inputs(plan, cfg, box["out"])
    assert torch.equal(out.reals.denom, one.reals.denom)


def test_s4_hip_graph_replay_matches_eager(gpu, small_data):
    """S4 (run_plan with its checks deferred: no host sync) captured as ONE HIP graph replays
    to bitwise the eager run's r_tilde / denom (PFML_Input_Data.py:318-491), and the deferred
    checks (finish_inputs) then run once."""
    import sys
    from pfml.config import get_features
    from pfml.data import io
    from pfml.models.pfml_inputs import finish_inputs, make_s4_plan, run_plan
    from pfml.models.risk import BarraCov
    from pfml.utils.dates import pfml_date_grids
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    cfg = small_data
    d = cfg.run.data_dir
    chars = io.read_processed_chars(d, get_features())
    barra = BarraCov.load(os.path.join(d, "Barra_Cov.npz"))
    wealth = pd.read_csv(os.path.join(d, "wealth_processed.csv"), parse_dates=["eom"])
    rf = io.read_risk_free(d)
    g = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"], 1971, 10)
    plan = make_s4_plan(cfg, chars, barra, wealth, rf, gpu, months=g["m2"][:30], batch=16)
    eager = finish_inputs(plan, cfg, run_plan(plan, cfg, defer_checks=True))
    box = {}

    def step():
        box["out"] = run_plan(plan, cfg, defer_checks=True)

    rep = bench.graphed(step, gpu)
    assert rep is not None
    box["out"].reals.denom.zero_()
    rep()
    torch.cuda.synchronize()
    out = finish_inputs(plan, cfg, box["out"])
    assert torch.equal(out.reals.denom, eager.reals.denom)
    assert torch.equal(out.reals.r_tilde, eager.reals.r_tilde)
    # the deferred repair path: months flagged on the device are re-run as one sub-batch and
    # patched in (here nothing needs repair, so the re-run must give the same bits: a month's
    # summands do not depend on the months batched with it)
    again = run_plan(plan, cfg, defer_checks=True)
    again.pending["mstat"][torch.tensor([3, 17, 29], device=gpu)] = 1
    again.reals.denom[:, 3] = float("nan")
    fixed = finish_inputs(plan, cfg, again)
    assert torch.equal(fixed.reals.denom, eager.reals.denom)
    assert torch.equal(fixed.reals.r_tilde, eager.reals.r_tilde)
    for gg in range(len(eager.signal_t)):
        assert torch.equal(fixed.signal_t[gg][17], eager.signal_t[gg][17])


def test_full_pipeline_gpu(gpu, small_data, tmp_path):
    """S4-S9 on the device against the same stages on the CPU oracle path, from copies of the
    same L0-L3 data: every validation utility (obj, cum_obj) to 1e-8, the ranks (hence the
    chosen hyper-parameters) exactly, then weights / pf / pf_summary to 1e-8."""
    import shutil
    from pfml.data.io import CSV_COLUMNS
    from pfml.pipeline import Pipeline
    stages = ["pfml-input", "pfml-search-coef", "pfml-hp-reals", "pfml-aim", "pfml-hps",
              "pfml-best-hps"]
    out = {}
    for dev in ("cuda", "cpu"):
        d = str(tmp_path / f"data_{dev}")
        shutil.copytree(small_data.run.data_dir, d)
        cfg = small_data.override([f"run.data_dir={d}", f"run.artifact_dir={tmp_path}/art_{dev}",
                                   "pf.dates.start_year=1999", "pf.dates.end_yr=2012",
                                   "pf.dates.split_years=3"])
        Pipeline(cfg, device=dev).run(stages)
        out[dev] = {n: pd.read_csv(os.path.join(d, n)) for n in
                    ("validation.csv", "weights.csv", "pf.csv", "pf_summary.csv")}
    for name, df in out["cuda"].items():
        assert list(df.columns) == CSV_COLUMNS[name]
    g, c = out["cuda"]["validation.csv"], out["cpu"]["validation.csv"]
    key = ["g", "p", "l", "hp_end", "eom"]
    g, c = g.sort_values(key).reset_index(drop=True), c.sort_values(key).reset_index(drop=True)
    assert g[key].equals(c[key])
    for col in ("obj", "cum_obj"):
        a, b = g[col].to_numpy(), c[col].to_numpy()
        assert np.array_equal(np.isnan(a), np.isnan(b)), col
        ok = ~np.isnan(a)
        assert np.allclose(a[ok], b[ok], rtol=1e-8, atol=1e-12 * np.abs(b[ok]).max()), col
    assert np.array_equal(g["rank"].fillna(-1).to_numpy(), c["rank"].fillna(-1).to_numpy())
    for name in ("weights.csv", "pf.csv", "pf_summary.csv"):
        a, b = out["cuda"][name], out["cpu"][name]
        assert a.shape == b.shape, name
        num = [k for k in a.columns if np.issubdtype(a[k].dtype, np.number)]
        assert np.allclose(a[num].to_numpy(float), b[num].to_numpy(float), rtol=1e-8,
                           atol=1e-12, equal_nan=True), name
    s = out["cuda"]["pf_summary.csv"]
    assert np.isfinite(s[["r", "sd", "sr", "obj"]].to_numpy()).all()


def test_grid_step_hip_graph_replay_matches_eager(gpu):
    """bench.py --graph: the grid step captured as a HIP graph (side streams joined through
    event waits) replays to exactly the eager step's utilities and scores."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from pfml.config import Config
    from pfml.parallel import dist as pdist
    pdist.set_env(None)
    cfg = Config.default().override(bench.TINY + ["pf_ml.p_vec=[8,16,64]"])
    reals = bench.synthetic_reals(cfg, gpu, n_months=180, n_stocks=40, seed=3)
    res_e, sc_e = bench.one_step(reals, cfg)
    ref_obj = res_e.obj.clone()
    ref_rank = [s[2].clone() for s in sc_e]
    box = {}

    def step():
        box["res"], box["sc"] = bench.one_step(reals, cfg)

    rep = bench.graphed(step, gpu)
    assert rep is not None
    box["res"].obj.zero_()
    rep()
    torch.cuda.synchronize()
    assert torch.equal(box["res"].obj, ref_obj)
    for s, r in zip(box["sc"], ref_rank):
        assert torch.equal(torch.nan_to_num(s[2], nan=-1.0), torch.nan_to_num(r, nan=-1.0))


@pytest.mark.gpu
def test_rccl_collectives_world1(gpu, monkeypatch):
    """Every collective of parallel/collectives.py through a real RCCL process group, in this
    process: PFML_DIST_FORCE=1 takes the distributed path at world size 1, the one
    configuration RCCL can run on a one-GPU box (tools/rccl_check.py; the driver step
    `tools/gpu_run.sh rccl1` also runs bench.py that way under torch.distributed.run)."""
    import socket
    import sys
    from pfml.parallel import dist as pdist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tools"))
    import rccl_check
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    for k, v in {"PFML_DIST_FORCE": "1", "WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0",
                 "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                 "PFML_CHECK_DEVICE": "cuda"}.items():
        monkeypatch.setenv(k, v)
    pdist.set_env(None)
    try:
        rec = rccl_check.run_checks()
    finally:
        pdist.shutdown()
        pdist.set_env(None)
    assert rec["backend"] == "nccl" and rec["forced"] and rec["all_ok"], rec
