#!/usr/bin/env python3
"""Headline benchmark: PFML hyper-parameter grid search (BASELINE.json metric).

One *step* is the full grid search of the reference's S5 + S6 stages on the S&P 500
production shapes:

* 2 g x 4 p (64, 128, 256, 512 RFFs) x 101 lambda ridge solves for each of 53 expanding
  hp-year windows = 42,824 "hp x window solves" (PFML_Search_Coef.py:102-137), computed from
  the per-month summands r_tilde_t (513) and denom_t (513 x 513) of ~710 PFML months,
  INCLUDING the expanding window sums (the reference's 0.50 s per (g, year) baseline includes
  its running sums);
* the out-of-sample utilities of every (g, year, p, lambda) on its 12 validation months =
  513,888 quadratic forms (PFML_hp_reals.py:73-102);
* the expanding-mean cum_obj and the dense rank per month (PFML_hp_reals.py:104-125).

Multi-GPU: hp years are sharded over ranks (strong scaling of the fixed reference grid),
window-sum shard totals are exchanged with one all-gather, utilities all-gathered at the
end; the time reported is the max over ranks.

Data: synthetic per-month summands of the production shape (no WRDS/JKP data exists here);
random SPD denom_t = X_t'X_t / N with X_t ~ N(0,1) of shape 500 x 513 (S&P 500 universe).

The same JSON line also carries the FULL grid-search wall-clock including the S4 input
construction (``s4_s5_s6_wall_ms``: every PFML month's Barra Sigma, m_func, (24) Horner
chains and (25) summands for 2 distinct g on a synthetic 500-stock universe, then S5 + S6),
timed the same way (barrier + synchronize on both sides, max over ranks).  Multi-GPU: each
rank builds the S4 summands of the months it owns (``search.s4_compute_rows``: its burn-in
pieces and hp-year blocks) and receives the one-block validation halo of its last year from
the next rank by one all-gather (``search.complete_local_reals``) - every month's S4 runs
once.  ``--no-inputs`` skips it; ``--with-inputs`` makes that full pipeline the timed step
itself.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time


def _rank_launch() -> None:
    """``--gpus N`` is authoritative.  Run without a launcher (no WORLD_SIZE) and N > 1, this
    process starts N ranks itself - ``torch.distributed.run`` as a CHILD process, before any
    GPU call and before the engine is imported - and exits with its code (rank 0 prints the
    one JSON line).  Under a launcher whose WORLD_SIZE differs from N it refuses to run: a
    1-rank measurement can never be reported as an N-GPU point, nor the other way round."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args()[0].gpus
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n:
            sys.stderr.write(f"bench.py: --gpus {n} but the launcher started WORLD_SIZE={ws} "
                             f"ranks; run with matching --gpus (or without a launcher)\n")
            sys.exit(2)
        return
    if n <= 1:
        return
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *sys.argv[1:]]
    sys.exit(subprocess.call(cmd))


if __name__ == "__main__":
    _rank_launch()

import logging  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

# the engine's stage logs go to stderr here: stdout carries the one JSON result line only
if not logging.getLogger("pfml").handlers:
    _h = logging.StreamHandler(sys.stderr)
    _h.setFormatter(logging.Formatter("[%(name)s] %(message)s"))
    logging.getLogger("pfml").addHandler(_h)
    logging.getLogger("pfml").setLevel(os.environ.get("PFML_LOGLEVEL", "INFO"))
    logging.getLogger("pfml").propagate = False

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import pfml  # noqa: E402
from pfml.config import Config  # noqa: E402
from pfml.models.search import (PfmlReals, complete_local_reals, grid_search,  # noqa: E402
                                validation_scores_all)
from pfml.ops.gemm import gemm  # noqa: E402
from pfml.ops.ridge import _HostClock  # noqa: E402
from pfml.parallel import collectives as coll  # noqa: E402
from pfml.parallel import dist as pdist  # noqa: E402
from pfml.utils.dates import mi_from_ym  # noqa: E402

BASELINE_SOLVES_PER_S = 808.0     # reference ridge grid, 8-core Xeon
BASELINE_FULL_S = 3600.0          # ~1-1.5 h grid search incl. S4 (8-core Xeon)
TINY = ["pf_ml.p_vec=[8,16]", "pf.dates.start_year=2008", "pf.dates.end_yr=2020"]
METRIC = "PFML hp×window solves/sec (whole node); full grid-search wall-clock, S&P500"


def synthetic_reals(cfg: Config, device, n_months: int = 710, n_stocks: int = 500,
                    seed: int = 0, collinear: int = 0) -> PfmlReals:
    """``collinear = R > 0``: X_t = Z_t B_g' with a fixed per-g basis B_g (P x R), so EVERY
    expanding window sum has rank <= R: the cells with p + 1 > R are exactly singular at
    lambda = 0 - the reference's np.linalg.solve on collinear RFF summands
    (PFML_Search_Coef.py:131-133, General_functions.py:81) - and go through the device repair."""
    G = len(cfg.g_vec)
    P = cfg.p_max + 1
    last = mi_from_ym(int(cfg.hp_years.max()), 11)
    months = np.arange(last - n_months + 1, last + 1, dtype=np.int64)
    denom = torch.empty((G, n_months, P, P), dtype=torch.float64, device=device)
    r = torch.empty((G, n_months, P), dtype=torch.float64, device=device)
    gen = torch.Generator(device=device)
    chunk = 32
    for g in range(G):
        gen.manual_seed(seed * 1000 + g)
        Bg = None
        if collinear:
            Bg = torch.randn((P, collinear), generator=gen, dtype=torch.float64,
                             device=device) / collinear ** 0.5
        for a in range(0, n_months, chunk):
            b = min(n_months, a + chunk)
            if Bg is None:
                X = torch.randn((b - a, n_stocks, P), generator=gen, dtype=torch.float64,
                                device=device)
            else:
                X = torch.randn((b - a, n_stocks, collinear), generator=gen,
                                dtype=torch.float64, device=device) @ Bg.T
            gemm(X, X, trans_a=True, alpha=1.0 / n_stocks, out=denom[g, a:b], backend="own")
            del X
        r[g] = 0.05 * torch.randn((n_months, P), generator=gen, dtype=torch.float64, device=device)
    return PfmlReals(months=months, r_tilde=r, denom=denom)


LAST_S4: dict = {}


def one_step(reals: PfmlReals, cfg: Config, engine=None):
    if engine is not None:
        # full grid-search wall-clock INCLUDING the S4 input construction of this rank's months;
        # S4's status checks (m_func repairs, singular const) are deferred to finish_s4() after
        # the timed steps: no host sync inside the step, which replays as one HIP graph
        from pfml.models.pfml_inputs import run_plan
        plan, all_months = engine
        s4 = run_plan(plan, cfg, defer_checks=True)
        LAST_S4.update(plan=plan, cfg=cfg, out=s4)
        out = s4.reals
        # this rank computed only the months it owns; the validation halo of its last hp year
        # (the next rank's first block) arrives by one all-gather instead of a second S4
        reals = complete_local_reals(out.r_tilde, out.denom, all_months, cfg.hp_years)
    res = grid_search(reals, cfg)
    th = _HostClock()
    out = validation_scores_all(res.obj, cfg.run.compat_mode)     # every frame, 2 launches
    th("validation_scores")
    return res, out


def finish_s4() -> None:
    """The deferred S4 checks of the last step (one host sync; repairs counted in COUNTERS)."""
    if LAST_S4.get("out") is not None:
        from pfml.models.pfml_inputs import finish_inputs
        finish_inputs(LAST_S4["plan"], LAST_S4["cfg"], LAST_S4["out"])
    LAST_S4.clear()


def engine_setup(cfg: Config, env, n_stocks: int, precision: str = "fp64"):
    """Synthetic post-prep panel + Barra model (engine_inputs) and this rank's S4 plan (index
    layout and device copies only - the arithmetic is all in the timed step)."""
    from pfml.data.synthetic import engine_inputs
    from pfml.models.pfml_inputs import make_s4_plan
    from pfml.models.search import s4_compute_rows
    from pfml.utils.dates import pfml_date_grids
    cfg.run.compat_mode = False          # distinct RFF draw per g: no Q1 duplication
    cfg.run.precision = precision
    chars, barra, wealth, rf = engine_inputs(n_stocks=n_stocks)
    g = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"],
                        int(cfg.settings["pf"]["dates"]["start_year"]),
                        int(cfg.settings["pf"]["dates"]["split_years"]))
    months = g["m2"]
    rows = s4_compute_rows(months, cfg.hp_years, env.world_size, env.rank)
    plan = make_s4_plan(cfg, chars, barra, wealth, rf, env.device, months[rows])
    return (plan, months), (chars, barra, wealth, rf)


def graphed(fn, dev):
    """Capture one step into a HIP graph (torch.cuda.graph -> hipStreamBeginCapture; the side
    streams of the ridge grid join the capture through their event waits).  Returns the replay
    function - every kernel of the step runs on each replay, only the host-side launch work is
    gone - or None when the step cannot be captured."""
    try:
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            fn()                                   # plans, allocator state, code objects
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()                   # the eager run's blocks: the graph has a pool
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        torch.cuda.synchronize(dev)
        return g.replay
    except Exception as e:                         # noqa: BLE001 - fall back to eager launches
        import traceback
        print(f"[bench] graph capture failed, eager launches: {type(e).__name__}: {e}",
              file=sys.stderr)
        traceback.print_exc()
        return None


def segmented(fn, dev):
    """Segment-wise graph capture of a multi-rank step (collectives eager in between);
    None (eager launches) when the capture fails - the same decision on every rank."""
    from pfml.parallel.graphs import SegmentedGraph
    ok, rep, err = 1.0, None, None
    try:
        rep = SegmentedGraph(dev).capture(fn)
    except Exception as e:                         # noqa: BLE001
        ok, err = 0.0, e
    # every rank must take the same path (the replay's collectives pair up across ranks)
    if coll.all_reduce_max(1.0 - ok, device=dev) > 0.0:
        if err is not None:
            print(f"[bench] segmented graph capture failed, eager launches: "
                  f"{type(err).__name__}: {err}", file=sys.stderr)
        return None
    return rep


def timed(fn, steps: int, warmup: int, dev) -> float:
    """ms per step: W untimed steps, then K steps bracketed by barrier + synchronize, max over
    ranks."""
    for _ in range(warmup):
        fn()
    pdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    pdist.barrier()
    dt = coll.all_reduce_max(time.perf_counter() - t0, device=dev)
    return 1000.0 * dt / max(1, steps)


def s4_stress(args) -> None:
    """BASELINE config 4 (3000-stock universe): per-month S4 cost at a large N (Barra Sigma,
    m_func with its 20+ N x N inversions, the (24) Horner chains over [S | I] of width
    2P + N, the LU solves and the (25) products), months batched to fill HBM."""
    from pfml.data.synthetic import engine_inputs
    from pfml.models.pfml_inputs import finish_inputs, make_s4_plan, run_plan
    from pfml.utils.dates import pfml_date_grids
    env = pdist.init(args.device)
    dev = env.device
    cfg = Config.default()
    cfg.run.compat_mode = False
    chars, barra, wealth, rf = engine_inputs(n_stocks=args.stocks)
    g = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"], 1971, 10)
    months = g["m2"][-args.s4_stress:]
    mine = months[np.asarray(list(coll.contiguous_split(len(months), env.world_size, env.rank)))]
    # the plan (index layout, device copies of the panel slices) is set-up, as in the headline
    # bench; the timed region is the S4 arithmetic of every month plus its deferred checks
    t_plan = time.perf_counter()
    plan = make_s4_plan(cfg, chars, barra, wealth, rf, dev, mine)
    t_plan = time.perf_counter() - t_plan
    for _ in range(args.warmup):
        finish_inputs(plan, cfg, run_plan(plan, cfg, defer_checks=True))
    pdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    out = finish_inputs(plan, cfg, run_plan(plan, cfg, defer_checks=True))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    pdist.barrier()
    dt = coll.all_reduce_max(time.perf_counter() - t0, device=dev)
    # all finite <=> min and max finite (both propagate NaN): one reduction pass over the
    # ~3 GB denom stack instead of isfinite's abs / compare / all passes
    mn, mx = torch.aminmax(out.reals.denom)
    finite = bool((torch.isfinite(mn) & torch.isfinite(mx)).item())
    peak = torch.cuda.max_memory_allocated(dev) / 2**30 if dev.type == "cuda" else 0.0
    if env.is_main:
        print(json.dumps({
            "metric": "S4 PFML input construction (m_func, (24), (25)) months/s",
            "value": round(len(months) / dt, 3), "unit": "months/s", "n_gpus": env.world_size,
            "ms_per_month": round(1000 * dt / len(months), 2), "higher_is_better": True,
            "dtype": "fp64" if args.precision == "fp64" else f"fp64 (S4 GEMMs {args.precision})", "data": "synthetic engine inputs (no WRDS/JKP data available)",
            "config": {"n_stocks": args.stocks, "months": len(months), "P": cfg.p_max + 1,
                       "G": len(cfg.g_vec), "peak_hbm_gib": round(peak, 1),
                       "plan_setup_s": round(t_plan, 2), "warmup": args.warmup,
                       "outputs_finite": finite}}), flush=True)
    pdist.shutdown()


def risk_stress(args) -> None:
    """Auxiliary: the Barra risk model's hot kernels (S3) at production
    shapes - daily cross-sectional OLS over 18,783 trading days of ~500 stocks and 25 factors
    (12 FF12 dummies + 13 cluster z-scores), the monthly EWMA factor covariance over a
    2520-day window for 720 month-ends, and the per-stock EWMA idiosyncratic vol - on
    synthetic data of that shape.  Reference: ~182 s for the OLS loop alone."""
    from pfml.ops.risk_kernels import daily_ols, ewma_factor_cov, ewma_vol
    env = pdist.init(args.device)
    dev = env.device
    g = torch.Generator(device="cpu").manual_seed(0)
    days, K, obs = 18783, 25, 2520
    n_d = np.full(days, 500, dtype=np.int64) - (np.arange(days) % 7)      # ragged days
    off = np.concatenate([[0], np.cumsum(n_d)])
    R = int(off[-1])
    X = torch.randn(R, K, generator=g, dtype=torch.float64)
    X[:, :12] = torch.nn.functional.one_hot(torch.randint(0, 12, (R,), generator=g), 12).double()
    y = 0.02 * torch.randn(R, generator=g, dtype=torch.float64)
    X, y, offt = X.to(dev), y.to(dev), torch.as_tensor(off)
    ends = np.arange(obs, days, 21)[:720]
    tr = np.arange(obs, 0, -1, dtype=np.float64)
    w_cor, w_var = (0.5 ** (1 / 378.0)) ** tr, (0.5 ** (1 / 126.0)) ** tr
    stocks = 3000                                       # per-stock residual histories
    gs = np.linspace(0, R, stocks + 1).astype(np.int64)
    lam = 0.5 ** (1 / 126)

    def step():
        coef, resid, _ = daily_ols(X, y, offt)
        F = ewma_factor_cov(coef, ends, obs, w_cor, w_var)
        vol = ewma_vol(resid, gs, lam, 63)
        return coef, F, vol

    for _ in range(max(1, args.warmup)):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t = {}
    for name, fn in (("daily_ols", lambda: daily_ols(X, y, offt)), ("all", step)):
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t[name] = (time.perf_counter() - t0) / args.steps
    coef, F, vol = step()
    if env.is_main:
        print(json.dumps({
            "metric": "Barra risk model kernels (daily OLS + EWMA factor cov + EWMA vol) s/run",
            "value": round(t["all"], 4), "unit": "s", "n_gpus": env.world_size,
            "higher_is_better": False, "daily_ols_s": round(t["daily_ols"], 4),
            "reference_daily_ols_s": 182.0, "dtype": "fp64",
            "data": "synthetic daily panel of production shape (no CRSP data available)",
            "config": {"days": days, "rows": R, "factors": K, "cov_window": obs,
                       "month_ends": len(ends), "stock_histories": stocks,
                       "outputs_finite": bool(torch.isfinite(coef).all() and
                                              torch.isfinite(F).all())}}), flush=True)
    pdist.shutdown()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--months", type=int, default=710)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=True,
                    help="replay the grid step (without S4) as a captured HIP graph - one rank: "
                         "one graph; several ranks: graph segments between the eager "
                         "collectives; falls back to eager launches if the capture fails")
    ap.add_argument("--with-inputs", action="store_true",
                    help="time S4 (PFML input construction for every month) + S5 + S6 as the step")
    ap.add_argument("--rank-deficient", type=int, default=0, metavar="NT",
                    help="synthetic denom_t of rank <= NT per month (X_t: NT x P, so early "
                         "expanding windows are singular at lambda = 0 and exercise the device "
                         "LU repair of the band path); reports the repair count")
    ap.add_argument("--collinear", type=int, default=0, metavar="R",
                    help="synthetic summands whose every expanding window has rank <= R (a "
                         "fixed per-g basis): the cells with p + 1 > R are singular at lambda "
                         "= 0 and are repaired on the device (reported as 'repairs')")
    ap.add_argument("--dump", default="",
                    help="rank 0 saves the gathered utilities of the last step here (tests)")
    ap.add_argument("--no-inputs", action="store_true",
                    help="skip the extra full (S4 + S5 + S6) wall-clock measurement")
    ap.add_argument("--stocks", type=int, default=500)
    ap.add_argument("--precision", default="fp64", choices=["fp64", "fp32", "bf16", "fp8"],
                    help="with --with-inputs: S4 covariance / RFF / risk GEMMs in fp32, or on bf16 / "
                         "fp8 MFMA (experimental; error vs fp64 reported); solves stay fp64")
    ap.add_argument("--tiny", action="store_true",
                    help="CI only: p in {8, 16}, 180 months (exercises the multi-rank path on "
                         "CPU/gloo; not the benchmark config)")
    ap.add_argument("--s4-stress", type=int, default=0, metavar="MONTHS",
                    help="auxiliary: time only the S4 input construction of the last MONTHS "
                         "PFML months for a --stocks universe (e.g. the 3000-stock stress)")
    ap.add_argument("--risk-stress", action="store_true",
                    help="auxiliary: time the Barra risk-model kernels (S3) at production shapes")
    args = ap.parse_args()
    if args.s4_stress:
        return s4_stress(args)
    if args.risk_stress:
        return risk_stress(args)

    env = pdist.init(args.device)
    dev = env.device
    cfg = Config.default()
    if args.tiny:
        cfg = cfg.override(TINY)
        args.months, args.stocks = min(args.months, 180), min(args.stocks, 40)
    n_solves = (len(cfg.g_vec) * len(cfg.hp_years) * len(cfg.p_vec) * len(cfg.l_vec))
    n_util = n_solves * 12

    t_setup = time.perf_counter()
    engine = None
    if args.with_inputs:
        engine, _ = engine_setup(cfg, env, args.stocks, args.precision)
        args.months = len(engine[1])
        reals = None
    else:
        reals = synthetic_reals(cfg, dev, n_months=args.months,
                                n_stocks=args.rank_deficient or args.stocks,
                                collinear=args.collinear)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup

    box = {}

    def step():
        box["res"], box["scores"] = one_step(reals, cfg, engine)

    use_graph = False
    if args.graph and dev.type == "cuda":
        if env.is_dist:
            # one process per GPU: the compute between the collectives replays as graph
            # segments, the collectives run eagerly between them (parallel/graphs.py)
            rep = segmented(step, dev)
        else:
            rep = graphed(step, dev)
        if rep is not None:
            use_graph = True
            ms = timed(rep, args.steps, args.warmup, dev)
    if not use_graph:
        ms = timed(step, args.steps, args.warmup, dev)
    res = box["res"]
    finish_s4()
    value = n_solves / (ms / 1000.0)
    # sanity: finite outputs; device repairs (non-SPD ridge systems) of the last step
    finite = bool(torch.isfinite(res.obj).all().item())
    from pfml.ops.ridge import coop_errors, repairs_done
    from pfml.utils.log import COUNTERS
    repairs = repairs_done() if dev.type == "cuda" else 0
    if dev.type == "cuda":
        # cooperative hand-off timeouts of the last step (NaN betas: a production run's S5
        # guard recomputes those cells, pipeline._guard_grid); counted, never silent
        nto = coop_errors()
        if nto:
            COUNTERS.add("ridge.coop_timeouts", nto)
    if args.dump and env.is_main:
        torch.save({"obj": res.obj.cpu(), "val_months": torch.as_tensor(res.val_months),
                    "val_year": torch.as_tensor(res.val_year)}, args.dump)
    full = None
    if not args.with_inputs and not args.no_inputs:
        # the full grid-search wall-clock INCLUDING S4 (BASELINE.json's second metric)
        del reals
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        cfg_full = Config.default()
        if args.tiny:
            cfg_full = cfg_full.override(TINY)
        t_s = time.perf_counter()
        eng, _ = engine_setup(cfg_full, env, args.stocks, "fp64")
        setup_full = time.perf_counter() - t_s
        from pfml.models.pfml_inputs import finish_inputs, run_plan
        sbox = {}

        def s4_step():
            sbox["out"] = run_plan(eng[0], cfg_full, defer_checks=True)

        # S4 alone and S4 + S5 + S6, each replayed as a HIP graph (segments between the
        # collectives on several ranks) unless --no-graph; one graph alive at a time; each
        # the median of >= 3 individually timed replays (min / max reported too)
        n_rep = 1 if args.tiny else 3
        rep4 = graphed(s4_step, dev) if (args.graph and dev.type == "cuda") else None
        fn4 = rep4 or s4_step
        fn4()
        t_s4 = [timed(fn4, 1, 0, dev) for _ in range(n_rep)]
        finish_inputs(eng[0], cfg_full, sbox["out"])
        del rep4, sbox
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        fbox = {}

        def full_step():
            fbox["res"], _ = one_step(None, cfg_full, eng)

        repf = None
        if args.graph and dev.type == "cuda":
            repf = segmented(full_step, dev) if env.is_dist else graphed(full_step, dev)
        fnf = repf or full_step
        fnf()
        t_full = [timed(fnf, 1, 0, dev) for _ in range(n_rep)]
        ms_full = float(np.median(t_full))
        # repairs / fallbacks of the S4-FED grid (the only grid built from real PFML
        # summands): ridge band-LU repairs of its last step, m_func repairs and singular
        # consts of its S4 (counted by finish_inputs), cooperative timeouts
        c0 = dict(COUNTERS.as_dict())
        s4_rep = repairs_done() if dev.type == "cuda" else 0
        finish_s4()
        if dev.type == "cuda":
            nto = coop_errors()
            if nto:
                COUNTERS.add("ridge.coop_timeouts", nto)
        c1 = COUNTERS.as_dict()
        s4_fb = {k: v - c0.get(k, 0) for k, v in c1.items() if v != c0.get(k, 0)}
        full = {"s4_ms": round(float(np.median(t_s4)), 1),
                "s4_ms_min": round(min(t_s4), 1), "s4_ms_median": round(float(np.median(t_s4)), 1),
                "s4_ms_max": round(max(t_s4), 1),
                "s4_s5_s6_wall_ms": round(ms_full, 1),
                "s4_s5_s6_wall_ms_min": round(min(t_full), 1),
                "s4_s5_s6_wall_ms_max": round(max(t_full), 1),
                "s4_replays": n_rep,
                "s4_repairs": int(s4_rep), "s4_fallbacks": s4_fb,
                "s4_hip_graph": repf is not None,
                "s4_months": int(len(eng[1])), "s4_months_rank": int(len(eng[0].months)),
                "s4_setup_s": round(setup_full, 2),
                "s4_outputs_finite": bool(torch.isfinite(fbox["res"].obj).all().item())}
    prec_err = None
    if args.with_inputs and args.precision != "fp64":
        from pfml.models.pfml_inputs import run_plan
        lo = run_plan(engine[0], cfg).reals
        cfg.run.precision = "fp64"
        hi = run_plan(engine[0], cfg).reals
        rel = lambda a, b: float((a - b).norm() / b.norm())                       # noqa: E731
        prec_err = {"denom_rel_fro": rel(lo.denom, hi.denom),
                    "r_tilde_rel": rel(lo.r_tilde, hi.r_tilde)}
    if env.is_main:
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "solves/s",
            "n_gpus": env.world_size,
            "world_size": (torch.distributed.get_world_size() if env.is_dist else 1),
            "nccl_ranks": (torch.distributed.get_world_size()
                           if env.is_dist and env.backend == "nccl" else 0),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / BASELINE_SOLVES_PER_S, 2),
            "dtype": "fp64" if args.precision == "fp64" else f"fp64 (S4 GEMMs {args.precision})",
            "data": "synthetic (per-month PFML summands of production shape: 710 months, "
                    "P=513, denom_t = X'X/500 with X~N(0,1); no WRDS/JKP data available)",
            "config": {
                "model": "PFML grid search S5+S6: 2 g x 4 p(64..512) x 101 lambda x 53 hp-year "
                         "expanding windows, P=513 (512 RFF + constant), S&P500 universe",
                "global_batch": n_solves,
                "seq_len": args.months,
                "parallelism": f"dp{env.world_size}",
                "dist_backend": env.backend if env.is_dist else "none",
                "utilities_per_step": n_util,
                "device": torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu",
                "setup_s": round(t_setup, 2),
                "outputs_finite": finite,
                "includes_s4_inputs": bool(args.with_inputs),
                "s4_precision_error_vs_fp64": prec_err,
                "ridge_solve_dtype": "fp64 (lambda = 0 / rank-deficient systems: bf16 cannot "
                                     "carry them, SURVEY 7.4)",
                "rank_deficient_nt": args.rank_deficient or None,
                "collinear_rank": args.collinear or None,
                "hip_graph": use_graph,
            },
            "repairs": repairs,
            "fallbacks": COUNTERS.as_dict(),
        }
        if args.rank_deficient:
            rec["data"] = (f"synthetic rank-deficient summands: denom_t = X_t'X_t/NT with X_t "
                           f"~ N(0,1) of shape {args.rank_deficient} x 513 (rank <= "
                           f"{args.rank_deficient} per month), {args.months} months")
        if args.collinear:
            rec["data"] = (f"synthetic collinear summands: X_t = Z_t B_g' with a fixed P x "
                           f"{args.collinear} basis per g (every window rank <= "
                           f"{args.collinear}: cells with p + 1 > {args.collinear} singular at "
                           f"lambda = 0), {args.months} months")
        if full is not None:
            rec.update(full)
            rec["full_vs_baseline"] = round(BASELINE_FULL_S / (full["s4_s5_s6_wall_ms"] / 1000.0), 1)
            rec["config"]["full_pipeline"] = (
                "S4 (Barra Sigma, m_func, (24) Horner chains, (25) summands; 2 distinct g, "
                f"{args.stocks}-stock synthetic universe) + S5 + S6, all PFML months")
        print(json.dumps(rec), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
