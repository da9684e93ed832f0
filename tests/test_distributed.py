"""Multi-process (gloo, world_size 2-4) runs must reproduce the single-process results: the
hp-year sharded grid search (full and rank-local month windows), bench.py --with-inputs on 2
ranks, the whole pipeline from pfml-input to pfml-best-hps on 2 and 3 ranks (S4 per rank on
its hp-year blocks + validation halo, sharded aims and m_t, recursion chained across ranks),
and the collectives themselves."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _small_reals():
    from pfml.config import Config
    from pfml.models.search import PfmlReals
    from pfml.utils.dates import mi_from_ym
    cfg = Config.default().override(["pf_ml.p_vec=[8,16]", "pf.dates.start_year=2001",
                                     "pf.dates.end_yr=2009"])
    G, P = 2, 17
    months = np.arange(mi_from_ym(1994, 6), mi_from_ym(2009, 11) + 1)
    T = len(months)
    g = torch.Generator().manual_seed(7)
    X = torch.randn(G * T, 30, P, generator=g, dtype=torch.float64)
    D = (X.transpose(1, 2) @ X / 30).view(G, T, P, P)
    r = 0.1 * torch.randn(G, T, P, generator=g, dtype=torch.float64)
    return cfg, PfmlReals(months, r, D)


def _worker(rank, world, port, out_dir, task):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from pfml.parallel import collectives as coll
    from pfml.parallel import dist as pdist
    env = pdist.init("cpu")
    try:
        if task in ("grid", "grid_local"):
            from pfml.models.search import (PfmlReals, gather_beta, grid_search,
                                            local_month_rows)
            cfg, reals = _small_reals()
            if task == "grid_local":
                # each rank holds ONLY its chunks' months + validation halo (S4 sharding)
                rows = local_month_rows(reals.months, cfg.hp_years, world, rank)
                reals = PfmlReals(reals.months[rows], reals.r_tilde[:, rows].clone(),
                                  reals.denom[:, rows].clone(), all_months=reals.months)
            res = grid_search(reals, cfg)
            years, beta = gather_beta(res)
            if rank == 0:
                torch.save({"obj": res.obj, "vm": torch.as_tensor(res.val_months),
                            "vy": torch.as_tensor(res.val_year),
                            "beta": beta, "years": torch.as_tensor(years)},
                           os.path.join(out_dir, "grid.pt"))
        elif task == "halo":
            # S4 of the owned months only, the validation halo by the all-gather: every
            # rank's local summands are BITWISE the rows of the one-process arrays
            from pfml.models.search import (complete_local_reals, local_month_rows,
                                            s4_compute_rows)
            cfg, reals = _small_reals()
            comp = s4_compute_rows(reals.months, cfg.hp_years, world, rank)
            loc = local_month_rows(reals.months, cfg.hp_years, world, rank)
            got = complete_local_reals(reals.r_tilde[:, comp].clone(),
                                       reals.denom[:, comp].clone(), reals.months, cfg.hp_years)
            ok = (np.array_equal(got.months, reals.months[loc])
                  and torch.equal(got.denom, reals.denom[:, loc])
                  and torch.equal(got.r_tilde, reals.r_tilde[:, loc]))
            torch.save({"ok": ok, "n_comp": len(comp), "n_loc": len(loc)},
                       os.path.join(out_dir, f"halo{rank}.pt"))
        elif task == "pipeline":
            from pfml.pipeline import Pipeline
            cfg = _PIPE_CFG[0].override([f"run.data_dir={out_dir}",
                                         f"run.artifact_dir={os.path.join(out_dir, 'art')}"])
            Pipeline(cfg, device="cpu", checkpoint=True).run(_PIPE_STAGES)
        elif task == "coll":
            x = torch.full((rank + 1, 3), float(rank))
            g = coll.all_gather_varlen(x)
            pre = coll.exclusive_prefix_sum(torch.tensor([float(rank + 1)]))
            mx = coll.all_reduce_max(float(rank))
            k = coll.all_gather_known(torch.full((rank, 2), float(rank)), [0, 1, 2])
            torch.save({"g": g, "pre": pre, "mx": mx, "k": k},
                       os.path.join(out_dir, f"coll{rank}.pt"))
    finally:
        pdist.shutdown()


_PIPE_CFG: list = []
_PIPE_STAGES = ["pfml-input", "pfml-search-coef", "pfml-hp-reals", "pfml-aim", "pfml-hps",
                "pfml-best-hps"]


def _run(world, task, tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path), task), nprocs=world,
                       join=True, start_method="fork")


@pytest.mark.parametrize("world,task", [(2, "grid"), (4, "grid"), (2, "grid_local"),
                                        (3, "grid_local")])
def test_grid_search_sharded_matches_single(world, task, tmp_path):
    from pfml.models.search import gather_beta, grid_search
    from pfml.parallel import dist as pdist
    pdist.set_env(None)
    cfg, reals = _small_reals()
    ref = grid_search(reals, cfg)
    _, ref_beta = gather_beta(ref)
    _run(world, task, tmp_path)
    got = torch.load(os.path.join(tmp_path, "grid.pt"), weights_only=True)
    assert np.array_equal(got["vm"].numpy(), ref.val_months)
    assert np.array_equal(got["vy"].numpy(), ref.val_year)
    assert np.array_equal(got["years"].numpy(), np.asarray(cfg.hp_years))
    # canonical chunked window sums: BITWISE the one-process coefficients and utilities
    assert torch.equal(got["obj"], ref.obj)
    assert torch.equal(got["beta"], ref_beta)


def test_local_month_rows_cover_once_plus_halo():
    """Every month is computed by exactly one rank, plus each rank's one-block validation
    halo; the burn-in is spread, so S4 months balance (max / mean <= 1.15 at world 8 on the
    production date grid)."""
    from pfml.config import Config
    from pfml.models.search import local_month_rows, make_plan, s4_month_counts
    from pfml.utils.dates import mi_from_ym
    cfg, reals = _small_reals()
    years = np.asarray(cfg.hp_years)
    plan = make_plan(reals.months, years)
    for world in (2, 3, 5, 8):
        rows = [local_month_rows(reals.months, years, world, r) for r in range(world)]
        allr = np.concatenate(rows)
        assert set(allr.tolist()) == set(range(int(plan.val_stop[-1])))
        extra = len(allr) - len(np.unique(allr))
        assert extra <= 12 * (world - 1)                # halos only
    prod = Config.default()
    m2 = np.arange(mi_from_ym(1963, 1), mi_from_ym(2023, 11) + 1)     # 731 PFML months
    for world in (2, 4, 8):
        cnt = np.asarray(s4_month_counts(m2, np.asarray(prod.hp_years), world))
        assert cnt.sum() == len(m2)
        # water-filled burn-in pieces: the ranks' S4 months within 1 % (W = 8: 92 / 92 / 92 /
        # 91 / 91 / 91 / 91 / 91; W = 2: 367 / 364 - the cut is the C = 8 one of every W)
        assert cnt.max() / cnt.mean() <= 1.01, (world, cnt)


def test_water_fill_levels_the_loads():
    """search._water_fill: non-negative integers summing to ``total`` that level base + s
    (the burn-in months that balance the per-rank S4 load), deterministic."""
    from pfml.models.search import _water_fill
    rng = np.random.default_rng(0)
    for _ in range(200):
        base = rng.integers(0, 60, size=int(rng.integers(1, 10)))
        total = int(rng.integers(0, 400))
        s = _water_fill(total, base)
        assert s.min() >= 0 and int(s.sum()) == total
        lv = base + s
        # every filled slot sits at the top level (within one of the remainder deal)
        if total:
            top = lv[s > 0]
            assert top.max() - top.min() <= 1
            assert lv.min() >= top.min() - 1 or (s == 0).all()
        assert (s == _water_fill(total, base)).all()
    assert list(_water_fill(5, np.array([3, 0, 0]))) == [0, 3, 2]
    assert list(_water_fill(0, np.array([1, 2]))) == [0, 0]


def test_s4_compute_rows_partition_the_months():
    """Every local month is computed by exactly one rank (s4_compute_rows partition the union
    of the local rows), and a rank's halo months are computed by other ranks."""
    from pfml.models.search import local_month_rows, s4_compute_rows
    cfg, reals = _small_reals()
    years = np.asarray(cfg.hp_years)
    for world in (2, 3, 5, 8):
        loc = [local_month_rows(reals.months, years, world, r) for r in range(world)]
        comp = [s4_compute_rows(reals.months, years, world, r) for r in range(world)]
        allc = np.concatenate(comp)
        assert len(allc) == len(np.unique(allc))
        assert set(allc.tolist()) == set(np.concatenate(loc).tolist())
        for r in range(world):
            halo = np.setdiff1d(loc[r], comp[r])
            assert len(halo) <= 12
            others = set(np.concatenate([comp[s] for s in range(world) if s != r]).tolist())
            assert set(halo.tolist()) <= others


@pytest.mark.parametrize("world", [2, 3])
def test_halo_exchange_matches_local_rows(world, tmp_path):
    _run(world, "halo", tmp_path)
    short = 0
    for r in range(world):
        d = torch.load(os.path.join(tmp_path, f"halo{r}.pt"), weights_only=True)
        assert d["ok"], (r, d)
        assert d["n_comp"] <= d["n_loc"]
        short += d["n_comp"] < d["n_loc"]
    assert short >= 1                              # some rank did receive a halo


def test_collectives_gloo(tmp_path):
    _run(3, "coll", tmp_path)
    for r in range(3):
        d = torch.load(os.path.join(tmp_path, f"coll{r}.pt"), weights_only=True)
        assert d["g"].shape == (6, 3)
        assert d["g"][:, 0].tolist() == [0.0, 1.0, 1.0, 2.0, 2.0, 2.0]
        assert d["pre"].item() == sum(range(1, r + 1))
        assert d["mx"] == 2.0
        assert d["k"][:, 0].tolist() == [1.0, 2.0, 2.0]


def test_bench_contract_two_ranks_gloo(tmp_path):
    """bench.py under the driver's exact launcher (torch.distributed.run, 2 ranks, 127.0.0.1):
    one JSON line from rank 0 with the contract keys, timing max-reduced over ranks."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=root)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--tiny", "--device", "cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=str(tmp_path),
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    # stdout: the JSON line (the engine's logs go to stderr; gloo's own connect messages,
    # printed by its C++ layer, are the only other stdout lines)
    assert "[pfml." not in r.stdout
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["value"] > 0 and rec["config"]["outputs_finite"]


def test_bench_gpus_flag_spawns_ranks(tmp_path):
    """``bench.py --gpus 2`` WITHOUT a launcher starts the two ranks itself: the
    record says n_gpus 2 / dp2 / world_size 2, and the gathered utilities are bitwise those of
    the one-rank run."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=root)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    common = [sys.executable, os.path.join(root, "bench.py"), "--steps", "1", "--warmup", "0",
              "--tiny", "--device", "cpu", "--no-inputs"]
    recs = {}
    for n in (1, 2):
        r = subprocess.run([*common, "--gpus", str(n), "--dump", str(tmp_path / f"w{n}.pt")],
                           capture_output=True, text=True, timeout=600, env=env,
                           cwd=str(tmp_path))
        assert r.returncode == 0, r.stderr[-3000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        recs[n] = json.loads(lines[0])
    assert recs[2]["n_gpus"] == 2 and recs[2]["world_size"] == 2
    assert recs[2]["config"]["parallelism"] == "dp2"
    assert recs[1]["n_gpus"] == 1 and recs[1]["config"]["parallelism"] == "dp1"
    a = torch.load(tmp_path / "w1.pt", weights_only=True)
    b = torch.load(tmp_path / "w2.pt", weights_only=True)
    assert torch.equal(a["val_months"], b["val_months"])
    assert torch.equal(a["obj"], b["obj"])                      # bitwise


def test_bench_gpus_mismatch_fails():
    """A launcher whose WORLD_SIZE differs from --gpus is refused (non-zero exit, a message),
    before any work is done."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", PYTHONPATH=root)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1",
                        "--tiny", "--device", "cpu"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, (r.returncode, r.stderr[-2000:])
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_with_inputs_two_ranks_equals_one(tmp_path):
    """bench.py --with-inputs: each rank builds the S4 summands of its own hp-year blocks +
    validation halo only; the gathered utilities equal the single-process run."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=root)
    common = [os.path.join(root, "bench.py"), "--steps", "1", "--warmup", "0", "--tiny",
              "--device", "cpu", "--with-inputs"]
    r1 = subprocess.run([sys.executable, *common, "--dump", str(tmp_path / "w1.pt")],
                        capture_output=True, text=True, timeout=600, env=env)
    assert r1.returncode == 0, r1.stderr[-3000:]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *common,
           "--gpus", "2", "--dump", str(tmp_path / "w2.pt")]
    r2 = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r2.returncode == 0, r2.stderr[-3000:]
    a = torch.load(tmp_path / "w1.pt", weights_only=True)
    b = torch.load(tmp_path / "w2.pt", weights_only=True)
    assert torch.equal(a["val_months"], b["val_months"])
    assert torch.equal(a["obj"], b["obj"])                      # bitwise


def _copy_inputs(src: str, dst: str) -> None:
    import shutil
    os.makedirs(dst, exist_ok=True)
    for n in os.listdir(src):
        p = os.path.join(src, n)
        if os.path.isfile(p):
            shutil.copy(p, os.path.join(dst, n))


@pytest.mark.parametrize("world,start", [(2, 1999), (3, 1999), (8, 1999), (6, 2008)])
def test_pipeline_sharded_matches_single(world, start, small_data, tmp_path):
    """The main pipeline from pfml-input to pfml-best-hps on ``world`` gloo ranks - S4 built
    per rank on its hp-year blocks + validation halo (no denom all-gather), betas sharded,
    aims formed where beta and signals live, m_t sharded and the weight recursion chained
    across ranks - writes the same CSVs as one process.  (6, 2008): five hp years on six
    ranks, so one rank holds no year at all (empty shard: ADVICE r1)."""
    import pandas as pd
    from pfml.parallel import dist as pdist
    from pfml.pipeline import Pipeline
    base = small_data.override([f"pf.dates.start_year={start}", "pf.dates.end_yr=2012",
                                "pf.dates.split_years=3"])
    d1, d2 = str(tmp_path / "w1"), str(tmp_path / "wn")
    _copy_inputs(small_data.run.data_dir, d1)
    _copy_inputs(small_data.run.data_dir, d2)
    pdist.set_env(None)
    cfg1 = base.override([f"run.data_dir={d1}", f"run.artifact_dir={os.path.join(d1, 'art')}"])
    Pipeline(cfg1, device="cpu").run(_PIPE_STAGES)
    pdist.set_env(None)
    _PIPE_CFG[:] = [base]
    _run(world, "pipeline", d2)
    for name in ("validation.csv", "weights.csv", "pf.csv", "pf_summary.csv"):
        a = pd.read_csv(os.path.join(d1, name))
        b = pd.read_csv(os.path.join(d2, name))
        assert list(a.columns) == list(b.columns) and len(a) == len(b), name
        # bitwise: the CSV texts are identical (canonical window-sum order on every world)
        with open(os.path.join(d1, name)) as fa, open(os.path.join(d2, name)) as fb:
            assert fa.read() == fb.read(), name
    # per-rank done markers of the sharded stages
    for st in ("pfml-input", "pfml-search-coef"):
        for r in range(world):
            assert os.path.exists(os.path.join(d2, "art", st, f"_DONE.rank{r}.json"))


@pytest.mark.timeout(600)
def test_pipeline_partial_resume_two_ranks(small_data, tmp_path):
    """Resume of a 2-rank run where ONE rank's pfml-input marker is gone: the rank
    whose shard is up to date still joins the halo all-gather of the rank that recomputes (no
    deadlock) and the resumed run writes the CSVs of the uninterrupted one, bitwise."""
    from pfml.parallel import dist as pdist
    base = small_data.override(["pf.dates.start_year=1999", "pf.dates.end_yr=2012",
                                "pf.dates.split_years=3"])
    d = str(tmp_path / "wn")
    _copy_inputs(small_data.run.data_dir, d)
    pdist.set_env(None)
    _PIPE_CFG[:] = [base]
    _run(2, "pipeline", d)
    first = {}
    for name in ("validation.csv", "weights.csv", "pf.csv", "pf_summary.csv"):
        with open(os.path.join(d, name)) as f:
            first[name] = f.read()
        os.remove(os.path.join(d, name))
    # rank 1's S4 shard is stale; every later stage's marker too (they re-run on the resume)
    os.remove(os.path.join(d, "art", "pfml-input", "_DONE.rank1.json"))
    for st in _PIPE_STAGES[1:]:
        art = os.path.join(d, "art", st)
        for n in (os.listdir(art) if os.path.isdir(art) else []):
            if n.startswith("_DONE"):
                os.remove(os.path.join(art, n))
    _run(2, "pipeline", d)
    for name, txt in first.items():
        with open(os.path.join(d, name)) as f:
            assert f.read() == txt, name


@pytest.mark.parametrize("fault", ["pfml-search-coef", "pfml-best-hps"])
def test_pipeline_fault_injection_two_ranks(fault, small_data, tmp_path):
    """Failure recovery on 2 ranks: a poisoned S5 coefficient cell on EVERY rank is
    repaired locally before the utilities are gathered (no rank raises, none waits in the
    gather), and a poisoned S9 w_start makes every rank rerun the chained recursion on the CPU
    with its collectives staged for the backend.  The 2-rank outputs equal the 1-rank outputs
    of the same fault bitwise, and the clean run's to 1e-10."""
    import pandas as pd
    from pfml.parallel import dist as pdist
    from pfml.pipeline import Pipeline
    dates = ["pf.dates.start_year=1999", "pf.dates.end_yr=2012", "pf.dates.split_years=3"]
    base = small_data.override(dates + [f"run.fault_inject={fault}"])
    clean = small_data.override(dates)
    dirs = {k: str(tmp_path / k) for k in ("clean", "w1", "w2")}
    for d in dirs.values():
        _copy_inputs(small_data.run.data_dir, d)
    for k, c in (("clean", clean), ("w1", base)):
        pdist.set_env(None)
        Pipeline(c.override([f"run.data_dir={dirs[k]}",
                             f"run.artifact_dir={os.path.join(dirs[k], 'art')}"]),
                 device="cpu").run(_PIPE_STAGES)
    pdist.set_env(None)
    _PIPE_CFG[:] = [base]
    _run(2, "pipeline", dirs["w2"])
    for name in ("validation.csv", "weights.csv", "pf.csv", "pf_summary.csv"):
        with open(os.path.join(dirs["w1"], name)) as fa, open(os.path.join(dirs["w2"], name)) as fb:
            assert fa.read() == fb.read(), name
        a = pd.read_csv(os.path.join(dirs["clean"], name))
        b = pd.read_csv(os.path.join(dirs["w2"], name))
        for c in a.columns:
            if a[c].dtype.kind in "fc":
                assert np.allclose(a[c].to_numpy(), b[c].to_numpy(), rtol=1e-10, atol=1e-13,
                                   equal_nan=True), (name, c)


def test_collectives_check_gloo_two_ranks():
    """tools/rccl_check.py (every collective, host-staged reduce, p2p hand-off) under
    torch.distributed.run with 2 gloo ranks on CPU; the GPU suite runs it over RCCL."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    envv = dict(os.environ, PFML_CHECK_DEVICE="cpu")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", "29581", os.path.join(root, "tools", "rccl_check.py")],
                       capture_output=True, text=True, timeout=240, env=envv, cwd=root)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads(lines[-1])
    assert rec["backend"] == "gloo" and rec["world_size"] == 2 and rec["all_ok"], rec
