"""Multi-process (gloo, world_size 2 and 4) runs must reproduce the single-process results:
hp-year sharded grid search with the cross-rank exclusive prefix of window sums, month
sharded PFML inputs, and the collectives themselves."""
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
        if task == "grid":
            from pfml.models.search import gather_beta, grid_search
            cfg, reals = _small_reals()
            res = grid_search(reals, cfg)
            years, beta = gather_beta(res)
            if rank == 0:
                torch.save({"obj": res.obj, "vm": torch.as_tensor(res.val_months),
                            "vy": torch.as_tensor(res.val_year),
                            "beta": beta, "years": torch.as_tensor(years)},
                           os.path.join(out_dir, "grid.pt"))
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


def _run(world, task, tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path), task), nprocs=world,
                       join=True, start_method="fork")


@pytest.mark.parametrize("world", [2, 4])
def test_grid_search_sharded_matches_single(world, tmp_path):
    from pfml.models.search import gather_beta, grid_search
    from pfml.parallel import dist as pdist
    pdist.set_env(None)
    cfg, reals = _small_reals()
    ref = grid_search(reals, cfg)
    _, ref_beta = gather_beta(ref)
    _run(world, "grid", tmp_path)
    got = torch.load(os.path.join(tmp_path, "grid.pt"), weights_only=True)
    assert np.array_equal(got["vm"].numpy(), ref.val_months)
    assert np.array_equal(got["vy"].numpy(), ref.val_year)
    assert np.array_equal(got["years"].numpy(), np.asarray(cfg.hp_years))
    assert torch.allclose(got["obj"], ref.obj, rtol=1e-10, atol=1e-13)
    assert torch.allclose(got["beta"], ref_beta, rtol=1e-9, atol=1e-12)


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
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["value"] > 0 and rec["config"]["outputs_finite"]
