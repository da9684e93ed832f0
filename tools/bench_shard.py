#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE GPU: time the grid-search step of every rank of a
W-rank run (its hp-year shard; collectives are no-ops) and report the slowest rank per W.

This is the compute part of `bench.py --gpus W` (the driver runs the real multi-GPU bench);
it shows whether the per-rank work shrinks as 1/W or hits a latency floor.  PFML_SHARD_GRAPH=1
replays each rank's step as a captured HIP graph.  ``--with-inputs``: each rank's S4 (its own
PFML months) and its S4 + S5 + S6 step instead (the whole-node projection of the full
grid-search wall-clock), both replayed as HIP graphs (PFML_SHARD_GRAPH=0: eager launches).

    python tools/bench_shard.py [1,2,4,8] [steps]
    python tools/bench_shard.py --with-inputs [1,2,4,8] [steps]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pfml.config import Config  # noqa: E402
from pfml.parallel import dist as pdist  # noqa: E402


def _median_ms(fn, reps: int) -> float:
    """Median wall time of ``reps`` synchronised calls (one slow replay - another process on
    the box, a clock dip - must not become a rank's number)."""
    ts = []
    for _ in range(max(1, reps)):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t))
    return float(sorted(ts)[len(ts) // 2])


def with_inputs(worlds, steps: int) -> dict:
    """Per-rank S4 (the PFML months this rank computes: s4_compute_rows, its burn-in pieces
    and hp-year blocks; the validation halo of its last year arrives from the next rank by an
    all-gather, zeros here) and its S4 + S5 + S6 step, every rank of each W in turn on this
    one GPU (PFML_Input_Data.py:318-491 sharded by month blocks; collectives no-ops)."""
    from pfml.data.synthetic import engine_inputs
    from pfml.models.pfml_inputs import make_s4_plan, run_plan
    from pfml.models.search import s4_compute_rows
    from pfml.utils.dates import pfml_date_grids
    dev = torch.device("cuda", 0)
    cfg = Config.default()
    cfg.run.compat_mode = False                  # as bench.py: distinct RFF draw per g
    chars, barra, wealth, rf = engine_inputs(n_stocks=500)
    g = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"],
                        int(cfg.settings["pf"]["dates"]["start_year"]),
                        int(cfg.settings["pf"]["dates"]["split_years"]))
    months = g["m2"]
    graph = os.environ.get("PFML_SHARD_GRAPH", "1") != "0"
    hip_graph = graph
    out = {"months_total": int(len(months))}
    for W in worlds:
        s4, grid, nm = [], [], []
        for r in range(W):
            env = pdist.DistEnv(rank=r, world_size=W, device=dev)
            pdist.set_env(env)
            rows = s4_compute_rows(months, cfg.hp_years, W, r)
            plan = make_s4_plan(cfg, chars, barra, wealth, rf, dev, months[rows])
            eng = (plan, months)
            # both timed forms replay as captured HIP graphs (S4's checks deferred: no host
            # sync inside), as bench.py --with-inputs does; eager launches if capture fails
            f_s4 = lambda: run_plan(plan, cfg, defer_checks=True)          # noqa: E731
            rep = bench.graphed(f_s4, dev) if graph else None
            hip_graph &= rep is not None
            rep = rep or f_s4
            rep()                                                 # warm-up
            t_s4 = _median_ms(rep, steps)
            del rep
            torch.cuda.empty_cache()
            f_all = lambda: bench.one_step(None, cfg, eng)                 # noqa: E731
            rep = bench.graphed(f_all, dev) if graph else None
            hip_graph &= rep is not None
            rep = rep or f_all
            rep()                                                 # warm-up (plans, caches)
            t_all = _median_ms(rep, steps)
            del rep
            bench.LAST_S4.clear()
            s4.append(round(t_s4, 1))
            grid.append(round(t_all - t_s4, 1))
            nm.append(int(len(rows)))
            del plan, eng
            torch.cuda.empty_cache()
            print(f"W={W} rank={r}: {len(rows)} months, S4 {t_s4:.1f} ms, "
                  f"S5+S6 {t_all - t_s4:.1f} ms", file=sys.stderr, flush=True)
        out[f"w{W}_s4_ms"] = s4
        out[f"w{W}_s5s6_ms"] = grid
        out[f"w{W}_months"] = nm
        out[f"w{W}_s4_max_ms"] = max(s4)
        out[f"w{W}_s4_max_over_min"] = round(max(s4) / max(min(s4), 1e-9), 3)
        out[f"w{W}_total_max_ms"] = round(max(a + b for a, b in zip(s4, grid)), 1)
    if "w1_s4_max_ms" in out:
        for W in worlds:
            out[f"w{W}_s4_max_vs_ideal"] = round(out[f"w{W}_s4_max_ms"] * W / out["w1_s4_max_ms"], 3)
    pdist.set_env(None)
    out["hip_graph"] = bool(hip_graph)
    return out


def main():
    if "--with-inputs" in sys.argv:
        args = [a for a in sys.argv[1:] if a != "--with-inputs"]
        worlds = [int(w) for w in (args[0] if args else "1,2,4,8").split(",")]
        steps = int(args[1]) if len(args) > 1 else 2
        print(json.dumps(with_inputs(worlds, steps)))
        return
    worlds = [int(w) for w in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8").split(",")]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    only = [int(r) for r in sys.argv[3].split(",")] if len(sys.argv) > 3 else None
    dev = torch.device("cuda", 0)
    cfg = Config.default()
    reals = bench.synthetic_reals(cfg, dev)
    out = {}
    for W in worlds:
        per_rank = []
        for r in (only if only is not None else range(W)):
            pdist.set_env(pdist.DistEnv(rank=r, world_size=W, device=dev))
            fn = lambda: bench.one_step(reals, cfg)                 # noqa: E731
            if os.environ.get("PFML_SHARD_GRAPH"):                  # per-rank HIP graph replay
                fn = bench.graphed(fn, dev) or fn
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            per_rank.append(1e3 * (time.perf_counter() - t) / steps)
        out[f"w{W}_max_ms"] = round(max(per_rank), 3)
        out[f"w{W}_ranks_ms"] = [round(x, 2) for x in per_rank]
    pdist.set_env(None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
