#!/usr/bin/env python3
"""S4 (PFML input construction) wall-clock on the production shape: ~731 PFML months of a
500-stock synthetic universe, 2 distinct g (corrected mode) or compat (--compat), fp64.
Plan (index layout, device copies of the raw arrays) built once; every timed step does all
the arithmetic.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.config import Config  # noqa: E402
from pfml.data.synthetic import engine_inputs  # noqa: E402
from pfml.models.pfml_inputs import make_s4_plan, run_plan  # noqa: E402
from pfml.utils.dates import pfml_date_grids  # noqa: E402
from pfml.utils.log import COUNTERS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stocks", type=int, default=500)
    ap.add_argument("--months", type=int, default=0)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--compat", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = Config.default()
    cfg.run.compat_mode = args.compat
    t0 = time.perf_counter()
    chars, barra, wealth, rf = engine_inputs(n_stocks=args.stocks)
    g = pfml_date_grids(int(barra.months.min()), 11, cfg.settings["split"]["test_end"], 1971, 10)
    months = g["m2"] if not args.months else g["m2"][-args.months:]
    t1 = time.perf_counter()
    plan = make_s4_plan(cfg, chars, barra, wealth, rf, dev, months)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    run_plan(plan, cfg)                     # warmup
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.steps):
        a = time.perf_counter()
        out = run_plan(plan, cfg)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    print(json.dumps({"s4_ms": round(1000 * min(ts), 1), "s4_ms_all": [round(1000 * t, 1) for t in ts],
                      "months": len(months), "stocks": args.stocks, "N_pad": plan.N,
                      "G_distinct": plan.Gc, "batches": len(plan.batches),
                      "data_s": round(t1 - t0, 2), "plan_s": round(t2 - t1, 2),
                      "finite": bool(torch.isfinite(out.reals.denom).all()),
                      "counters": COUNTERS.as_dict()}), flush=True)


if __name__ == "__main__":
    main()
