#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE GPU: time the grid-search step of every rank of a
W-rank run (its hp-year shard; collectives are no-ops) and report the slowest rank per W.

This is the compute part of `bench.py --gpus W` (the driver runs the real multi-GPU bench);
it shows whether the per-rank work shrinks as 1/W or hits a latency floor.  PFML_SHARD_GRAPH=1
replays each rank's step as a captured HIP graph."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pfml.config import Config  # noqa: E402
from pfml.parallel import dist as pdist  # noqa: E402


def main():
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
