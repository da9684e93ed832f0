#!/usr/bin/env python3
"""Exercise every collective of parallel/collectives.py through a real RCCL process group.

Run under ``torch.distributed.run`` (one process per GPU).  With PFML_DIST_FORCE=1 a world of
ONE rank takes the distributed code path too, which is how RCCL itself runs on a one-GPU box
(ranks sharing a GPU need the gloo rehearsal instead).  Checks device tensors, a host tensor
staged through the rank's GPU (the S9 CPU-recompute case), the known-size gather used inside
the captured grid step, the cross-rank exclusive prefix and the barriers; prints one JSON line.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pfml.parallel import collectives as coll  # noqa: E402
from pfml.parallel import dist as pdist  # noqa: E402


def run_checks() -> dict:
    """The checks on the process group of pdist.init (rank 0's record; every rank returns)."""
    want = os.environ.get("PFML_CHECK_DEVICE", "cuda")        # (cpu: gloo dry run of the logic)
    env = pdist.init(want)
    assert env.is_dist and env.backend == ("nccl" if want == "cuda" else "gloo"), env
    W, r, dev = env.world_size, env.rank, env.device
    x = torch.full((3, 5), float(r + 1), dtype=torch.float64, device=dev)
    g = coll.all_gather_cat(x)
    ok = {"all_gather_cat": bool(torch.equal(g, torch.cat(
        [torch.full((3, 5), float(q + 1), dtype=torch.float64, device=dev) for q in range(W)])))}
    counts = [q + 1 for q in range(W)]
    y = torch.full((counts[r], 4), float(r), dtype=torch.float64, device=dev)
    gk = coll.all_gather_known(y, counts)
    ok["all_gather_known"] = bool(gk.shape[0] == sum(counts) and torch.equal(
        gk, torch.cat([torch.full((counts[q], 4), float(q), dtype=torch.float64, device=dev)
                       for q in range(W)])))
    gv = coll.all_gather_varlen(y)
    ok["all_gather_varlen"] = bool(torch.equal(gv, gk))
    tot = torch.full((2, 2), float(r + 1), dtype=torch.float64, device=dev)
    pre = coll.exclusive_prefix_sum(tot)
    ok["exclusive_prefix_sum"] = bool(torch.allclose(pre, torch.full_like(tot, r * (r + 1) / 2)))
    ok["all_reduce_max"] = coll.all_reduce_max(float(r)) == float(W - 1)
    h = torch.full((7,), float(r + 1), dtype=torch.float64)            # host tensor: staged
    coll.all_reduce_sum_(h)
    ok["all_reduce_sum_host_staged"] = bool(torch.all(h == W * (W + 1) / 2))
    ok["broadcast_object"] = coll.broadcast_object({"k": r}, src=0) == {"k": 0}
    z = torch.arange(6, dtype=torch.float64, device=dev) + r
    coll.send_next(z)
    got = coll.recv_prev(z)
    ok["send_recv"] = bool(r == 0 or torch.equal(got, torch.arange(6, dtype=torch.float64,
                                                                   device=dev) + r - 1))
    if dev.type == "cuda":
        # a segment-wise captured step with collectives inside (parallel/graphs.py, the
        # multi-rank bench path): replays equal the eager step, and the process group's
        # watchdog survives the captures (no collective event on a capturing stream)
        from pfml.parallel.graphs import SegmentedGraph
        a = torch.randn(64, 64, dtype=torch.float64, device=dev, generator=torch.Generator(
            device=dev).manual_seed(7))
        res = {}

        def step():
            u = a @ a + float(r)
            v = coll.all_gather_known(u[: counts[r]], counts)
            res["out"] = (v @ a[:, :8]).sum(0) + coll.all_gather_known(u[:1, :3], [1] * W).sum()

        step()
        eager = res["out"].clone()
        rep = SegmentedGraph(dev).capture(step)
        outs = []
        for _ in range(3):
            rep()
            outs.append(res["out"].clone())
        torch.cuda.synchronize()
        ok["segmented_capture"] = all(bool(torch.equal(o, eager)) for o in outs)
    pdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return {"backend": env.backend, "world_size": W, "forced": env.force,
            "rccl": str(torch.cuda.nccl.version()) if dev.type == "cuda" else None,
            "checks": ok, "all_ok": all(ok.values()), "main": env.is_main}


def main():
    rec = run_checks()
    if rec.pop("main"):
        print(json.dumps(rec), flush=True)
    pdist.shutdown()
    return 0 if rec["all_ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
