#!/bin/bash
# Multi-process rehearsal of the driver's N-GPU bench on ONE GPU: N ranks share cuda:0 with
# gloo collectives staged through the host (PFML_DIST_BACKEND=gloo; RCCL needs one GPU per
# rank).  The gathered utilities of 2, 4 and 8 ranks must equal the 1-rank run's BITWISE (the
# cooperative band reduction gives the same betas at every workgroups-per-cell choice).
set -o pipefail
TAG=${1:-mproc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python bench.py --no-inputs --steps 3 --warmup 1 --dump $OUT/w1.pt > $OUT/b1.json 2> $OUT/b1.err
rc=$?; cat $OUT/b1.json; if [ $rc -ne 0 ]; then tail -5 $OUT/b1.err; exit $rc; fi
for n in 2 4 8; do
  PFML_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --no-inputs --steps 3 --warmup 1 --dump $OUT/w$n.pt > $OUT/b$n.json 2> $OUT/b$n.err
  rc=$?; cat $OUT/b$n.json; if [ $rc -ne 0 ]; then tail -20 $OUT/b$n.err; exit $rc; fi
  python - <<PY
import torch
a = torch.load("$OUT/w1.pt", weights_only=True); b = torch.load("$OUT/w$n.pt", weights_only=True)
assert torch.equal(a["val_months"], b["val_months"]), "val_months"
d = ((a["obj"] - b["obj"]).abs() / a["obj"].abs().clamp_min(1e-300)).max().item()
print("ranks $n vs 1: max rel diff of utilities", d, "bitwise", torch.equal(a["obj"], b["obj"]))
assert torch.equal(a["obj"], b["obj"]), "utilities differ from the 1-rank run"
PY
  rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
done
