#!/bin/bash
# Strong-scaling rehearsal under band-mode / stream overrides (graph replay).
set -o pipefail
TAG=${1:-shm}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for cfg in "PFML_BAND_MODE=multi" "PFML_BAND_MODE=single PFML_RIDGE_STREAMS=2" "PFML_BAND_MODE=single PFML_RIDGE_STREAMS=1" "PFML_BAND_MODE=multi PFML_RIDGE_STREAMS=2"; do
  env $cfg PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py 2,4,8 > $OUT/shard.json 2> $OUT/shard.err
  rc=$?; echo "$cfg $(cat $OUT/shard.json)"; if [ $rc -ne 0 ]; then tail -3 $OUT/shard.err; exit $rc; fi
done
