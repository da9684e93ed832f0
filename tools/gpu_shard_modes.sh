#!/bin/bash
set -o pipefail
TAG=${1:-shardmodes}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for cfg in "auto -" "multi 2" "multi 1"; do
  set -- $cfg
  if [ "$1" = auto ]; then
    timeout -k 10 300 python tools/bench_shard.py 1,2,4,8 3 > $OUT/shard_$1.json 2> $OUT/shard_$1.err
  else
    PFML_BAND_MODE=$1 PFML_RIDGE_STREAMS=$2 timeout -k 10 300 python tools/bench_shard.py 2,4,8 3 > $OUT/shard_$1_$2.json 2> $OUT/shard_$1_$2.err
  fi
  rc=$?; echo "$cfg: $(cat $OUT/shard_$1*.json | tail -1)"; if [ $rc -ne 0 ]; then exit $rc; fi
done
