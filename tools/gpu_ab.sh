#!/bin/bash
# A/B: the same timing scripts against the current kernels and abtest/libpfml_hip_prev.so
set -o pipefail
TAG=${1:-ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for v in prev cur prev2 cur2; do
  if [ "${v:0:4}" = "prev" ]; then export PFML_HIP_LIB=$ROOT/abtest/libpfml_hip_prev.so; else unset PFML_HIP_LIB; fi
  timeout -k 10 200 python tools/bench_band.py 14 > $OUT/band_$v.json 2> $OUT/band_$v.err || exit 1
  echo "$v $(cat $OUT/band_$v.json)"
done
timeout -k 10 300 python tools/bench_shard.py 8 5 7 > $OUT/shard_cur.json 2>&1; echo "cur $(tail -1 $OUT/shard_cur.json)"
PFML_HIP_LIB=$ROOT/abtest/libpfml_hip_prev.so timeout -k 10 300 python tools/bench_shard.py 8 5 7 > $OUT/shard_prev.json 2>&1; echo "prev $(tail -1 $OUT/shard_prev.json)"
