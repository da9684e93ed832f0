#!/bin/bash
set -o pipefail
TAG=${1:-host}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PFML_HOST_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 2 > $OUT/bench.json 2> $OUT/host.txt
rc=$?; cat $OUT/bench.json; tail -24 $OUT/host.txt; exit $rc
