#!/bin/bash
set -o pipefail
TAG=${1:-quad}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 120 python tools/bench_quad.py > $OUT/quad.json 2> $OUT/quad.err
rc=$?; cat $OUT/quad.json; tail -2 $OUT/quad.err; exit $rc
