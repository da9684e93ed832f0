#!/bin/bash
set -o pipefail
TAG=${1:-stress}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python bench.py --with-inputs --steps 1 --warmup 1 > $OUT/bench_s4.json 2> $OUT/bench_s4.err
rc=$?; cat $OUT/bench_s4.json; grep "months per batch" $OUT/bench_s4.err | head -1; if [ $rc -ne 0 ]; then tail -3 $OUT/bench_s4.err; exit $rc; fi
timeout -k 10 900 python -u bench.py --s4-stress 48 --stocks 3000 --warmup 1 > $OUT/stress3000.json 2> $OUT/stress3000.err
rc=$?; cat $OUT/stress3000.json; grep "months per batch" $OUT/stress3000.err | head -2; tail -2 $OUT/stress3000.err; exit $rc
