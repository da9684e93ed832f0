#!/bin/bash
# band-domain LU repair: its GPU tests, the rank-deficient bench, the headline bench
set -o pipefail
TAG=${1:-bandlu}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "repair or ridge or grid" > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-inputs --steps 5 --warmup 1 --rank-deficient 4 > $OUT/bench_rd.json 2> $OUT/bench_rd.err
rc=$?; cat $OUT/bench_rd.json; if [ $rc -ne 0 ]; then tail -5 $OUT/bench_rd.err; exit $rc; fi
timeout -k 10 300 python bench.py --no-inputs --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; exit $rc
