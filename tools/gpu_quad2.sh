#!/bin/bash
set -o pipefail
TAG=${1:-quad2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 120 python tools/bench_quad.py > $OUT/quad.json 2> $OUT/quad.err
rc=$?; cat $OUT/quad.json; if [ $rc -ne 0 ]; then tail -2 $OUT/quad.err; exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "quadform or grid_search" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; exit $rc
