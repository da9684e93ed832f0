#!/bin/bash
# ridge/band GPU tests + headline bench + single-mode phase timing (one n = 513 cell)
set -o pipefail
TAG=${1:-q2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_kernels.log 2>&1
rc=$?; tail -2 $OUT/pytest_kernels.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_kernels.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench.err; exit $rc; fi
PFML_BAND_MODE=single timeout -k 10 120 python tools/bench_ridge.py --timing > $OUT/timing_single.json 2>&1
rc=$?; cat $OUT/timing_single.json; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_band.py 1,14,106 > $OUT/band.json 2> $OUT/band.err
rc=$?; cat $OUT/band.json; exit $rc
