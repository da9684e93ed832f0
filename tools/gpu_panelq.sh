#!/bin/bash
set -o pipefail
TAG=${1:-panelq}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ridge or band or grid" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest.log | head; exit $rc; fi
timeout -k 10 120 python tools/time_panel.py 14 > $OUT/panel14.json 2>&1; cat $OUT/panel14.json | tail -1
PFML_BAND_MODE=single timeout -k 10 120 python tools/bench_ridge.py --timing > $OUT/timing_single.json 2>&1; cat $OUT/timing_single.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json | cut -c1-220
timeout -k 10 400 python tools/bench_shard.py 1,8 > $OUT/shard.json 2> $OUT/shard.err; cat $OUT/shard.json
exit $rc
