#!/bin/bash
set -o pipefail
TAG=${1:-panel}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ridge or grid or band" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest.log | head; exit $rc; fi
timeout -k 10 120 python tools/time_panel.py 14 > $OUT/time_panel.json 2>&1
rc=$?; cat $OUT/time_panel.json; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_band.py 1,14,106 > $OUT/band.json 2> $OUT/band.err
rc=$?; cat $OUT/band.json; if [ $rc -ne 0 ]; then tail -3 $OUT/band.err; exit $rc; fi
timeout -k 10 300 python tools/bench_shard.py 1,8 > $OUT/shard.json 2> $OUT/shard.err
rc=$?; cat $OUT/shard.json; exit $rc
