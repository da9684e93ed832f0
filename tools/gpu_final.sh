#!/bin/bash
# end-of-session check: full GPU suite, smoke, headline bench, strong-scaling rehearsal
set -o pipefail
TAG=${1:-final}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; grep '^{' $OUT/bench.json | cut -c1-200; if [ $rc -ne 0 ]; then tail -5 $OUT/bench.err; exit $rc; fi
PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py 1,2,4,8 > $OUT/shard.json 2> $OUT/shard.err
rc=$?; cat $OUT/shard.json; exit $rc
