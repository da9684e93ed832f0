#!/bin/bash
# GPU kernel tests + headline bench + rocprof kernel stats of the headline bench
set -o pipefail
TAG=${1:-q3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_kernels.log 2>&1
rc=$?; tail -2 $OUT/pytest_kernels.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_kernels.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 5 --warmup 1 > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 8 > $OUT/kernels.txt 2>&1
cat $OUT/kernels.txt
timeout -k 10 120 python tools/bench_quad.py > $OUT/quad.json 2> $OUT/quad.err; cat $OUT/quad.json
exit $rc
