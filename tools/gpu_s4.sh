#!/bin/bash
# GPU tests + headline bench + S4-inclusive bench + rocprof of the S4-inclusive step.
set -o pipefail
TAG=${1:-s4}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -25 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err
if [ $rc -ne 0 ]; then echo "bench rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py --with-inputs --steps 1 --warmup 1 > $OUT/bench_s4.json 2> $OUT/bench_s4.err
rc=$?; cat $OUT/bench_s4.json; tail -3 $OUT/bench_s4.err
if [ $rc -ne 0 ]; then echo "bench_s4 rc=$rc: stopping"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --with-inputs --steps 1 --warmup 0 > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 25 > $OUT/kernels.txt 2>&1
cat $OUT/kernels.txt
exit $rc
