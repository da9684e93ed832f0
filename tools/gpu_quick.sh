#!/bin/bash
# GPU tests + headline bench + ridge micro-bench (no profiler)
set -o pipefail
TAG=${1:-q}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_ridge.py > $OUT/ridge.txt 2>&1
cat $OUT/ridge.txt | grep -v amdgpu
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 5 --warmup 1 > $OUT/prof.log 2>&1
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 12 > $OUT/kernels.txt 2>&1
cat $OUT/kernels.txt
