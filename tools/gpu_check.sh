#!/bin/bash
# One GPU round: GPU tests, 1-GPU bench, rocprofv3 kernel stats of the bench.
# usage (on the GPU box, from the repo root): tools/gpu_check.sh [tag] [bench args...]
set -o pipefail
TAG=${1:-run}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err
if [ $rc -ne 0 ]; then echo "bench rc=$rc: stopping"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 5 --warmup 1 "$@" > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 15 > $OUT/kernels.txt 2>&1
cat $OUT/kernels.txt
exit $rc
