#!/bin/bash
# S4 without library GEMMs: S4 GPU tests, the full bench, kernel names of one S4 run
set -o pipefail
TAG=${1:-s4lib}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "s4 or input or golden or pipeline or smoke" > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
cd $ROOT
grep '^{' $OUT/bench.json | cut -c1-120
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 60 > $OUT/kernels.txt 2>&1
echo "library GEMM kernels (Cijk / hipBLASLt):"; grep -ci "cijk\|hipblaslt\|rocblas" $OUT/kernels.txt || true
exit $rc
