#!/bin/bash
set -o pipefail
TAG=${1:-sprof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --s4-stress 12 --stocks 3000 --warmup 0 > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 16 > $OUT/kernels.txt 2>&1; cat $OUT/kernels.txt
exit $rc
