#!/bin/bash
set -o pipefail
TAG=${1:-risk}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python bench.py --risk-stress --steps 5 --warmup 1 > $OUT/risk.json 2> $OUT/risk.err
rc=$?; cat $OUT/risk.json; if [ $rc -ne 0 ]; then tail -3 $OUT/risk.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --risk-stress --steps 2 --warmup 1 > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 8 > $OUT/kernels.txt 2>&1; cat $OUT/kernels.txt
exit $rc
