#!/bin/bash
set -o pipefail
TAG=${1:-band}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python tools/bench_band.py > $OUT/band.json 2> $OUT/band.err
rc=$?; cat $OUT/band.json; tail -3 $OUT/band.err
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
PFML_BAND_MODE=multi timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof14 -o run -- python3 $ROOT/tools/bench_band.py 14 > $OUT/prof14.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof14 -name "*.db" | head -1) --top 12 > $OUT/kernels14.txt 2>&1
cat $OUT/kernels14.txt
exit $rc
