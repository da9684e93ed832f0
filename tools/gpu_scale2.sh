#!/bin/bash
set -o pipefail
TAG=${1:-scale2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PFML_HOST_TIMING=1 timeout -k 10 300 python tools/bench_shard.py 8 2 0 > $OUT/shard8.json 2> $OUT/shard8.err
rc=$?; cat $OUT/shard8.json; grep host $OUT/shard8.err | tail -14; if [ $rc -ne 0 ]; then tail -3 $OUT/shard8.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof8 -o run -- python3 $ROOT/tools/bench_shard.py 8 5 0 > $OUT/prof8.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof8 -name "*.db" | head -1) --top 22 > $OUT/kernels8.txt 2>&1
cat $OUT/kernels8.txt
exit $rc
