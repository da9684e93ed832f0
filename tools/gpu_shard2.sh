#!/bin/bash
set -o pipefail
TAG=${1:-shard2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python tools/bench_shard.py 1,2,4,8 > $OUT/shard.json 2> $OUT/shard.err
rc=$?; cat $OUT/shard.json; if [ $rc -ne 0 ]; then tail -3 $OUT/shard.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof8 -o run -- python3 $ROOT/tools/bench_shard.py 8 3 7 > $OUT/prof8.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof8 -name "*.db" | head -1) --top 12 > $OUT/kernels8.txt 2>&1
cat $OUT/kernels8.txt
exit $rc
