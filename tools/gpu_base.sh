#!/bin/bash
# Baseline measurements: shard rehearsal (graph replay) at 1/2/4/8 ranks, a kernel timeline
# of one 8-rank shard step and of one full 1-GPU step.
set -o pipefail
TAG=${1:-base}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PFML_SHARD_GRAPH=1 timeout -k 10 300 python tools/bench_shard.py 1,2,4,8 > $OUT/shard.json 2> $OUT/shard.err
rc=$?; cat $OUT/shard.json; if [ $rc -ne 0 ]; then tail -3 $OUT/shard.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof8 -o run -- python3 $ROOT/tools/bench_shard.py 8 3 7 > $OUT/prof8.log 2>&1
rc=$?; if [ $rc -ne 0 ]; then tail -3 $OUT/prof8.log; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof1 -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-inputs > $OUT/prof1.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_timeline.py $(find $OUT/prof8 -name "*.db" | head -1) --last 120 > $OUT/timeline8.txt 2>&1
python tools/rocprof_timeline.py $(find $OUT/prof1 -name "*.db" | head -1) --last 40 > $OUT/timeline1.txt 2>&1
tail -45 $OUT/timeline1.txt
exit $rc
