#!/bin/bash
set -o pipefail
TAG=${1:-s4only}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python bench.py --with-inputs --steps 1 --warmup 1 "$@" > $OUT/bench_s4.json 2> $OUT/bench_s4.err
rc=$?; cat $OUT/bench_s4.json; tail -2 $OUT/bench_s4.err; if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --with-inputs --steps 1 --warmup 0 "$@" > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 14 > $OUT/kernels.txt 2>&1
cat $OUT/kernels.txt
exit $rc
