#!/bin/bash
# full GPU suite + headline bench + S4-inclusive bench with kernel stats
set -o pipefail
TAG=${1:-s4b}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench.err; exit $rc; fi
timeout -k 10 400 python bench.py --with-inputs --steps 2 --warmup 1 > $OUT/bench_inputs.json 2> $OUT/bench_inputs.err
rc=$?; cat $OUT/bench_inputs.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench_inputs.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --with-inputs --steps 1 --warmup 1 > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 14 > $OUT/kernels.txt 2>&1
cat $OUT/kernels.txt
exit $rc
