#!/bin/bash
# S4 kernel/pipeline GPU tests, then bench_s4 (3 steps) and a rocprof kernel-stats run of it.
set -o pipefail
TAG=${1:-s4ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pfml or golden or s4 or standard or panel or smoke" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/bench_s4.py --steps 3 > $OUT/bench_s4.json 2> $OUT/bench_s4.err
rc=$?; tail -1 $OUT/bench_s4.json; if [ $rc -ne 0 ]; then tail -3 $OUT/bench_s4.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/tools/bench_s4.py --steps 1 > $OUT/prof.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) --top 16 > $OUT/kernels.txt 2>&1
cat $OUT/kernels.txt
exit $rc
