#!/bin/bash
# quadform tile order: GPU tests of the utilities path, bench, step timeline
set -o pipefail
TAG=${1:-quadord}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "quad or util or grid or golden or ridge" > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-inputs --steps 20 --warmup 3 > $OUT/bench_$i.json 2> $OUT/bench_$i.err
  rc=$?; echo "run $i: $(python -c "import json;d=json.load(open('$OUT/bench_$i.json'));print(d['ms_per_step'], d['config']['outputs_finite'])")"
  if [ $rc -ne 0 ]; then tail -5 $OUT/bench_$i.err; exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof1 -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-inputs > $OUT/prof1.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_timeline.py $(find $OUT/prof1 -name "*.db" | head -1) --last 30 --grep "ridge|quad|wsum|window|rank|prefix" > $OUT/timeline1.txt 2>&1
cat $OUT/timeline1.txt
exit $rc
