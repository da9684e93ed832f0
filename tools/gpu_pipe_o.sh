#!/bin/bash
# pipelined per-g window sums under graph replay: group issue order A/B + timeline
set -o pipefail
TAG=${1:-pipeo}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for o in small_first big_first; do
  for v in 0 1; do
    PFML_PIPE_ORDER=$o PFML_PIPE_SUMS=$v timeout -k 10 300 python bench.py --no-inputs --steps 20 --warmup 3 > $OUT/bench_${o}_p${v}.json 2> $OUT/bench_${o}_p${v}.err
    rc=$?; echo "order=$o pipe=$v: $(python -c "import json;d=json.load(open('$OUT/bench_${o}_p${v}.json'));print(d['ms_per_step'], d['config'].get('hip_graph'))")"
    if [ $rc -ne 0 ]; then tail -5 $OUT/bench_${o}_p${v}.err; exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
PFML_PIPE_SUMS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof1 -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-inputs > $OUT/prof1.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_timeline.py $(find $OUT/prof1 -name "*.db" | head -1) --last 40 --grep "ridge|quad|wsum|segsum|rank|prefix" > $OUT/timeline1.txt 2>&1
cat $OUT/timeline1.txt
exit $rc
