#!/bin/bash
# pipelined per-g window sums, eager launches (no graph) A/B + a timeline of the eager form
set -o pipefail
TAG=${1:-pipee}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for i in 1 2; do
  for v in 0 1; do
    PFML_PIPE_SUMS=$v timeout -k 10 300 python bench.py --no-inputs --no-graph --steps 20 --warmup 3 > $OUT/bench_p${v}_$i.json 2> $OUT/bench_p${v}_$i.err
    rc=$?; echo "eager pipe=$v run $i: $(python -c "import json;d=json.load(open('$OUT/bench_p${v}_$i.json'));print(d['ms_per_step'], d['config'].get('hip_graph'))")"
    if [ $rc -ne 0 ]; then tail -5 $OUT/bench_p${v}_$i.err; exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
PFML_PIPE_SUMS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof1 -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-inputs --no-graph > $OUT/prof1.log 2>&1
rc=$?
cd $ROOT
python tools/rocprof_timeline.py $(find $OUT/prof1 -name "*.db" | head -1) --last 40 --grep "ridge|quad|wsum|segsum|rank|prefix" > $OUT/timeline1.txt 2>&1
cat $OUT/timeline1.txt
exit $rc
